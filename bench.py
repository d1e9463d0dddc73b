#!/usr/bin/env python3
"""bench.py -- PacBio bases aligned/s of the MI355X jf_aligner path.

Workload (BASELINE.json configs[1], the largest single-GPU config): E. coli
scale, 50k synthetic PacBio CLR reads (lognormal, mean 12 kb, 13% errors) per
GPU against 200k synthetic super-reads (~250 Mbp), k=17, with the production
flags `-m 17 --psa-min 13 -l ul.txt -k 31 -f -B 15 --max-count 5000
--stretch-cap 10000`.  One step = the whole GPU hot path over
the rank's 50k resident reads: k-mer seeding + hash lookups + 99% threshold ->
per-(read, super-read) grouping -> order-exact LIS + least squares + filters
-> coords records sorted per read, left in HBM.  Index build is outside the
timed region (reported separately).  The rank's batch is spread over
`--streams` aligners (pbgpu.StreamAligner: own HIP stream and host thread
each, one shared index), so one stream's host waits and kernel tails are
filled by the other's work; stage and kernel times are summed over streams.

Multi-GPU: one process per GPU (torchrun); every rank builds its own replica
of the index and aligns its own 50k-read shard (weak scaling, no collective on
the data path).  Timing: barrier + device sync on both sides of exactly
`--steps` steps, max over ranks.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def _dist():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


class Comm:
    """Barrier + max-reduction over ranks.  gloo on the host: the path itself
    has no exchange step (read sharding), so no RCCL traffic is needed."""

    def __init__(self, world):
        self.world = world
        if world > 1:
            import torch.distributed as dist
            dist.init_process_group("gloo")
            self.dist = dist

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def max(self, x):
        if self.world == 1:
            return x
        import torch
        t = torch.tensor([float(x)], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum(self, x):
        if self.world == 1:
            return x
        import torch
        t = torch.tensor([float(x)], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())


# the rocprofv3 kernel each timed slot corresponds to (tools/pmc_summary.py file names)
ROCPROF_FILE = {"k_seed": "k_seed_256_8_0", "k_group": "k_group_false_256u", "k_lis": "k_lis_w_255_8",
                "k_coords": "k_coords_8", "k_rec_sort": "k_rec_sort_256_2048"}


def _kernel_bytes(st):
    """Algorithmic HBM bytes per launch of each individually timed kernel
    (DESIGN.md "Roofline"): every byte the algorithm must move at least once,
    from the kernels' own counters, divided by that kernel's launch count."""
    kn = st["kernel_launches"]
    per = lambda v, k: v / max(1, kn[k])
    return {
        # read bases (1 B), one presence-filter word (8 B) per lookup, one 64-B bucket per probe
        # that passes it, kept k-mer records (16 B) written
        "k_seed": per(st["n_bases"] + st["n_filter"] * 8 + st["n_probes"] * 64 + st["n_kept"] * 16, "k_seed"),
        # first-tier launches only (the timed ones): k-mer records (16 B) + occurrence headers
        # (16 B) read, every occurrence (8 B) read once, every hit (8 B) written, chain
        # descriptors (24 B) written -- counted by the kernel for the reads it completed
        "k_group": per(st["g0_kept"] * 32 + st["g0_hits"] * 16 + st["g0_chains"] * 24, "k_group"),
        # tier-0 k_lis_w (strands <= 255 hits), counted by the kernel: every hit read (8 B)
        # and its lis point written (<= 8 B); per strand its item, chain descriptor (24 B),
        # length and lis length (12 B)
        "k_lis": per(st["l0_hits"] * 16 + st["l0_strands"] * 36, "k_lis"),
        # counted by the kernel: per chain its list entry (4 B), descriptor (24 B), both lis
        # lengths (8 B), super-read length + unitig range (16 B) and read range (16 B); every lis
        # point (8 B) read once; every record (96 B) written (kmers_info pairs not counted)
        "k_coords": per(st["fit_chains"] * 68 + st["fit_points"] * 8 + st["n_records"] * 96, "k_coords"),
        # records read + written
        "k_rec_sort": per(st["n_records"] * 96 * 2, "k_rec_sort"),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="C2", choices=["C1", "C2", "C3"])
    ap.add_argument("--reads", type=int, default=0, help="override reads per GPU")
    ap.add_argument("--cpu-sample-reads", type=int, default=0, help="CPU baseline sample (0 = auto)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-brand", action="store_true", help="skip the B_rand gather microbenchmark")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU-baseline sample duration")
    ap.add_argument("--streams", type=int, default=2,
                    help="aligners (HIP stream + host thread each) the rank's batch is spread over")
    ap.add_argument("--hit-budget", type=float, default=0, help="hits per sub-batch (0 = the library default)")
    args = ap.parse_args()

    rank, world, local = _dist()
    comm = Comm(world)
    from pacbio_amd import pbgpu
    from tools.synth import Dataset, PRESETS

    # more ranks than visible GPUs (a rehearsal of the N>1 launch on a 1-GPU box): ranks share
    ndev = pbgpu.lib().pbgpu_device_count()
    if ndev > 0:
        local %= ndev

    # B_rand: random 64-B sector gathers over a 64 GB buffer, this GPU, this run
    b_rand = pbgpu.measure_gather(local, 64 << 30) if not args.no_brand else None

    k = 21 if args.workload == "C3" else 17
    n_pb = args.reads or PRESETS[args.workload]["n_pb"]
    threads = min(16, os.cpu_count() or 1)
    t0 = time.time()
    ds = Dataset(args.workload, seed=42, threads=threads, n_pb=n_pb, pb_index_base=rank * n_pb)
    t_gen = time.time() - t0
    names, seqs = ds.sr_names(), ds.sr_seqs()
    t0 = time.time()
    index = pbgpu.Index.from_records(names, seqs, k, psa_min=13, device=local)
    t_index = time.time() - t0
    info = index.info()
    al = pbgpu.StreamAligner(index, streams=args.streams, k=k, forward=True, unitigs_k=31,
                             unitig_lengths=ds.unitig_lengths, bases_matching=15.0, max_count=5000,
                             stretch_cap=10000.0)
    if args.hit_budget:
        al.set_hit_budget(int(args.hit_budget))
    blob, off = ds.pb_blob()
    reads = al.upload(blob=blob, offsets=off)
    bases_rank = int(off[-1])

    for _ in range(args.warmup):
        al.align_resident(reads)
    al.reset_stats()
    pbgpu.device_synchronize(local)
    comm.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        al.align_resident(reads)
    pbgpu.device_synchronize(local)
    comm.barrier()
    elapsed = comm.max(time.perf_counter() - t0)
    st = al.stats()

    total_bases = comm.sum(bases_rank) * args.steps
    value = total_bases / elapsed
    stage_ms = {"seed": st["ms_seed"], "group": st["ms_group"], "lis": st["ms_lis"], "fit": st["ms_fit"],
                "records": st["ms_records"]}
    kb = _kernel_bytes(st)
    kms, kn = st["kernel_ms"], st["kernel_launches"]
    dom = max(kb, key=lambda k: kms[k])
    avg_ms = kms[dom] / max(1, kn[dom])
    achieved = kb[dom] / (avg_ms * 1e-3) / 1e9
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", f"pmc_{ROCPROF_FILE[dom]}.json")
    if os.path.exists(pmc_path):
        try:
            with open(pmc_path) as f:
                traffic = json.load(f).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle.oracle import OracleIndex, params
        cthreads = args.cpu_threads or threads
        oix = OracleIndex.from_records(names, seqs, k, threads=cthreads)
        p = params(k=k, forward=True, unitigs_k=31, unitig_lengths=ds.unitig_lengths, bases_matching=15.0,
                   max_count=5000, stretch_cap=10000.0)
        allp = ds.pb_seqs()
        if args.cpu_sample_reads:
            nsamp = min(len(allp), args.cpu_sample_reads)
        else:
            # bounded sample: a pilot sizes it to about --cpu-seconds of oracle work
            pilot = allp[:max(1, min(len(allp), 4 * cthreads))]
            psec, _ = oix.align_timed(p, pilot, threads=cthreads)
            rate = sum(len(x) for x in pilot) / max(psec, 1e-6)
            want = rate * args.cpu_seconds
            nsamp, acc = 0, 0
            while nsamp < len(allp) and acc < want:
                acc += len(allp[nsamp])
                nsamp += 1
            nsamp = max(nsamp, len(pilot))
        pseqs = allp[:nsamp]
        sec, nrec = oix.align_timed(p, pseqs, threads=cthreads)
        sbases = sum(len(x) for x in pseqs)
        cpu = {"value": sbases / sec, "unit": "bases/s", "cores": cthreads, "kind": "port",
               "sample": f"first {nsamp} reads of the rank-0 shard ({sbases} bases, {nrec} records) against the full "
                         f"{args.workload} index; oracle/ C restatement (bit-identical output), {cthreads} threads, "
                         f"{sec:.2f} s"}
        oix.close()

    if rank == 0:
        out = {
            "metric": "PacBio bases aligned/sec (coords out)",
            "value": value,
            "unit": "bases/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (tools/pbsynth.cc, seed 42; SURVEY.md §8d generator)",
            "config": {
                "workload": {"C1": "C1: 100 PB x 10 kb vs 1k SRs, k=17",
                             "C2": "C2 E. coli-scale: 50k PB (lognormal mean 12 kb, CLR 13%) per GPU vs 200k SRs, k=17",
                             "C3": "C3 yeast-scale: PB (mean 12 kb) vs 1M SRs, k=21"}[args.workload],
                "flags": f"-m {k} --psa-min 13 -l ul.txt -k 31 -f -B 15 --max-count 5000 --stretch-cap 10000",
                "reads_per_gpu": len(off) - 1,
                "bases_per_gpu": bases_rank,
                "parallelism": f"read-sharded x{world}, index replicated per GPU",
                "streams_per_gpu": args.streams,
                "index": {"n_sr": info["n_sr"], "text_len": info["text_len"], "n_kmers": info["n_kmers"],
                          "device_bytes": info["device_bytes"], "build_s": round(t_index, 3),
                          "generate_s": round(t_gen, 3)},
                "stage_ms_per_step": {s: round(v / args.steps, 3) for s, v in stage_ms.items()},
                "kernel_ms_per_launch": {k: round(kms[k] / max(1, kn[k]), 3) for k in kms},
                "kernel_launches": dict(kn),
                "counters_per_step": {n: st[n] // args.steps for n in
                                      ("n_kmers", "n_probes", "n_kept", "n_hits", "n_chains", "n_lis_tests",
                                       "n_records")},
                "fit_dtype": "f64",
            },
            "roofline": {"bound": "hbm", "kernel": dom, "rocprof_kernel": ROCPROF_FILE[dom], "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "alg_bytes_per_launch": kb[dom], "avg_launch_ms": avg_ms,
                         # the S aligners' launches of this kernel run concurrently (the rocprofv3 trace
                         # shows the per-step union of the S launches ~= one launch's duration): the
                         # device-level rate is S launches' bytes in one launch's time
                         "concurrent_launches": args.streams,
                         "achieved_concurrent": achieved * args.streams,
                         "frac_concurrent": achieved * args.streams / HBM_PEAK_GBS,
                         "b_rand_gbs": b_rand, "frac_of_b_rand": (achieved / b_rand) if b_rand else None},
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    al.free(reads)
    al.close()
    index.close()


if __name__ == "__main__":
    main()
