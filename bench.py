#!/usr/bin/env python3
"""bench.py -- PacBio bases aligned/s of the MI355X jf_aligner path, coords out.

Workload (BASELINE.json configs[1], the largest single-GPU config): E. coli
scale, 50k synthetic PacBio CLR reads (lognormal, mean 12 kb, 13% errors) per
GPU against 200k synthetic super-reads (~250 Mbp), k=17, with the production
flags `-m 17 --psa-min 13 -l ul.txt -k 31 -f -B 15 --max-count 5000
--stretch-cap 10000`.

`value` is the metric as SURVEY 8(d) defines it: one step = one pass of
pbgpu_run (the jf_aligner CLI's driver) over the rank's PacBio FASTA -- parse,
upload, the whole device path, device-side coords formatting, D2H into
pinned memory, write() of the coords file -- timed from the first batch read
to the closed coords file.  The index is built once before the timed region
(reported as config.index.build_s).

`value_device` keeps round 1's device-only figure: the same reads resident
in HBM, the device path from seeding to per-read sorted records in HBM, no
formatting or output -- run with one aligner (--device-streams 1), so every
kernel launch runs alone and its HIP-event time is the kernel's own.  The
`roofline` object is for the dominant kernel of that leg.

Multi-GPU: one process per GPU (torchrun); every rank builds its own index
replica and aligns its own 50k-read shard into its own coords file (weak
scaling, no collective on the data path).  Timing: barrier + device sync on
both sides of exactly `--steps` steps, max over ranks.
"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def _dist():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawn_ranks(n, argv):
    """`bench.py --gpus N` without a launcher: start N fresh rank processes (one per
    GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their environment) and wait for
    them.  Called before this process touches the GPU, and it never execs: the ranks
    are children.  Rank 0 inherits stdout and prints the one JSON line; the others'
    stdout goes to stderr.  Returns the worst exit code (a failed rank fails the job)."""
    import subprocess
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR=os.environ.get("MASTER_ADDR", "127.0.0.1"), MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env,
                                      stdout=None if r == 0 else sys.stderr.fileno()))
    rc = 0
    for p in procs:
        c = p.wait()
        if c and not rc:
            rc = c
            for q in procs:  # one rank failed: the others would wait at a barrier forever
                if q.poll() is None:
                    q.terminate()
    return rc


def _device_count():
    """GPUs visible, counted in a child process: this one makes no HIP call before its
    create_mega_reads leg (see there)."""
    import subprocess
    code = f"import sys; sys.path.insert(0, {ROOT!r}); from pacbio_amd import pbgpu; print(pbgpu.lib().pbgpu_device_count())"
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True)
    if r.returncode:
        raise RuntimeError(f"counting GPUs failed: {r.stderr[-2000:]}")
    return int(r.stdout.split()[-1])


def _check_world(gpus):
    """`--gpus N` and the launcher's WORLD_SIZE must agree.  Returns True when this
    process is a rank (launched by torchrun, by _spawn_ranks, or N == 1) and False
    when it should spawn the N ranks itself."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is None:
        return gpus <= 1
    if int(ws) != gpus:
        raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={ws}: the launcher and the flag disagree")
    return True


class Comm:
    """Barrier + max/sum over ranks.  gloo on the host: the path itself has no
    exchange step (read sharding), so no RCCL traffic is needed."""

    def __init__(self, world):
        self.world = world
        if world > 1:
            import torch.distributed as dist
            # gloo prints "[Gloo] Rank r is connected to ..." on stdout while it
            # connects: send it to stderr, so stdout holds rank 0's JSON line alone
            sys.stdout.flush()
            saved = os.dup(1)
            os.dup2(2, 1)
            try:
                dist.init_process_group("gloo")
                dist.barrier()
            finally:
                sys.stdout.flush()
                os.dup2(saved, 1)
                os.close(saved)
            self.dist = dist

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def _red(self, x, op):
        if self.world == 1:
            return x
        import torch
        t = torch.tensor([float(x)], dtype=torch.float64)
        self.dist.all_reduce(t, op=op)
        return float(t.item())

    def max(self, x):
        return self._red(x, self.dist.ReduceOp.MAX if self.world > 1 else None)

    def sum(self, x):
        return self._red(x, self.dist.ReduceOp.SUM if self.world > 1 else None)


# the rocprofv3 kernel each timed slot corresponds to (tools/pmc_summary.py file names)
ROCPROF_FILE = {"k_seed": "k_seed_256_8_0", "k_group": "k_group_false_256u", "k_lis": "k_lis_w_255_8",
                "k_coords": "k_coords_8", "k_rec_sort": "k_rec_sort_256_2048"}
STAGE_OF = {"k_seed": "seed", "k_group": "group", "k_lis": "lis", "k_coords": "fit", "k_rec_sort": "records"}


def _kernel_bytes(st):
    """Algorithmic HBM bytes per launch of each individually timed kernel
    (DESIGN.md s.3): every byte the algorithm must move at least once, from the
    kernels' own counters, divided by that kernel's launch count."""
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
        # tier-0 k_lis_w (strands <= 255 hits), counted by the kernel: every hit read (8 B),
        # every lis point written (8 B); per strand its item, chain descriptor (24 B), length and
        # lis length (12 B)
        "k_lis": per(st["l0_hits"] * 8 + st["l0_points"] * 8 + st["l0_strands"] * 36, "k_lis"),
        # per chain its list entry (4 B), descriptor (24 B), both lis lengths (8 B), super-read
        # length + unitig range (16 B) and read range (16 B); every lis point (8 B) read once;
        # every record (96 B) written (kmers_info pairs not counted)
        "k_coords": per(st["fit_chains"] * 68 + st["fit_points"] * 8 + st["n_records"] * 96, "k_coords"),
        # records read + written
        "k_rec_sort": per(st["n_records"] * 96 * 2, "k_rec_sort"),
    }


def _pick_workdir(want, workload, n_pb):
    """The work directory must hold, for every rank of this node, its FASTA files
    (~1.4 B per PacBio base) and two coords files (~6.6 B a base each: the step's and
    the previous one while it is being removed): ~15 B a base with margin.  /tmp on a
    GPU box is ~80 GB, which 8 ranks of C2 come close to (~74 GB), so fall back to
    /dev/shm when `want` is too small."""
    import shutil
    from tools.synth import PRESETS
    local_ranks = int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1")))
    need = 15.0 * n_pb * PRESETS[workload]["pb_len_mean"] * local_ranks + 2e9
    for d in (want, "/dev/shm"):
        try:
            if shutil.disk_usage(d).free >= need:
                return d
        except OSError:
            pass
    print(f"bench: warning: no work directory with {need / 1e9:.0f} GB free; using {want}", file=sys.stderr)
    return want


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_share():
    """This job's CPU share of the box.  On the GPU box os.cpu_count() and the
    affinity mask show the whole 256-thread machine, but a one-GPU job's share is
    16 (OMP_NUM_THREADS / MAX_JOBS are set to it there, and `nproc` honours it)."""
    for var in ("OMP_NUM_THREADS", "MAX_JOBS"):
        v = os.environ.get(var, "")
        if v.isdigit() and int(v) > 0:
            return int(v)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def _calibration(value):
    """SURVEY 8(d)'s calibration of the CPU restatement against the reference on
    identical inputs (tools/calib_ref.py, committed profile): the reference's own
    PSA::search and lis_align::indices, compiled from its sources, against the
    oracle's, one thread each on C2 reads; the reference's whole-path rate is
    estimated from the oracle's with those two components swapped in."""
    path = os.path.join(ROOT, "profiles", "r05_calib_ref.json")
    try:
        with open(path) as f:
            c = json.load(f)
    except (OSError, ValueError):
        return {}
    r = c["path"]["ratio_vs_reference"]
    return {"ratio_vs_reference": r, "reference_estimate_value": value / r,
            "calibration": {"profile": "profiles/r05_calib_ref.json", "cpu_model": c["cpu_model"],
                            "threads": c["threads"], "inputs": c["inputs"],
                            "lookup_reference_over_oracle": c["lookup"]["reference_over_oracle"],
                            "lis_reference_over_oracle": c["lis"]["reference_over_oracle"],
                            "note": "ratio_vs_reference = reference time / oracle time on the same reads (> 1: "
                                    "the oracle is faster); measured in the build container, not on the GPU box"}}


def _cmr_runs(cmr, flags, steps):
    """bin/create_mega_reads `steps` + 1 times (the first untimed): the runs' own --timing
    JSON (with PBGPU_DEBUG_STALL=1: any HIP call that blocked > 0.5 s, kept per run)"""
    import subprocess
    runs = []
    for i in range(steps + 1):
        r = subprocess.run([cmr, *flags], capture_output=True, text=True, env=dict(os.environ, PBGPU_DEBUG_STALL="1"))
        if r.returncode:
            raise RuntimeError(f"create_mega_reads failed: {r.stderr[-2000:]}")
        t = json.loads(r.stderr.strip().splitlines()[-1])
        t["stalls"] = [ln for ln in r.stderr.splitlines() if ln.startswith("pbgpu stall")]
        if i:
            runs.append(t)
    return runs


def strong_split(n_total, world, rank):
    """Rank `rank`'s reads of a strong-scaling run: the contiguous range [lo, hi) of
    the n_total reads, equal counts (+-1), in rank order -- the reference's
    split-and-cat of one read set over its jobs (mega_reads_assemble_cluster2.sh:325-354,
    447: the read file split into batches, one create_mega_reads each, outputs
    concatenated in batch order).  The generator draws read i from its own seed
    (tools/pbsynth.cc: stream_seed(seed, 5, i)), so a rank makes exactly its reads."""
    lo = n_total * rank // world
    hi = n_total * (rank + 1) // world
    return lo, hi


def _chunk_cuts(off, chunk_bases):
    """Read cuts of a resident batch into chunks of at most chunk_bases bases"""
    cuts = [0]
    for r in range(1, len(off)):
        if int(off[r]) - int(off[cuts[-1]]) > chunk_bases and r - 1 > cuts[-1]:
            cuts.append(r - 1)
    cuts.append(len(off) - 1)
    return cuts


def _device_leg(pbgpu, index, akw, blob, off, chunk_bases, steps, comm, local, streams=1):
    """The device path over resident reads (uploaded in chunks of <= chunk_bases before
    the clock): one untimed pass, then `steps` timed passes between barriers and device
    syncs; returns (max-over-ranks seconds, stats of the timed passes, chunk count)"""
    cuts = _chunk_cuts(off, chunk_bases)
    al = pbgpu.StreamAligner(index, streams=streams, **akw)
    chunks = []
    for r0, r1 in zip(cuts[:-1], cuts[1:]):
        if r0 == 0 and r1 == len(off) - 1:
            chunks.append(al.upload(blob=blob, offsets=off))
        else:
            b0, b1 = int(off[r0]), int(off[r1])
            chunks.append(al.upload(blob=bytes(memoryview(blob)[b0:b1]), offsets=off[r0:r1 + 1] - off[r0]))
    for c in chunks:
        al.align_resident(c)
    al.reset_stats()
    pbgpu.device_synchronize(local)
    comm.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        for c in chunks:
            al.align_resident(c)
    pbgpu.device_synchronize(local)
    comm.barrier()
    el = comm.max(time.perf_counter() - t0)
    st = al.stats()
    for c in chunks:
        al.free(c)
    al.close()
    return el, st, len(cuts) - 1


def _per_kernel(st, steps, b_rand=None, b_filt=None, b_table=None, info=None):
    """Every individually timed kernel's algorithmic bytes per launch, mean HIP-event
    launch time and fraction of the HBM peak; k_seed also at its access
    granularity against the mixed roof of gathers measured at the filter's and the
    table's own sizes (b_filt, b_table)"""
    kb = _kernel_bytes(st)
    kms, kn = st["kernel_ms"], st["kernel_launches"]
    per_kernel = {kk: {"alg_bytes_per_launch": kb[kk], "avg_launch_ms": round(kms[kk] / max(1, kn[kk]), 3),
                       "achieved_gbs": round(kb[kk] / (kms[kk] / max(1, kn[kk]) * 1e-3) / 1e9, 1),
                       "frac": round(kb[kk] / (kms[kk] / max(1, kn[kk]) * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                       "stage_ms_per_step": round(st["ms_" + STAGE_OF[kk]] / steps, 3)}
                  for kk in kb if kn.get(kk)}
    if kn.get("k_seed"):
        nl = kn["k_seed"]
        sec = (st["n_bases"] + (st["n_filter"] + st["n_probes"]) * 64 + st["n_kept"] * 16) / nl
        k_ms = kms["k_seed"] / nl
        sgbs = sec / (k_ms * 1e-3) / 1e9
        sv = {"bytes_per_launch": sec, "achieved_gbs": round(sgbs, 1), "frac": round(sgbs / HBM_PEAK_GBS, 4),
              "frac_of_b_rand": round(sgbs / b_rand, 4) if b_rand else None,
              "random_accesses_per_launch": (st["n_filter"] + st["n_probes"]) / nl}
        if b_filt and b_table and info:
            roof_ms = ((st["n_filter"] / nl) * 64 / (b_filt * 1e9) + (st["n_probes"] / nl) * 64 / (b_table * 1e9) +
                       ((st["n_bases"] + st["n_kept"] * 16) / nl) / (HBM_PEAK_GBS * 1e9)) * 1e3
            sv["mixed_roof"] = {"b_filter_gbs": round(b_filt, 1), "filter_bytes": info["filter_bytes"],
                                "b_table_gbs": round(b_table, 1), "table_bytes": info["table_buckets"] * 64,
                                "roof_ms": round(roof_ms, 3), "launch_ms": round(k_ms, 3),
                                "frac": round(roof_ms / k_ms, 4)}
        per_kernel["k_seed"]["sector_view"] = sv
    return per_kernel


def _path_roofline(st, steps, el):
    """SURVEY 8(d)'s whole-path algorithmic bytes of a device leg per step"""
    path_bytes = (0.25 * st["n_bases"] + 64 * st["n_probes"] + 8 * st["n_hits"] + 16 * st["n_hits"] +
                  16 * st["n_lis_tests"] + 96 * st["n_records"]) / steps
    gbs = path_bytes / (el / steps) / 1e9
    return {"bytes_alg_per_step": path_bytes, "achieved": gbs, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
            "formula": "0.25*bases + 64*probes + 8*occurrences + 16*hits + 16*lis_tests + 96*records (SURVEY 8d)"}


PROD_KW = dict(forward=True, unitigs_k=31, bases_matching=15.0, max_count=5000, stretch_cap=10000.0)


def c4_leg(args, comm, rank, world, local, threads, pbgpu, Dataset, brand=True):
    """BASELINE configs[3], the configuration north_star targets: the full C4 index (10M
    super-reads, ~10 Gbp of text over a 250 Mbp genome with 2% 5-50-copy repeats, built on
    the GPU -- in partitions when its sort does not fit -- from the generator's buffers)
    and this GPU's share of the 2M reads of 15 kb N50 (--c4-reads, 250k = 2M / 8; weak:
    every rank its own share, index replicated), production flags, reads resident, one
    aligner.  Unlike C2's 16 MB presence filter, C4's filter and table are far past the
    256 MB Infinity Cache, so k_seed is priced with gathers measured at their sizes."""
    t0 = time.time()
    ds = Dataset("C4", seed=42, threads=min(threads, 16), n_pb=args.c4_reads, pb_index_base=rank * args.c4_reads)
    gen_s = time.time() - t0
    t0 = time.time()
    ix = pbgpu.Index.from_pointers(*ds.sr_pointers(), k=17, device=local)
    pbgpu.device_synchronize(local)
    build_s = time.time() - t0
    info = ix.info()
    print(f"bench c4: index {json.dumps(info)} built in {build_s:.1f} s", file=sys.stderr, flush=True)
    b_filt = b_table = None
    if brand:
        b_filt = pbgpu.measure_gather(local, max(1 << 20, info["filter_bytes"])) if info["filter_bytes"] else None
        b_table = pbgpu.measure_gather(local, max(1 << 20, info["table_buckets"] * 64))
    akw = dict(PROD_KW, k=17, unitig_lengths=ds.unitig_lengths)
    blob, off = ds.pb_blob()
    bases = int(off[-1])
    steps = max(1, args.device_steps)
    # resident calls of at most 0.5 Gbases: beside the ~110 GB index, a 1.5-Gbase call's
    # records and per-hit buffers did not fit the remaining HBM
    el, st, nch = _device_leg(pbgpu, ix, akw, blob, off, min(args.device_chunk_bases, args.c4_chunk_bases), steps,
                              comm, local)
    # size-independent properties of the output (the oracle cannot hold this index): the
    # first reads' records, sorted per read, inside their read and super-read
    al = pbgpu.Aligner(ix, **akw)
    ns = min(200, ds.pb.n)
    rr = al.upload(blob=bytes(memoryview(blob)[:int(off[ns])]), offsets=off[:ns + 1])
    al.align_resident(rr)
    co = al.download()
    rr.close()
    al.close()
    import numpy as np
    r = co.records
    sr_off = np.ctypeslib.as_array(ds.sr.off, shape=(ds.sr.n + 1,))
    sr_len = (sr_off[1:] - sr_off[:-1]).astype(np.int64)
    rl = np.diff(off[:ns + 1].astype(np.int64))
    rid = np.repeat(np.arange(co.n_reads), np.diff(co.read_offsets.astype(np.int64)))
    props = bool(len(r) > 0 and np.all(r["ql"].astype(np.int64) == sr_len[r["sr_index"]]) and
                 np.all((1 <= r["rs"]) & (r["rs"] <= r["re"]) & (r["re"] <= rl[rid])) and
                 np.all((1 <= r["qs"]) & (r["qs"] <= r["qe"]) & (r["qe"].astype(np.int64) <= r["ql"].astype(np.int64))))
    key = r["rs"].astype(np.int64) * (1 << 32) + r["re"].astype(np.int64)
    same = rid[1:] == rid[:-1]
    props &= bool(np.all(key[1:][same] >= key[:-1][same]))
    ix.close()
    ds.close()
    total = comm.sum(bases)
    per_kernel = _per_kernel(st, steps, None, b_filt, b_table, info)
    # k_group's per-launch figure is its first tier's (the timed launch), which on C4 holds a
    # few reads: the group stage is priced whole -- every tier, split and bucket launch --
    # by the algorithmic bytes of all its hits over the stage's time
    g_alg = (st["n_kept"] * 32 + st["n_hits"] * 16 + st["n_chains"] * 24) / steps
    g_ms = st["ms_group"] / steps
    per_kernel["group_stage"] = {"alg_bytes_per_step": g_alg, "stage_ms_per_step": round(g_ms, 3),
                                 "achieved_gbs": round(g_alg / (g_ms * 1e-3) / 1e9, 1),
                                 "frac": round(g_alg / (g_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                 "formula": "kept*32 + hits*16 + chains*24 over the group stage (all launches)"}
    cand = {kk: v for kk, v in per_kernel.items() if kk != "k_group"}
    dom = max(cand, key=lambda kk: cand[kk]["stage_ms_per_step"])
    return {
        "workload": ("C4 chr1-scale (BASELINE configs[3]): full index of 10M super-reads over a 250 Mbp genome with "
                     "2% 5-50-copy repeats, built on this GPU; PacBio reads of 15 kb N50 (lognormal mean 12.5 kb, "
                     f"sigma 0.6), {args.c4_reads} per GPU (2M / 8 at N = 8), production flags, reads resident"),
        "scaling": "weak",
        "bases_per_gpu": bases,
        "value_device": total * steps / el,
        "value_device_note": "reads resident in HBM, device path to sorted records in HBM, one aligner per GPU",
        "ms_per_step": el / steps * 1e3,
        "chunks": nch,
        "stage_ms_per_step": {s: round(st["ms_" + s] / steps, 3) for s in ("seed", "group", "lis", "fit", "records")},
        "counters_per_base": {n: st[n] / max(1, st["n_bases"]) for n in
                              ("n_kmers", "n_filter", "n_probes", "n_kept", "n_hits", "n_chains", "n_lis_tests",
                               "n_records")},
        "kernel_ms_per_launch": {kk: round(st["kernel_ms"][kk] / max(1, st["kernel_launches"][kk]), 3)
                                 for kk in st["kernel_ms"]},
        "kernel_launches": dict(st["kernel_launches"]),
        "group_refines_per_step": st["group_refines"] / steps,
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": per_kernel[dom]["achieved_gbs"],
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": per_kernel[dom]["frac"], "by_kernel": per_kernel},
        "path_roofline": _path_roofline(st, steps, el),
        "index": {"n_sr": info["n_sr"], "text_len": info["text_len"], "n_kmers": info["n_kmers"],
                  "device_bytes": info["device_bytes"], "filter_bytes": info["filter_bytes"],
                  "table_bytes": info["table_buckets"] * 64, "build_s": round(build_s, 3),
                  "generate_s": round(gen_s, 3)},
        "properties_ok": comm.sum(1.0 if props else 0.0) == world,
        "properties": f"first {ns} reads of each rank: records per read in (rs, re) order, inside their read and "
                      "super-read, ql = the super-read's length",
    }


def c3_leg(args, comm, rank, world, local, threads, pbgpu, Dataset):
    """BASELINE configs[2] as a strong-scaling run: the 300k C3 reads (--c3-reads) split over
    the job's ranks (strong_split), the 1M-super-read k=21 index replicated (every rank
    builds its own), production flags, reads resident, one aligner per GPU.  `value_device`
    = all the reads' bases / the max-over-ranks time, so at N ranks it is the whole job's
    rate on a fixed read set."""
    lo, hi = strong_split(args.c3_reads, world, rank)
    t0 = time.time()
    ds = Dataset("C3", seed=42, threads=min(threads, 16), n_pb=max(1, hi - lo), pb_index_base=lo)
    gen_s = time.time() - t0
    t0 = time.time()
    ix = pbgpu.Index.from_pointers(*ds.sr_pointers(), k=21, device=local)
    pbgpu.device_synchronize(local)
    build_s = time.time() - t0
    akw = dict(PROD_KW, k=21, unitig_lengths=ds.unitig_lengths)
    blob, off = ds.pb_blob()
    bases = int(off[-1]) if hi > lo else 0
    steps = max(1, args.device_steps)
    el, st, nch = _device_leg(pbgpu, ix, akw, blob, off, args.device_chunk_bases, steps, comm, local)
    ix.close()
    ds.close()
    total = comm.sum(bases)
    return {
        "workload": ("C3 yeast-scale (BASELINE configs[2]): 1M super-reads, k=21, index replicated per GPU; "
                     f"{args.c3_reads} PacBio reads (mean 12 kb) split over the ranks, production flags, reads resident"),
        "scaling": "strong",
        "reads_total": args.c3_reads,
        "reads_this_rank": [lo, hi],
        "bases_total": total,
        "value_device": total * steps / el,
        "value_device_note": "all ranks' bases / max-over-ranks time; one aligner per GPU, records in HBM",
        "ms_per_step": el / steps * 1e3,
        "chunks_rank0": nch,
        "stage_ms_per_step_rank0": {s: round(st["ms_" + s] / steps, 3) for s in ("seed", "group", "lis", "fit", "records")},
        "index_build_s": round(build_s, 3),
        "generate_s": round(gen_s, 3),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="C2", choices=["C1", "C2", "C3", "C4r"])
    ap.add_argument("--reads", type=int, default=0, help="override reads per GPU")
    ap.add_argument("--cpu-sample-reads", type=int, default=0, help="CPU baseline sample (0 = auto)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-brand", action="store_true", help="skip the B_rand gather microbenchmark")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = this process's CPU share")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU-baseline sample duration")
    ap.add_argument("--streams", type=int, default=2, help="aligners (HIP stream + host thread each) per GPU")
    ap.add_argument("--batch-bases", type=float, default=64e6, help="pbgpu_run batch size in bases")
    ap.add_argument("--device-steps", type=int, default=3, help="steps of the device-only leg (value_device)")
    ap.add_argument("--device-streams", type=int, default=1,
                    help="aligners of the device-only leg: 1 = every launch runs alone, so the per-launch event times "
                         "(the roofline) measure the kernel, not two overlapping launches")
    ap.add_argument("--device-aligners", type=int, default=2,
                    help="the device leg again with this many aligners per GPU, the product's count (their launches "
                         "overlap: value_device_aligners, no per-kernel figure); 0 or 1 = skip")
    ap.add_argument("--device-chunk-bases", type=float, default=1.5e9,
                    help="the device leg aligns its resident reads in chunks of at most this many bases (C2's "
                         "617 Mbases are one; C3's 3.6 Gbases in one call need more than 288 GB of working buffers)")
    ap.add_argument("--parts", type=int, default=2,
                    help="part files of the extra coords-out leg (value_parts; 0 = no such leg)")
    ap.add_argument("--cmr-steps", type=int, default=3,
                    help="runs of bin/create_mega_reads over the same files (value_create_mega_reads; 0 = none)")
    ap.add_argument("--skip-default-leg", action="store_true",
                    help="no default-flags device leg (profiling runs: every large-grid launch is then the "
                         "production leg's)")
    ap.add_argument("--workdir", default=os.environ.get("PBGPU_BENCH_DIR", "/tmp"),
                    help="where the input FASTA and the coords output are written")
    ap.add_argument("--c4r-reads", type=int, default=20000,
                    help="reads of the C4r leg (C4's repeat model and 15-kb-N50 reads; 0 = no such leg): device path, "
                         "create_mega_reads and the CPU oracle on the same reads, reported under c4r")
    ap.add_argument("--c4r-cmr-steps", type=int, default=2, help="timed create_mega_reads runs of the C4r leg")
    ap.add_argument("--c4r-cpu-seconds", type=float, default=8.0, help="target C4r CPU-oracle sample duration")
    ap.add_argument("--c4-reads", type=int, default=250000,
                    help="reads per GPU of the C4 leg (BASELINE configs[3]: the full 10M-super-read index, 15-kb-N50 "
                         "reads; 2M / 8 = 250k; 0 = no such leg), reported under c4")
    ap.add_argument("--c4-chunk-bases", type=float, default=0.5e9,
                    help="the C4 leg's resident calls hold at most this many bases each")
    ap.add_argument("--c3-reads", type=int, default=300000,
                    help="reads of the C3 strong-scaling leg (BASELINE configs[2]: 300k reads split over the ranks, "
                         "index replicated; 0 = no such leg), reported under c3")
    ap.add_argument("--only", choices=["c4", "c3"], default=None,
                    help="run only this leg and print its object (profiling runs)")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU work: the ranks meet at the barrier and rank 0 prints n_gpus (launch rehearsal)")
    args = ap.parse_args()

    if not _check_world(args.gpus):
        sys.exit(_spawn_ranks(args.gpus, sys.argv[1:]))
    rank, world, local = _dist()
    comm = Comm(world)
    if args.dry_run:
        comm.barrier()
        ranks = comm.sum(1.0)
        if rank == 0:
            print(json.dumps({"metric": "PacBio bases aligned/sec (coords out)", "value": None, "n_gpus": world,
                              "ranks_at_barrier": int(ranks), "dry_run": True}), flush=True)
        return
    from pacbio_amd import pbgpu
    from tools.synth import Dataset, PRESETS

    if args.only:
        ndev = _device_count()
        if ndev > 0:
            local %= ndev
        if args.only == "c4":
            leg = c4_leg(args, comm, rank, world, local, _cpu_share(), pbgpu, Dataset, brand=not args.no_brand)
        else:
            leg = c3_leg(args, comm, rank, world, local, _cpu_share(), pbgpu, Dataset)
        if rank == 0:
            print(json.dumps({"only": args.only, "n_gpus": world, args.only: leg}), flush=True)
        return

    # more ranks than visible GPUs (a rehearsal of the N>1 launch on a 1-GPU box): ranks share
    ndev = _device_count()
    if ndev > 0:
        local %= ndev

    b_filt = b_table = None  # random 64-B gathers over buffers the size of the filter and the table
    k = 21 if args.workload == "C3" else 17
    n_pb = args.reads or PRESETS[args.workload]["n_pb"]
    threads = _cpu_share()
    t0 = time.time()
    ds = Dataset(args.workload, seed=42, threads=min(threads, 16), n_pb=n_pb, pb_index_base=rank * n_pb)
    wd = tempfile.mkdtemp(prefix=f"pbgpu_bench_r{rank}_", dir=_pick_workdir(args.workdir, args.workload, n_pb))
    ds.write(wd)
    t_gen = time.time() - t0
    sr_fa, pb_fa, ul_txt = (os.path.join(wd, f) for f in ("sr.fa", "pb.fa", "ul.txt"))
    # ---- create_mega_reads (row f3, the aligner's production caller): the CLI over the
    # same files, overlap graph / tiling on the GPU; its own clock (--timing wall_s: first
    # batch read -> mega-reads file closed; the index build is before it), one warm-up run.
    # First, before this process makes any HIP call: with another process holding a HIP
    # context on the card, a run's hipMalloc now and then blocks for ~4 s
    # (PBGPU_DEBUG_STALL reports); the CLI runs alone in production.
    el_cmr, cmr_t, worst_cmr, cmr_runs = None, None, None, None
    if args.cmr_steps > 0:
        import json as _json
        import subprocess
        cmr = os.path.join(ROOT, "pacbio_amd", "bin", "create_mega_reads")
        cflags = ["-s", "1M", "-m", str(k), "--psa-min", "13", "-k", "31", "-l", ul_txt, "-B", "15", "--max-count",
                  "5000", "--stretch-cap", "10000", "-t", str(threads), "-r", sr_fa, "-p", pb_fa, "--timing",
                  "--devices", str(local), "-o", os.path.join(wd, "mega_reads")]
        walls, cmr_runs = [], []
        for i in range(args.cmr_steps + 1):
            # PBGPU_DEBUG_STALL=1: the library names any HIP call that blocked > 0.5 s (kept per run)
            r = subprocess.run([cmr, *cflags], capture_output=True, text=True,
                               env=dict(os.environ, PBGPU_DEBUG_STALL="1"))
            if r.returncode:
                raise RuntimeError(f"create_mega_reads failed: {r.stderr[-2000:]}")
            cmr_t = _json.loads(r.stderr.strip().splitlines()[-1])
            cmr_t["stalls"] = [ln for ln in r.stderr.splitlines() if ln.startswith("pbgpu stall")]
            if i:
                walls.append(cmr_t["wall_s"])
                cmr_runs.append(cmr_t)
        # the median run, the worst beside it (every run's wall is listed too)
        el_cmr = comm.max(sorted(walls)[len(walls) // 2])
        worst_cmr = comm.max(max(walls))
    # ---- the C4r leg's inputs and its create_mega_reads runs (before any HIP call here too):
    # C4's repeat model (2% of the genome in 5-50-copy repeats) and read lengths (15 kb N50)
    # on a 16 Mbp genome, the shape of BASELINE's chr1 / whole-human configs at a size one
    # GPU and the CPU oracle both run (such reads ran >10x slower per base)
    c4 = None
    if args.c4r_reads > 0:
        c4 = {"n_pb": args.c4r_reads}
        t0 = time.time()
        ds4 = Dataset("C4r", seed=42, threads=min(threads, 16), n_pb=args.c4r_reads,
                      pb_index_base=rank * args.c4r_reads)
        c4["wd"] = tempfile.mkdtemp(prefix=f"pbgpu_bench_c4r_r{rank}_", dir=wd)
        ds4.write(c4["wd"])
        c4["gen_s"] = time.time() - t0
        c4["ds"] = ds4
        sr4, pb4, ul4 = (os.path.join(c4["wd"], f) for f in ("sr.fa", "pb.fa", "ul.txt"))
        if args.c4r_cmr_steps > 0:
            cmr = os.path.join(ROOT, "pacbio_amd", "bin", "create_mega_reads")
            c4["cmr_runs"] = _cmr_runs(cmr, ["-s", "1M", "-m", "17", "--psa-min", "13", "-k", "31", "-l", ul4, "-B",
                                             "15", "--max-count", "5000", "--stretch-cap", "10000", "-t",
                                             str(threads), "-r", sr4, "-p", pb4, "--timing", "--devices",
                                             str(local), "-o", os.path.join(c4["wd"], "mega_reads")],
                                       args.c4r_cmr_steps)
            walls4 = [t["wall_s"] for t in c4["cmr_runs"]]
            c4["cmr_wall"] = comm.max(sorted(walls4)[len(walls4) // 2])
            c4["cmr_worst"] = comm.max(max(walls4))
    # B_rand: random 64-B sector gathers over a 64 GB buffer, this GPU, this run
    b_rand = pbgpu.measure_gather(local, 64 << 30) if not args.no_brand else None
    # the same for random 512-B runs of 8-B words: the shape of k_group's occurrence-list reads
    b_run = pbgpu.measure_gather(local, 64 << 30, unit_bytes=512) if not args.no_brand else None

    t0 = time.time()
    index = pbgpu.Index.from_fasta([sr_fa], k, psa_min=13, device=local)
    t_index = time.time() - t0
    info = index.info()
    if not args.no_brand:
        b_filt = pbgpu.measure_gather(local, max(1 << 20, info["filter_bytes"])) if info["filter_bytes"] else None
        b_table = pbgpu.measure_gather(local, max(1 << 20, info["table_buckets"] * 64))
    akw = dict(k=k, forward=True, unitigs_k=31, unitig_lengths=ds.unitig_lengths, bases_matching=15.0,
               max_count=5000, stretch_cap=10000.0)
    blob, off = ds.pb_blob()
    bases_rank = int(off[-1])

    # ---- device-only leg (value_device): reads resident in HBM, records left in HBM
    # (in chunks of at most --device-chunk-bases: every chunk resident before the clock)
    cuts = [0]
    for r in range(1, len(off)):
        if int(off[r]) - int(off[cuts[-1]]) > args.device_chunk_bases and r - 1 > cuts[-1]:
            cuts.append(r - 1)
    cuts.append(len(off) - 1)

    def upload_chunks(a):
        out = []
        for r0, r1 in zip(cuts[:-1], cuts[1:]):
            if r0 == 0 and r1 == len(off) - 1:
                out.append(a.upload(blob=blob, offsets=off))
            else:
                b0, b1 = int(off[r0]), int(off[r1])
                out.append(a.upload(blob=bytes(blob[b0:b1]), offsets=off[r0:r1 + 1] - off[r0]))
        return out

    al = pbgpu.StreamAligner(index, streams=args.device_streams, **akw)
    chunks = upload_chunks(al)
    for c in chunks:
        al.align_resident(c)
    al.reset_stats()
    pbgpu.device_synchronize(local)
    comm.barrier()
    td = time.perf_counter()
    for _ in range(args.device_steps):
        for c in chunks:
            al.align_resident(c)
    pbgpu.device_synchronize(local)
    comm.barrier()
    el_dev = comm.max(time.perf_counter() - td)
    st = al.stats()
    for c in chunks:
        al.free(c)
    al.close()

    # the same leg with the product's aligners per GPU (pbgpu_run / the CLIs run 2): the reads
    # split between them, their launches overlapping -- throughput only
    el_dev_al = None
    if args.device_aligners > 1 and args.device_streams == 1:
        ala = pbgpu.StreamAligner(index, streams=args.device_aligners, **akw)
        chunks = upload_chunks(ala)
        for c in chunks:
            ala.align_resident(c)
        pbgpu.device_synchronize(local)
        comm.barrier()
        td = time.perf_counter()
        for _ in range(args.device_steps):
            for c in chunks:
                ala.align_resident(c)
        pbgpu.device_synchronize(local)
        comm.barrier()
        el_dev_al = comm.max(time.perf_counter() - td)
        for c in chunks:
            ala.free(c)
        ala.close()

    # SURVEY 8(d)'s second flag set: the defaults, without -l / -f (device leg only)
    el_dev2, st2 = None, None
    if not args.skip_default_leg:
        al2 = pbgpu.StreamAligner(index, streams=args.device_streams, k=k)
        chunks = upload_chunks(al2)
        for c in chunks:
            al2.align_resident(c)
        pbgpu.device_synchronize(local)
        comm.barrier()
        td = time.perf_counter()
        for _ in range(args.device_steps):
            for c in chunks:
                al2.align_resident(c)
        pbgpu.device_synchronize(local)
        comm.barrier()
        el_dev2 = comm.max(time.perf_counter() - td)
        st2 = al2.stats()
        for c in chunks:
            al2.free(c)
        al2.close()

    # ---- the C4r leg on the device: its reads resident, production flags, one aligner
    if c4 is not None:
        ds4 = c4["ds"]
        ix4 = pbgpu.Index.from_fasta([os.path.join(c4["wd"], "sr.fa")], 17, psa_min=13, device=local)
        akw4 = dict(akw, k=17, unitig_lengths=ds4.unitig_lengths)
        al4 = pbgpu.StreamAligner(ix4, streams=1, **akw4)
        blob4, off4 = ds4.pb_blob()
        c4["bases"] = int(off4[-1])
        rr4 = al4.upload(blob=blob4, offsets=off4)
        al4.align_resident(rr4)
        al4.reset_stats()
        pbgpu.device_synchronize(local)
        comm.barrier()
        td = time.perf_counter()
        for _ in range(args.device_steps):
            al4.align_resident(rr4)
        pbgpu.device_synchronize(local)
        comm.barrier()
        c4["el_dev"] = comm.max(time.perf_counter() - td)
        c4["st"] = al4.stats()
        al4.free(rr4)
        al4.close()
        c4["ix"] = ix4

    # ---- end to end (value): PacBio FASTA -> coords file, pbgpu_run
    # (a pbgpu_runner keeps its aligners and pinned buffers across steps: a service
    # aligning file after file; the CLI's single run pays their setup once).  Every
    # step writes a new coords file, as the CLI does; the previous step's file is
    # removed by a background thread while the next step runs (unlinking 4 GB of
    # page cache is not part of the path, and truncating it in place would be).
    import threading
    runner = pbgpu.Runner([index], aligners_per_device=args.streams, batch_bases=int(args.batch_bases), **akw)
    outs = [os.path.join(wd, f"out{i}.coords") for i in range(args.warmup + args.steps)]
    cleaners = []

    def _step(i):
        if i > 0:  # the previous step's file goes while this one is written
            th = threading.Thread(target=os.unlink, args=(outs[i - 1],))
            th.start()
            cleaners.append(th)
        return runner.run([pb_fa], outs[i])
    for i in range(args.warmup):
        _step(i)
    for th in cleaners:
        th.join()
    pbgpu.device_synchronize(local)
    comm.barrier()
    t0 = time.perf_counter()
    rstats = []
    for i in range(args.warmup, args.warmup + args.steps):
        rstats.append(_step(i))
    pbgpu.device_synchronize(local)
    comm.barrier()
    elapsed = comm.max(time.perf_counter() - t0)
    for th in cleaners:
        th.join()
    coords_bytes = rstats[-1]["coords_bytes"]
    runner.close()

    # ---- the same coords out into P part files (pbgpu_run_params.n_parts, the reference's
    # split-and-cat in one process): P readers / writers, 2 aligners each; the parts
    # concatenated are the one file above.  Reported beside `value`, never as it.
    el_parts, pstats = None, None
    if args.parts > 1:
        prunner = pbgpu.Runner([index], aligners_per_device=2 * args.parts, batch_bases=int(args.batch_bases),
                               n_parts=args.parts, **akw)
        pouts = [os.path.join(wd, f"parts{i}.coords") for i in range(args.steps + 1)]
        pclean = []

        def _rm_parts(path):
            for j in range(args.parts):
                try:
                    os.unlink(f"{path}.{j}")
                except OSError:
                    pass

        def _pstep(i):
            if i > 0:
                th = threading.Thread(target=_rm_parts, args=(pouts[i - 1],))
                th.start()
                pclean.append(th)
            return prunner.run([pb_fa], pouts[i])
        _pstep(0)
        for th in pclean:
            th.join()
        pbgpu.device_synchronize(local)
        comm.barrier()
        t0 = time.perf_counter()
        pstats = [_pstep(i) for i in range(1, args.steps + 1)]
        pbgpu.device_synchronize(local)
        comm.barrier()
        el_parts = comm.max(time.perf_counter() - t0)
        for th in pclean:
            th.join()
        _rm_parts(pouts[-1])
        prunner.close()

    value_cmr = comm.sum(bases_rank) / el_cmr if el_cmr else None

    total_bases = comm.sum(bases_rank) * args.steps
    value = total_bases / elapsed
    value_device = comm.sum(bases_rank) * args.device_steps / el_dev
    value_device_al = comm.sum(bases_rank) * args.device_steps / el_dev_al if el_dev_al else None
    # every collective runs on every rank, here, never inside the rank-0 report below
    value_device2 = comm.sum(bases_rank) * args.device_steps / el_dev2 if el_dev2 else None
    value_parts = comm.sum(bases_rank) * args.steps / el_parts if el_parts else None
    kb = _kernel_bytes(st)
    kms, kn = st["kernel_ms"], st["kernel_launches"]
    # the dominant kernel: the one whose stage takes the most device time per step
    # (k_group's stage is both of its tiers; its roofline is taken on the first tier's
    # launches, the ones its counters describe)
    dom = max(kb, key=lambda kk: st["ms_" + STAGE_OF[kk]])
    avg_ms = kms[dom] / max(1, kn[dom])
    achieved = kb[dom] / (avg_ms * 1e-3) / 1e9
    per_kernel = {kk: {"alg_bytes_per_launch": kb[kk], "avg_launch_ms": round(kms[kk] / max(1, kn[kk]), 3),
                       "achieved_gbs": round(kb[kk] / (kms[kk] / max(1, kn[kk]) * 1e-3) / 1e9, 1),
                       "frac": round(kb[kk] / (kms[kk] / max(1, kn[kk]) * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                       "stage_ms_per_step": round(st["ms_" + STAGE_OF[kk]] / args.device_steps, 3)}
                  for kk in kb if kn.get(kk)}
    # k_seed at its access granularity: every presence-filter check and bucket probe is a
    # random access that moves a 64-B sector (the 8-B filter word alone is the algorithmic
    # minimum above).  The two kinds hit different roofs: the filter (16 MB on C2) lives in
    # the 256 MB Infinity Cache, the table (GBs) in HBM, so each is priced at the random-64-B
    # gather rate measured over a buffer of its own size (b_filter_gbs, b_table_gbs), and the
    # streams (read bases, kept records) at the HBM peak: the mixed roof's time per launch
    # against the measured one is the kernel's roofline fraction
    if kn.get("k_seed"):
        nl = kn["k_seed"]
        sec = (st["n_bases"] + (st["n_filter"] + st["n_probes"]) * 64 + st["n_kept"] * 16) / nl
        k_ms = kms["k_seed"] / nl
        sgbs = sec / (k_ms * 1e-3) / 1e9
        sv = {"bytes_per_launch": sec, "achieved_gbs": round(sgbs, 1), "frac": round(sgbs / HBM_PEAK_GBS, 4),
              "frac_of_b_rand": round(sgbs / b_rand, 4) if b_rand else None,
              "random_accesses_per_launch": (st["n_filter"] + st["n_probes"]) / nl}
        if b_filt and b_table:
            roof_ms = ((st["n_filter"] / nl) * 64 / (b_filt * 1e9) + (st["n_probes"] / nl) * 64 / (b_table * 1e9) +
                       ((st["n_bases"] + st["n_kept"] * 16) / nl) / (HBM_PEAK_GBS * 1e9)) * 1e3
            sv["mixed_roof"] = {"b_filter_gbs": round(b_filt, 1), "filter_bytes": info["filter_bytes"],
                                "b_table_gbs": round(b_table, 1), "table_bytes": info["table_buckets"] * 64,
                                "roof_ms": round(roof_ms, 3), "launch_ms": round(k_ms, 3),
                                "frac": round(roof_ms / k_ms, 4)}
        per_kernel["k_seed"]["sector_view"] = sv
    # HBM traffic per launch of each kernel from the committed rocprofv3 summary of the
    # same bench (tools/prof_r03.sh, separate FETCH_SIZE / WRITE_SIZE passes over the
    # production device leg): FETCH_SIZE corrected for the kernel's read shape (random
    # 64-B sectors exact; occurrence runs by the 512-B-run calibration; row streams 2x)
    traffic, traffic_note, summ_name, summ_all = None, None, None, {}
    for name in ("r06z_rocprof_summary.json", "r05z_rocprof_summary.json", "r04z_rocprof_summary.json", "r04_rocprof_summary.json", "r03m_rocprof_summary.json", "r03k_rocprof_summary.json",
                 "r02e_rocprof_summary.json"):
        summ = os.path.join(ROOT, "profiles", name)
        if os.path.exists(summ):
            try:
                with open(summ) as f:
                    summ_all = json.load(f)
                summ_name = name
                break
            except Exception:
                pass
    for kk in per_kernel:
        t = summ_all.get(f"{kk}_traffic_bytes")
        if t:
            # k_group: 2 x FETCH + WRITE, calibrated on its exact access shape (round 6,
            # profiles/r06c_group_calibration.txt: FETCH_SIZE = 1/2 of the 128-B lines moved)
            shape = "guide_2x_fetch_plus_write" if kk == "k_group" else (t.get("shape") or "guide_2x_fetch_plus_write")
            per_kernel[kk]["traffic_bytes_per_launch"] = t.get(shape)
            per_kernel[kk]["traffic_over_alg"] = round(t.get(shape) / kb[kk], 3) if t.get(shape) else None
            per_kernel[kk]["rocprof_mean_ms"] = (summ_all.get(f"{kk}_device_leg") or {}).get("mean_ms")
            per_kernel[kk]["profile"] = f"profiles/{summ_name}"
    t = summ_all.get(f"{dom}_traffic_bytes", {})
    if t:
        traffic = per_kernel[dom].get("traffic_bytes_per_launch")
        traffic_note = {k: t.get(k) for k in ("raw_fetch_plus_write", "guide_2x_fetch_plus_write", "calibrated_runs")}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle.oracle import OracleIndex, params
        from tests._compare import split_reads
        cthreads = args.cpu_threads or threads
        oix = OracleIndex.from_fasta([sr_fa], k, threads=cthreads)
        p = params(**akw)
        allp, alln = ds.pb_seqs(), ds.pb_names()
        if args.cpu_sample_reads:
            nsamp = min(len(allp), args.cpu_sample_reads)
        else:
            # bounded sample: a pilot sizes it to about --cpu-seconds of oracle work (align + format)
            npil = max(1, min(len(allp), 4 * cthreads))
            tp = time.perf_counter()
            oix.align_format(p, alln[:npil], allp[:npil], threads=cthreads)
            psec = time.perf_counter() - tp
            rate = sum(len(x) for x in allp[:npil]) / max(psec, 1e-6)
            want = rate * args.cpu_seconds
            nsamp, acc = 0, 0
            while nsamp < len(allp) and acc < want:
                acc += len(allp[nsamp])
                nsamp += 1
            nsamp = max(nsamp, npil)
        pseqs, pnames = allp[:nsamp], alln[:nsamp]
        tc = time.perf_counter()
        exp = oix.align_format(p, pnames, pseqs, threads=cthreads)
        sec = time.perf_counter() - tc
        sbases = sum(len(x) for x in pseqs)
        oix.close()
        # the same sample through the GPU path (device formatting): parity of the baseline's output
        g = pbgpu.Aligner(index, **akw)
        rr = g.upload(pseqs, names=pnames)
        g.align_resident(rr)
        got = g.format_device(rr)
        rr.close()
        g.close()
        og, rg = split_reads(got)
        oe, re_ = split_reads(exp)
        mism = sum(1 for h in set(og) | set(oe) if sorted(rg.get(h, [])) != sorted(re_.get(h, [])))
        cpu = {"value": sbases / sec, "unit": "bases/s", "cores": cthreads, "kind": "port",
               "cpu_model": _cpu_model(),
               **_calibration(sbases / sec),
               "sample": f"first {nsamp} reads of the rank-0 shard ({sbases} bases, {exp.count(chr(10))} text lines) "
                         f"against the full {args.workload} index; oracle/ C restatement, align + coords text "
                         f"formatting, {cthreads} threads (the job's CPU share of the box), {sec:.2f} s",
               "gpu_parity_reads_checked": len(oe), "gpu_parity_reads_differing": mism}

    # ---- the C4r leg's figures (collectives on every rank) and its CPU oracle (rank 0, N = 1)
    c4_out = None
    if c4 is not None:
        bases4 = comm.sum(c4["bases"])
        st4, dsteps4 = c4["st"], max(1, args.device_steps)
        cpu4 = None
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            from oracle.oracle import OracleIndex, params
            from tests._compare import split_reads
            cthreads = args.cpu_threads or threads
            ds4 = c4["ds"]
            oix4 = OracleIndex.from_fasta([os.path.join(c4["wd"], "sr.fa")], 17, threads=cthreads)
            p4 = params(**dict(akw, k=17, unitig_lengths=ds4.unitig_lengths))
            allp4, alln4 = ds4.pb_seqs(), ds4.pb_names()
            npil = max(1, min(len(allp4), 2 * cthreads))
            tp = time.perf_counter()
            oix4.align_format(p4, alln4[:npil], allp4[:npil], threads=cthreads)
            rate = sum(len(x) for x in allp4[:npil]) / max(time.perf_counter() - tp, 1e-6)
            want, nsamp, acc = rate * args.c4r_cpu_seconds, 0, 0
            while nsamp < len(allp4) and acc < want:
                acc += len(allp4[nsamp])
                nsamp += 1
            nsamp = max(nsamp, npil)
            ps4, pn4 = allp4[:nsamp], alln4[:nsamp]
            tc = time.perf_counter()
            exp4 = oix4.align_format(p4, pn4, ps4, threads=cthreads)
            sec4 = time.perf_counter() - tc
            sb4 = sum(len(x) for x in ps4)
            oix4.close()
            g4 = pbgpu.Aligner(c4["ix"], **dict(akw, k=17, unitig_lengths=ds4.unitig_lengths))
            rr = g4.upload(ps4, names=pn4)
            g4.align_resident(rr)
            got4 = g4.format_device(rr)
            rr.close()
            g4.close()
            og, rg = split_reads(got4)
            oe, re_ = split_reads(exp4)
            mism4 = sum(1 for h in set(og) | set(oe) if sorted(rg.get(h, [])) != sorted(re_.get(h, [])))
            cpu4 = {"value": sb4 / sec4, "unit": "bases/s", "cores": cthreads, "kind": "port",
                    "sample": f"first {nsamp} C4r reads ({sb4} bases, {exp4.count(chr(10))} text lines), oracle/ C "
                              f"restatement, align + coords text, {cthreads} threads, {sec4:.2f} s",
                    "gpu_parity_reads_checked": len(oe), "gpu_parity_reads_differing": mism4}
        per_base = {n: st4[n] / max(1, st4["n_bases"]) for n in
                    ("n_kmers", "n_probes", "n_kept", "n_hits", "n_chains", "n_lis_tests", "n_records")}
        value_dev4 = bases4 * dsteps4 / c4["el_dev"]
        runs4 = c4.get("cmr_runs") or []
        c4_out = {
            "workload": "C4r: C4's repeat model (2% of a 16 Mbp genome in 5-50-copy repeats of 1-6 kb, 1% "
                        "substitutions) and read lengths (lognormal mean 12.5 kb, sigma 0.6: 15 kb N50), 800k "
                        f"super-reads, {args.c4r_reads} reads per GPU, production flags",
            "bases_per_gpu": c4["bases"],
            "value_device": value_dev4,
            "value_device_note": "reads resident in HBM, device path to sorted records in HBM, one aligner",
            "ms_per_step": c4["el_dev"] / dsteps4 * 1e3,
            "stage_ms_per_step": {s: round(st4["ms_" + s] / dsteps4, 3) for s in
                                  ("seed", "group", "lis", "fit", "records")},
            "counters_per_base": per_base,
            "group_refines_per_step": st4["group_refines"] / dsteps4,
            "value_create_mega_reads": bases4 / c4["cmr_wall"] if c4.get("cmr_wall") else None,
            "create_mega_reads_walls_s": [t["wall_s"] for t in runs4],
            "create_mega_reads_worst_wall_s": c4.get("cmr_worst"),
            "create_mega_reads_runs": runs4,
            "cpu_oracle": cpu4,
            "gpu_device_over_cpu": (value_dev4 / cpu4["value"]) if cpu4 else None,
            "generate_s": round(c4["gen_s"], 3),
        }
        c4["ix"].close()
        c4["ds"].close()
        shutil.rmtree(c4["wd"], ignore_errors=True)

    # ---- the C3 strong-scaling leg and the C4 leg (BASELINE configs[2] and [3]), after the C2
    # index is freed: every rank runs them (their collectives too)
    index_info_c2 = info
    index.close()
    index = None
    c3_out = c3_leg(args, comm, rank, world, local, threads, pbgpu, Dataset) if args.c3_reads > 0 else None
    c4_full = c4_leg(args, comm, rank, world, local, threads, pbgpu, Dataset, brand=not args.no_brand) \
        if args.c4_reads > 0 else None
    info = index_info_c2

    # SURVEY 8(d)'s whole-path algorithmic bytes of the device leg: 2-bit read stream,
    # 64-B index probes, occurrences enumerated (8 B), hits grouped (write + read, 16 B),
    # LIS predecessor tests (16 B), records out (96 B)
    dsteps = max(1, args.device_steps)
    path_bytes = (0.25 * st["n_bases"] + 64 * st["n_probes"] + 8 * st["n_hits"] + 16 * st["n_hits"] +
                  16 * st["n_lis_tests"] + 96 * st["n_records"]) / dsteps
    path_gbs = path_bytes / (el_dev / dsteps) / 1e9
    path_roof = {"bytes_alg_per_step": path_bytes, "achieved": path_gbs, "unit": "GB/s",
                 "frac": path_gbs / HBM_PEAK_GBS, "frac_of_b_rand": (path_gbs / b_rand) if b_rand else None,
                 "formula": "0.25*bases + 64*probes + 8*occurrences + 16*hits + 16*lis_tests + 96*records (SURVEY 8d)"}

    if rank == 0:
        stage = {n: round(sum(r[n] for r in rstats) / args.steps * 1e3, 3) for n in
                 ("read_seconds", "upload_seconds", "align_seconds", "format_seconds", "d2h_seconds",
                  "write_seconds", "writer_idle_seconds", "open_seconds", "close_seconds", "wall_seconds")}
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
            "data": "synthetic (tools/pbsynth.cc, seed 42; SURVEY.md §8d generator), written as FASTA",
            "value_device_aligners": value_device_al,
            "value_device_aligners_note": (f"value_device's leg with {args.device_aligners} aligners per GPU (the "
                                           "CLIs' default), the reads split between them and their launches "
                                           "overlapping; value_device and the roofline use one aligner"
                                           if value_device_al else None),
            "value_device": value_device,
            "value_device_note": "reads resident in HBM, device path to sorted records in HBM, no formatting / "
                                 "output (round-1 definition)",
            "value_create_mega_reads": value_cmr,
            "value_create_mega_reads_note": ("bin/create_mega_reads over the same files (overlap graph, tiling and "
                                             "paths on the GPU, text on the host), PacBio bases per second of the "
                                             f"median of {args.cmr_steps} cold runs (after one warm-up run; each "
                                             f"run's own --timing wall), -t {threads}") if value_cmr else None,
            "create_mega_reads_stage_s": ({kk: cmr_t[kk] for kk in ("wall_s", "align_s", "download_s", "graph_s",
                                                                     "output_bytes")} if cmr_t else None),
            "create_mega_reads_walls_s": walls if args.cmr_steps > 0 else None,
            "create_mega_reads_worst_wall_s": worst_cmr,
            # every timed run's own --timing stages (a slow run shows which stage it lost time in)
            "create_mega_reads_runs": cmr_runs if args.cmr_steps > 0 else None,
            "create_mega_reads_allocs": ({kk: cmr_t.get(kk) for kk in ("device_allocs", "device_allocs_late",
                                                                       "pinned_allocs", "pinned_allocs_late")}
                                         if cmr_t else None),
            "value_parts": value_parts,
            "value_parts_note": (f"the same coords out into {args.parts} part files per GPU (jf_aligner --parts, the "
                                 "reference's split-and-cat in one process: one reader / writer per part, 2 aligners "
                                 "each; the parts concatenated are the one-file output)") if value_parts else None,
            "parts_stage_ms_per_step": {n: round(sum(r[n] for r in pstats) / args.steps * 1e3, 3) for n in
                                        ("write_seconds", "align_seconds", "d2h_seconds", "writer_idle_seconds",
                                         "wall_seconds")} if pstats else None,
            "config": {
                "workload": {"C1": "C1: 100 PB x 10 kb vs 1k SRs, k=17",
                             "C2": "C2 E. coli-scale: 50k PB (lognormal mean 12 kb, CLR 13%) per GPU vs 200k SRs, k=17",
                             "C3": "C3 yeast-scale: PB (mean 12 kb) vs 1M SRs, k=21",
                             "C4r": "C4r: C4's repeat model and 15-kb-N50 reads on a 16 Mbp genome vs 800k SRs, k=17"}[
                                 args.workload],
                "flags": f"-m {k} --psa-min 13 -l ul.txt -k 31 -f -B 15 --max-count 5000 --stretch-cap 10000",
                "step": "pbgpu_run: pb.fa -> coords file (parse, upload, align, device format, D2H, write)",
                "reads_per_gpu": len(off) - 1,
                "bases_per_gpu": bases_rank,
                "coords_bytes_per_step": coords_bytes,
                "records_per_step": rstats[-1]["n_records"],
                "batches_per_step": rstats[-1]["n_batches"],
                "batch_bases": int(args.batch_bases),
                "parallelism": f"read-sharded x{world}, index replicated per GPU",
                "streams_per_gpu": args.streams,
                "index": {"n_sr": info["n_sr"], "text_len": info["text_len"], "n_kmers": info["n_kmers"],
                          "device_bytes": info["device_bytes"], "build_s": round(t_index, 3),
                          "generate_and_write_s": round(t_gen, 3)},
                "stage_ms_per_step": stage,
                # device / pinned allocations inside the timed steps (the runner is warm: 0)
                "allocs_in_timed_steps": {n: sum(r[n] for r in rstats) for n in
                                          ("n_device_allocs", "n_pinned_allocs")},
                "device_leg": {"ms_per_step": el_dev / args.device_steps * 1e3, "streams": args.device_streams,
                               "chunks": len(cuts) - 1,
                               "stage_ms_per_step": {s: round(st["ms_" + s] / args.device_steps, 3) for s in
                                                     ("seed", "group", "lis", "fit", "records")},
                               "kernel_ms_per_launch": {kk: round(kms[kk] / max(1, kn[kk]), 3) for kk in kms},
                               "kernel_launches": dict(kn),
                               "host_order_ms_per_step": round(st["ms_host_order"] / args.device_steps, 3),
                               "counters_per_step": {n: st[n] // args.device_steps for n in
                                                     ("n_kmers", "n_probes", "n_kept", "n_hits", "n_chains",
                                                      "n_lis_tests", "n_records")},
                               "path_roofline": path_roof},
                "device_leg_default_flags": {
                    "flags": f"-m {k} --psa-min 13 (defaults: no -l/-k/-f, -B 17, --max-count 5000)",
                    "value_device": value_device2,
                    "ms_per_step": el_dev2 / args.device_steps * 1e3,
                    "records_per_step": st2["n_records"] // max(1, args.device_steps)} if el_dev2 else None,
                "end_to_end_including_build_s": round(t_index + elapsed / args.steps, 3),
                "fit_dtype": "f64",
            },
            "roofline": {"bound": "hbm", "kernel": dom, "rocprof_kernel": ROCPROF_FILE[dom], "achieved": achieved,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "alg_bytes_per_launch": kb[dom], "avg_launch_ms": avg_ms,
                         "traffic_source": (f"profiles/{summ_name} (FETCH_SIZE as the read shape needs it -- "
                                            f"{(summ_all.get(dom + '_traffic_bytes') or {}).get('shape', '?')} -- "
                                            "+ WRITE_SIZE, per device-leg launch, separate passes)")
                         if traffic else None,
                         "traffic_alternatives": traffic_note,
                         "b_rand_gbs": b_rand, "frac_of_b_rand": (achieved / b_rand) if b_rand else None,
                         "b_run512_gbs": b_run, "frac_of_b_run512": (achieved / b_run) if b_run else None,
                         "by_kernel": per_kernel},
            "cpu_baseline": cpu,
            "c4r": c4_out,
            "c3": c3_out,
            "c4": c4_full,
        }
        print(json.dumps(out), flush=True)
    shutil.rmtree(wd, ignore_errors=True)


if __name__ == "__main__":
    main()
