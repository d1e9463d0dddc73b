#!/usr/bin/env python3
"""The C4 configuration's device path (full 10M-super-read index from the generator's
buffers, --reads reads of 15 kb N50, production flags, one resident call per <= 0.5 Gbases,
one aligner): stage times, counters and the group stage's work items; with the -DPBGPU_PROF
library (PBGPU_LIB=pacbio_amd/libpbgpu_prof.so) also k_group's per-tier phase ticks."""
import argparse
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=50000)
    ap.add_argument("--preset", default="C4")
    ap.add_argument("--chunk-bases", type=float, default=0.5e9)
    a = ap.parse_args()
    from pacbio_amd import pbgpu
    from tools.synth import Dataset
    t0 = time.time()
    ds = Dataset(a.preset, seed=42, threads=16, n_pb=a.reads)
    ix = pbgpu.Index.from_pointers(*ds.sr_pointers(), k=17)
    print(f"generate + build {time.time() - t0:.1f} s", flush=True)
    al = pbgpu.Aligner(ix, k=17, forward=True, unitigs_k=31, unitig_lengths=ds.unitig_lengths, bases_matching=15.0,
                       max_count=5000, stretch_cap=10000.0)
    blob, off = ds.pb_blob()
    cuts = [0]
    for r in range(1, len(off)):
        if int(off[r]) - int(off[cuts[-1]]) > a.chunk_bases and r - 1 > cuts[-1]:
            cuts.append(r - 1)
    cuts.append(len(off) - 1)
    chunks = [al.upload(blob=bytes(memoryview(blob)[int(off[r0]):int(off[r1])]), offsets=off[r0:r1 + 1] - off[r0])
              for r0, r1 in zip(cuts[:-1], cuts[1:])]
    for c in chunks:
        al.align_resident(c)
    L = pbgpu.lib()
    f = getattr(L, "pbgpu_debug_prof", None)  # -DPBGPU_PROF builds only
    buf = (C.c_ulonglong * 160)()
    if f is not None:
        f.argtypes = [C.POINTER(C.c_ulonglong), C.c_int, C.c_int]
        f(buf, 160, 1)
    al.reset_stats()
    pbgpu.device_synchronize(0)
    t = time.perf_counter()
    for c in chunks:
        al.align_resident(c)
    pbgpu.device_synchronize(0)
    el = time.perf_counter() - t
    st = al.stats()
    nb = st["n_bases"]
    print(f"{a.preset} {a.reads} reads, {nb} bases, {len(chunks)} calls: {el * 1e3:.1f} ms, {nb / el / 1e9:.3f} Gbases/s")
    print(f"stages ms: seed {st['ms_seed']:.1f} group {st['ms_group']:.1f} lis {st['ms_lis']:.1f} fit {st['ms_fit']:.1f} "
          f"records {st['ms_records']:.1f}")
    print(f"per base: hits {st['n_hits'] / nb:.3f} chains {st['n_chains'] / nb:.4f} kept {st['n_kept'] / nb:.4f} "
          f"records {st['n_records'] / nb:.4f}; hits per chain {st['n_hits'] / max(1, st['n_chains']):.1f}")
    print(f"group: refines {st['group_refines']}, HBM-table reads {st['group_hbm_reads']}, overflowing items "
          f"{st['group_overflow_items']}; launches {dict(st['kernel_launches'])}")
    if f is not None:
        f(buf, 160, 1)
        g = list(buf)
        print(f"k_group 8192-slot tier table work (wave ticks): pass 0 first probes {g[112]}, walks+counts {g[113]}, "
              f"windows walking {g[114]}; pass 1 first probes {g[115]}, walks {g[116]}, windows walking {g[117]}; "
              f"mine hits (pass 0) {g[118]}")
        waves = max(1, g[32])
        tot = max(1, g[33])
        print(f"k_coords: waves={g[32]} chunks/wave={g[39] / waves:.2f} fit_chains={st['fit_chains']} "
              f"fit_points={st['fit_points']}")
        for n, x in zip(["prologue", "pass1 fit+info", "pass2 err", "alloc/finish", "pass3 info", "emit"],
                        [g[34], g[35], g[36], g[37], g[38], g[42]]):
            print(f"  {n:16s} {x / waves:10.0f} ticks/wave ({100.0 * x / tot:5.1f}%)")
        for label, sb in (("k_group 2048-slot tier", 8), ("k_group 8192-slot tier", 14)):
            blocks = max(1, g[sb + 5])
            print(f"{label}: blocks={g[sb + 5]}")
            for n, x in zip(["setup", "pass0 steps", "pass1 steps", "compaction", "block_total"], g[sb:sb + 5]):
                print(f"  {n:16s} {x / blocks:12.0f} ticks/block ({100.0 * x / max(1, g[sb + 4]):5.1f}%)")


if __name__ == "__main__":
    main()
