#!/usr/bin/env python3
"""Phase profile of k_coords (s_memtime per wave, summed) with the -DPBGPU_PROF
library, and the wave-time split by chunk count (CH lis points per chunk):
  PBGPU_LIB=pacbio_amd/libpbgpu_prof.so python tools/prof_coords.py --reads 50000"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=50000)
    ap.add_argument("--workload", default="C2")
    a = ap.parse_args()
    from pacbio_amd import pbgpu
    from tools.synth import Dataset
    ds = Dataset(a.workload, seed=42, threads=16, n_pb=a.reads)
    ix = pbgpu.Index.from_records(ds.sr_names(), ds.sr_seqs(), 17)
    al = pbgpu.Aligner(ix, k=17, forward=True, unitigs_k=31, unitig_lengths=ds.unitig_lengths,
                       bases_matching=15.0, max_count=5000, stretch_cap=10000.0)
    blob, off = ds.pb_blob()
    rr = al.upload(blob=blob, offsets=off)
    al.align_resident(rr)
    L = pbgpu.lib()
    f = L.pbgpu_debug_prof
    f.argtypes = [C.POINTER(C.c_ulonglong), C.c_int, C.c_int]
    buf = (C.c_ulonglong * 96)()
    f(buf, 96, 1)
    al.reset_stats()
    al.align_resident(rr)
    pbgpu.device_synchronize(0)
    f(buf, 96, 1)
    st = al.stats()
    g = list(buf)
    waves = max(1, g[32])
    tot = max(1, g[33])
    print(f"k_coords: first launch {st['kernel_ms']['k_coords']:.2f} ms, fit stage {st['ms_fit']:.2f} ms; "
          f"waves={g[32]} chunks/wave={g[39] / waves:.2f} lane-chunk efficiency={g[40] / max(1, 64 * g[39]):.3f} "
          f"fit_chains={st['fit_chains']} fit_points={st['fit_points']} "
          f"pass3 waves={g[41]}")
    for n, x in zip(["prologue", "pass1 fit+info", "pass2 err", "alloc/finish", "pass3 info", "emit"],
                    [g[34], g[35], g[36], g[37], g[38], g[42]]):
        print(f"  {n:16s} {x / waves:10.0f} ticks/wave ({100.0 * x / tot:5.1f}%)")
    print("  by wave chunk count (log2 bucket): waves, ticks share, ticks/wave")
    for b in range(16):
        if g[64 + b]:
            lo = 0 if b == 0 else 1 << (b - 1)
            print(f"    nch in [{lo:6d},{(1 << b) - 1 if b else 0:6d}] waves={g[64 + b]:9d} "
                  f"share={100.0 * g[48 + b] / tot:5.1f}% ticks/wave={g[48 + b] / g[64 + b]:10.0f}")


if __name__ == "__main__":
    main()
