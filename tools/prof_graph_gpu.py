#!/usr/bin/env python3
"""Phase profile of k_graph (the create_mega_reads overlap graph on the GPU):
  PBGPU_LIB=pacbio_amd/libpbgpu_prof.so python tools/prof_graph_gpu.py --reads 10000"""
import argparse
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=10000)
    a = ap.parse_args()
    from pacbio_amd import pbgpu
    from tools.synth import Dataset
    ds = Dataset("C2", seed=42, threads=16, n_pb=a.reads)
    names = [n.decode() for n in ds.sr_names()]
    ix = pbgpu.Index.from_records(ds.sr_names(), ds.sr_seqs(), 17)
    ul = [int(x) for x in ds.unitig_lengths]
    al = pbgpu.Aligner(ix, k=17, forward=True, unitigs_k=31, unitig_lengths=ul, bases_matching=15.0,
                       max_count=5000, stretch_cap=10000.0)
    al.set_graph([pbgpu.parse_unitigs(n) for n in names], ul, 31, mega_reads=True)
    blob, off = ds.pb_blob()
    rr = al.upload(blob=blob, offsets=off)
    al.align_resident(rr)
    L = pbgpu.lib()
    f = getattr(L, "pbgpu_debug_prof", None)
    buf = (C.c_ulonglong * 96)()
    if f is not None:
        f.argtypes = [C.POINTER(C.c_ulonglong), C.c_int, C.c_int]
        f(buf, 96, 1)
    al.reset_stats()
    t = time.time()
    al.align_resident(rr)
    pbgpu.device_synchronize(0)
    wall = time.time() - t
    st = al.stats()
    print(f"align_resident {wall * 1e3:.1f} ms, graph {st['ms_graph']:.2f} ms over {st['graph_records']} records")
    if f is not None:
        f(buf, 96, 1)
        v = list(buf)[80:88]
        tot = max(1, v[6])
        print(f"k_graph: waves {v[7]}, nodes {v[5]}, chunks {v[4]} ({v[4] / max(1, v[5]):.2f} a node), "
              f"ticks a node {v[6] / max(1, v[5]):.0f}")
        for nm, x in zip(["chunk scan", "names + sums", "node updates", "unions"], v[:4]):
            print(f"  {nm:14s} {x / max(1, v[5]):8.0f} ticks a node ({100.0 * x / tot:5.1f}%)")
        w = list(buf)[88:96]
        nw = max(1, w[5])
        print(f"k_mega: waves {w[5]}, candidates {w[7] >> 32}, components {w[7] & 0xffffffff}, "
              f"longest wave {w[6]} ticks")
        for nm, x in zip(["candidates", "components", "sort + tiling", "final sort", "paths"], w[:5]):
            print(f"  {nm:14s} {x / nw:10.0f} ticks a wave")
    ds.close()


if __name__ == "__main__":
    main()
