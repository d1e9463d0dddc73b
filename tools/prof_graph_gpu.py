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
    ap.add_argument("--workload", default="C2", help="a tools/synth.py preset (C4r: C4's repeat model and read lengths)")
    a = ap.parse_args()
    from pacbio_amd import pbgpu
    from tools.synth import Dataset
    ds = Dataset(a.workload, seed=42, threads=16, n_pb=a.reads)
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
    buf = (C.c_ulonglong * 160)()
    if f is not None:
        f.argtypes = [C.POINTER(C.c_ulonglong), C.c_int, C.c_int]
        f(buf, 160, 1)
    al.reset_stats()
    t = time.time()
    al.align_resident(rr)
    pbgpu.device_synchronize(0)
    wall = time.time() - t
    st = al.stats()
    print(f"align_resident {wall * 1e3:.1f} ms, graph {st['ms_graph']:.2f} ms over {st['graph_records']} records, "
          f"{st['graph_ovf_nodes']} nodes of more than 64 edges")
    print(f"{a.workload}: {a.reads} reads, {st['graph_records'] / max(1, a.reads):.0f} records a read, "
          f"{st['graph_host_reads']} left to the host graph (> 8192 records): "
          f"{100.0 * st['graph_host_reads'] / max(1, a.reads):.3f}%")
    if f is not None:
        f(buf, 160, 1)
        for tier, base in (("<= 1024 records", 80), ("> 1024 records", 96)):
            v = list(buf)[base:base + 8]
            nn, nb = max(1, v[6]), max(1, v[7])
            print(f"k_graph_relax {tier}: blocks {v[7]}, nodes {v[6]}, chunks {v[1]} ({v[1] / nn:.2f} a node); "
                  f"ticks a node: paths wave {v[2] / nn:.0f} (chunk work {v[0] / nn:.0f}), "
                  f"union wave {v[5] / nn:.0f} (finds {v[3] / nn:.0f}, merges {v[4] / nn:.0f})")
        rb = list(buf)[140:144]
        if rb[3]:
            print(f"k_graph_relax_big: blocks {rb[3]}, nodes {rb[2]}; ticks a node: paths wave {rb[0] / max(1, rb[2]):.0f}, "
                  f"union wave {rb[1] / max(1, rb[2]):.0f}")
        e = list(buf)[128:131]
        print(f"k_graph_edges: positions scanned {e[0]} ({e[0] / max(1, st['graph_records']):.1f} a node), past the "
              f"staged window {e[1]}, name tests {e[2]}")
        w = list(buf)[88:96]
        nw = max(1, w[5])
        print(f"k_mega: waves {w[5]}, candidates {w[7] >> 32}, components {w[7] & 0xffffffff}, "
              f"longest wave {w[6]} ticks")
        for nm, x in zip(["candidates", "components", "sort + tiling", "final sort", "paths"], w[:5]):
            print(f"  {nm:14s} {x / nw:10.0f} ticks a wave")
    ds.close()


if __name__ == "__main__":
    main()
