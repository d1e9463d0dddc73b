#!/usr/bin/env python3
"""Phase profile of k_lis (s_memtime per wave, summed): run with the
-DPBGPU_PROF library, e.g.
  PBGPU_LIB=pacbio_amd/libpbgpu_prof.so python tools/prof_lis.py --reads 10000"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=10000)
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
    buf = (C.c_ulonglong * 160)()
    f = getattr(L, "pbgpu_debug_prof", None)  # -DPBGPU_PROF builds only
    if f is None:
        al.reset_stats()
        al.align_resident(rr)
        pbgpu.device_synchronize(0)
        st = al.stats()
        print(f"k_group tier0: {st['kernel_ms']['k_group']:.2f} ms, k_lis: {st['kernel_ms']['k_lis']:.2f} ms")
        print(f"stages ms: seed {st['ms_seed']:.1f} group {st['ms_group']:.1f} lis {st['ms_lis']:.1f} fit {st['ms_fit']:.1f} "
              f"records {st['ms_records']:.1f}; group refines {st['group_refines']}, HBM-table reads {st['group_hbm_reads']}")
        return
    f.argtypes = [C.POINTER(C.c_ulonglong), C.c_int, C.c_int]
    f(buf, 160, 1)
    al.reset_stats()
    al.align_resident(rr)
    pbgpu.device_synchronize(0)
    f(buf, 160, 1)
    st = al.stats()
    names = ["row_load_issue", "lds_fetch", "element_loop", "row_store", "sweep", "wave_total", "chunks", "waves"]
    v = list(buf)[:8]
    waves = max(1, v[7])
    print(f"k_lis: {st['kernel_ms']['k_lis']:.2f} ms, waves={waves}, chunks/wave={v[6] / waves:.1f}, "
          f"hits={st['n_hits']}, tests={st['n_lis_tests']}")
    for n, x in zip(names[:6], v[:6]):
        print(f"  {n:16s} {x / waves:12.0f} ticks/wave  ({100.0 * x / max(1, v[5]):5.1f}%)")
    g = list(buf)
    print(f"k_lis_w: literal steps={g[20]} (scan iterations {g[23]}), clean runs={g[21]} covering {g[22]} elements")
    for label, sb in (("k_lis_w<255>", 24), ("k_lis_w<511>", 28)):
        tot = max(1, g[sb + 3])
        print(f"  {label}: order {100.0 * g[sb] / tot:5.1f}% ({g[sb + 1]} rounds), forward {100.0 * g[sb + 2] / tot:5.1f}%, "
              f"backtrack+rest {100.0 * (tot - g[sb] - g[sb + 2]) / tot:5.1f}%, strand ticks {g[sb + 3]}")
    print(f"stages ms: seed {st['ms_seed']:.1f} group {st['ms_group']:.1f} lis {st['ms_lis']:.1f} fit {st['ms_fit']:.1f} "
          f"records {st['ms_records']:.1f}")
    print(f"counters: hits {st['n_hits']}, lis tests {st['n_lis_tests']}, chains {st.get('n_chains')}, "
          f"records {st.get('n_records')}, bases {sum(len(s) for s in ds.pb_seqs()) if a.reads <= 20000 else 'n/a'}")
    print(f"k_group 8192-slot tier table work (wave ticks): pass 0 first probes {g[112]}, walks+counts {g[113]}, "
          f"windows walking {g[114]}; pass 1 first probes {g[115]}, walks {g[116]}, windows walking {g[117]}; "
          f"mine hits (pass 0) {g[118]}")
    for label, sb in (("k_group 2048-slot tier", 8), ("k_group 8192-slot tier", 14)):
        blocks = max(1, g[sb + 5])
        print(f"{label}: blocks={g[sb + 5]} (ms: tier0 {st['kernel_ms']['k_group']:.2f})")
        for n, x in zip(["setup", "pass0 steps", "pass1 steps", "compaction", "block_total"], g[sb:sb + 5]):
            print(f"  {n:16s} {x / blocks:12.0f} ticks/block ({100.0 * x / max(1, g[sb + 4]):5.1f}%)")


if __name__ == "__main__":
    main()
