#!/usr/bin/env python3
"""k_coords timing of one library variant (PBGPU_LIB=...): first k_coords launch
and fit stage over the C2 workload (results of EXP variants are not checked)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=50000)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    from pacbio_amd import pbgpu
    from tools.synth import Dataset
    ds = Dataset("C2", seed=42, threads=16, n_pb=a.reads)
    ix = pbgpu.Index.from_records(ds.sr_names(), ds.sr_seqs(), 17)
    al = pbgpu.Aligner(ix, k=17, forward=True, unitigs_k=31, unitig_lengths=ds.unitig_lengths,
                       bases_matching=15.0, max_count=5000, stretch_cap=10000.0)
    blob, off = ds.pb_blob()
    rr = al.upload(blob=blob, offsets=off)
    al.align_resident(rr)
    al.reset_stats()
    for _ in range(a.reps):
        al.align_resident(rr)
    st = al.stats()
    n = st["kernel_launches"]["k_coords"]
    print(f"{os.path.basename(os.environ.get('PBGPU_LIB', 'libpbgpu.so')):28s} k_coords {st['kernel_ms']['k_coords'] / n:7.3f} ms/launch"
          f"  fit {st['ms_fit'] / a.reps:7.3f} ms/step  lis {st['ms_lis'] / a.reps:7.3f}  records {st['n_records'] // a.reps}",
          flush=True)


if __name__ == "__main__":
    main()
