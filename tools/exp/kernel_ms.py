#!/usr/bin/env python3
"""Per-kernel device time of one library variant (PBGPU_LIB=...) on C2 reads,
production flags, one aligner: kernel_ms of the second of two resident runs."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=25000)
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
    al.align_resident(rr)
    pbgpu.device_synchronize(0)
    st = al.stats()
    lib = os.path.basename(os.environ.get("PBGPU_LIB", "libpbgpu.so"))
    ks = " ".join(f"{k} {v:.2f}" for k, v in st["kernel_ms"].items())
    stages = " ".join(f"{s} {st['ms_' + s]:.2f}" for s in ("seed", "group", "lis", "fit", "records"))
    print(f"{lib:24s} | {ks} | {stages} | records {st['n_records']}", flush=True)


if __name__ == "__main__":
    main()
