#!/usr/bin/env python3
"""Experiment: k_coords time with and without kmers_info (-l/-k), C2 reads subset."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=20000)
    a = ap.parse_args()
    from pacbio_amd import pbgpu
    from tools.synth import Dataset
    ds = Dataset("C2", seed=42, threads=16, n_pb=a.reads)
    ix = pbgpu.Index.from_records(ds.sr_names(), ds.sr_seqs(), 17)
    blob, off = ds.pb_blob()
    for label, kw in (("with_info", dict(forward=True, unitigs_k=31, unitig_lengths=ds.unitig_lengths)),
                      ("no_info", dict(forward=True))):
        al = pbgpu.Aligner(ix, k=17, bases_matching=15.0, max_count=5000, stretch_cap=10000.0, **kw)
        rr = al.upload(blob=blob, offsets=off)
        al.align_resident(rr)
        al.reset_stats()
        al.align_resident(rr)
        st = al.stats()
        print(label, {k: round(v, 3) for k, v in st["kernel_ms"].items()}, "fit_ms", round(st["ms_fit"], 3),
              "points", st["fit_points"], "chains", st["fit_chains"], flush=True)
        rr.close()
        al.close()


if __name__ == "__main__":
    main()
