#!/usr/bin/env python3
"""One pbgpu_align_resident call on all of C3 (300k reads, ~3.6 Gbases, k = 21, production
flags): the aligner cuts it into read chunks of at most free memory / 128 bases itself
(round 5; round 4's single call ran out of HBM).  Prints the call's time, its k_seed
launches (one per chunk), records and the device's free-memory low point, then the same
reads in 1.5-Gbase calls for the record count to agree with.
  python tools/exp/c3_resident.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    from pacbio_amd import pbgpu
    from tools.synth import Dataset
    t0 = time.time()
    ds = Dataset("C3", seed=42, threads=16)
    blob, off = ds.pb_blob()
    print(f"C3 generated: {len(off) - 1} reads, {int(off[-1])} bases, {time.time() - t0:.1f} s", flush=True)
    ix = pbgpu.Index.from_records(ds.sr_names(), ds.sr_seqs(), 21)
    kw = dict(k=21, forward=True, unitigs_k=31, unitig_lengths=ds.unitig_lengths, bases_matching=15.0,
              max_count=5000, stretch_cap=10000.0)
    al = pbgpu.Aligner(ix, **kw)
    rr = al.upload(blob=blob, offsets=off)
    pbgpu.device_synchronize(0)
    t = time.time()
    al.align_resident(rr)
    pbgpu.device_synchronize(0)
    wall = time.time() - t
    st = al.stats()
    one = {"what": "C3 in one pbgpu_align_resident call", "reads": len(off) - 1, "bases": int(off[-1]),
           "wall_s": round(wall, 3), "gbases_per_s": round(int(off[-1]) / wall / 1e9, 3),
           "k_seed_launches": st["kernel_launches"]["k_seed"], "n_records": st["n_records"],
           "n_hits": st["n_hits"]}
    print(json.dumps(one), flush=True)
    rr.close()
    # the same reads in calls of <= 1.5 Gbases (bench.py's device leg)
    cuts, acc = [0], 0
    for r in range(1, len(off)):
        if int(off[r]) - int(off[cuts[-1]]) > 1.5e9 and r - 1 > cuts[-1]:
            cuts.append(r - 1)
    cuts.append(len(off) - 1)
    al.reset_stats()
    for r0, r1 in zip(cuts[:-1], cuts[1:]):
        b0, b1 = int(off[r0]), int(off[r1])
        c = al.upload(blob=bytes(blob[b0:b1]), offsets=off[r0:r1 + 1] - off[r0])
        al.align_resident(c)
        acc += al.stats()["n_records"]
        al.reset_stats()
        c.close()
    print(json.dumps({"what": "C3 in calls of <= 1.5 Gbases", "calls": len(cuts) - 1, "n_records": acc,
                      "same_records": acc == one["n_records"]}), flush=True)
    al.close()
    ix.close()
    ds.close()


if __name__ == "__main__":
    main()
