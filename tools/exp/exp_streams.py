#!/usr/bin/env python3
"""Wall time of one C2 step with the 50k reads split over S aligners (own
stream and buffers each, one host thread each) sharing one index."""
import argparse
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", default="1,2,3,4")
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    import numpy as np
    from pacbio_amd import pbgpu
    from tools.synth import Dataset
    ds = Dataset("C2", seed=42, threads=16, n_pb=50000)
    ix = pbgpu.Index.from_records(ds.sr_names(), ds.sr_seqs(), 17, psa_min=13)
    blob, off = ds.pb_blob()
    raw = bytes(blob)
    off = np.asarray(off, dtype=np.uint64)
    for S in [int(x) for x in a.streams.split(",")]:
        als, rds = [], []
        n = len(off) - 1
        cuts = [n * i // S for i in range(S + 1)]
        for i in range(S):
            al = pbgpu.Aligner(ix, k=17, forward=True, unitigs_k=31, unitig_lengths=ds.unitig_lengths,
                               bases_matching=15.0, max_count=5000, stretch_cap=10000.0)
            lo, hi = cuts[i], cuts[i + 1]
            sub_off = off[lo:hi + 1] - off[lo]
            sub_blob = raw[int(off[lo]):int(off[hi])]
            rds.append(al.upload(blob=sub_blob, offsets=sub_off))
            als.append(al)

        def step():
            th = [threading.Thread(target=al.align_resident, args=(r,)) for al, r in zip(als, rds)]
            for t in th: t.start()
            for t in th: t.join()
        step()
        pbgpu.device_synchronize(0)
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        pbgpu.device_synchronize(0)
        ms = (time.perf_counter() - t0) / a.steps * 1e3
        recs = sum(al.stats()["n_records"] for al in als)
        print(f"S={S}: {ms:.2f} ms/step, {int(off[-1]) / ms / 1e6:.3f} Gbases/s, records/step={recs // (a.steps + 1)}",
              flush=True)
        for r in rds: r.close()
        for al in als: al.close()
    ix.close()


if __name__ == "__main__":
    main()
