#!/usr/bin/env python3
"""The device leg alone (bench.py's value_device: C2 50k reads resident, one aligner, production
flags), a warm-up call and two timed calls, for a kernel trace of one call's launches and gaps:
  rocprofv3 --kernel-trace --output-format csv -d DIR -- python3 tools/exp/device_leg_trace.py
  python3 tools/exp/device_leg_trace.py --parse DIR/.../kernel_trace.csv"""
import csv
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def run():
    from pacbio_amd import pbgpu
    from tools.synth import Dataset
    ds = Dataset("C2", seed=42, threads=16, n_pb=50000)
    blob, off = ds.pb_blob()
    ix = pbgpu.Index.from_records(ds.sr_names(), ds.sr_seqs(), 17)
    al = pbgpu.Aligner(ix, k=17, forward=True, unitigs_k=31, unitig_lengths=ds.unitig_lengths, bases_matching=15.0,
                       max_count=5000, stretch_cap=10000.0)
    rr = al.upload(blob=blob, offsets=off)
    for i in range(3):
        pbgpu.device_synchronize(0)
        t = time.time()
        al.align_resident(rr)
        pbgpu.device_synchronize(0)
        print(f"call {i}: {1e3 * (time.time() - t):.2f} ms", flush=True)
    rr.close(); al.close(); ix.close(); ds.close()


def parse(path):
    rows = list(csv.DictReader(open(path)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
    seeds = [i for i, k in enumerate(ks) if "k_seed" in k[2]]
    a = seeds[-1]
    # back to the first launch after the previous call's last kernel (a gap > 2 ms)
    while a > 0 and ks[a][0] - ks[a - 1][1] < 2_000_000:
        a -= 1
    t0, prev, busy = ks[a][0], ks[a][0], 0
    for s, e, n in ks[a:]:
        print(f"{(s - t0) / 1e6:9.3f} gap {(s - prev) / 1e6:7.3f} dur {(e - s) / 1e6:7.3f}  {n[:90]}")
        busy += e - s
        prev = max(prev, e)
    print(f"span {(prev - t0) / 1e6:.3f} ms, kernels busy {busy / 1e6:.3f} ms, launches {len(ks) - a}")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--parse":
        parse(sys.argv[2])
    else:
        run()
