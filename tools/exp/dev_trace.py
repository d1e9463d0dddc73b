#!/usr/bin/env python3
"""The bench's device leg (C2, one aligner, reads resident) twice, for a kernel / copy
trace: rocprofv3 --kernel-trace --memory-copy-trace -- python3 tools/exp/dev_trace.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from pacbio_amd import pbgpu  # noqa: E402
from tools.synth import Dataset  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 50000
ds = Dataset("C2", seed=42, threads=16, n_pb=n)
d = "/tmp/dev_trace_c2"
os.makedirs(d, exist_ok=True)
ds.write(d)
ix = pbgpu.Index.from_fasta([os.path.join(d, "sr.fa")], 17, psa_min=13)
al = pbgpu.StreamAligner(ix, streams=1, k=17, forward=True, unitigs_k=31, unitig_lengths=ds.unitig_lengths,
                         bases_matching=15.0, max_count=5000, stretch_cap=10000.0)
blob, off = ds.pb_blob()
rr = al.upload(blob=blob, offsets=off)
for i in range(3):
    pbgpu.device_synchronize(0)
    t = time.perf_counter()
    al.align_resident(rr)
    pbgpu.device_synchronize(0)
    print(f"align_resident {i}: {(time.perf_counter() - t) * 1e3:.1f} ms", flush=True)
ds.close()
