#!/usr/bin/env python3
"""C2 index: build from FASTA vs load from the on-disk cache (pbgpu_index_save/load)."""
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    from pacbio_amd import pbgpu
    from tools.synth import Dataset
    d = tempfile.mkdtemp(prefix="ixc_", dir="/tmp")
    ds = Dataset("C2", seed=42, threads=16, n_pb=10)
    ds.write(d)
    sr = os.path.join(d, "sr.fa")
    pbgpu.Index.from_fasta([sr], 17).close()  # warm-up (device init, file in page cache)
    t0 = time.perf_counter()
    ix = pbgpu.Index.from_fasta([sr], 17, threads=16)
    t1 = time.perf_counter()
    path = os.path.join(d, "c2.pbix")
    ix.save(path, tag="c2")
    t2 = time.perf_counter()
    info = ix.info()
    ix.close()
    t3 = time.perf_counter()
    ix2 = pbgpu.Index.load(path, tag="c2")
    t4 = time.perf_counter()
    assert ix2.info()["device_bytes"] == info["device_bytes"]
    print(f"C2 index: build from FASTA {t1 - t0:.3f} s, save {t2 - t1:.3f} s ({os.path.getsize(path) / 1e9:.2f} GB), "
          f"load {t4 - t3:.3f} s; device bytes {info['device_bytes'] / 1e9:.2f} GB", flush=True)


if __name__ == "__main__":
    main()
