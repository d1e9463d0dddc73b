#!/usr/bin/env python3
"""create_mega_reads (row f3) on the C2 workload: the CLI from FASTA on disk to
the mega-reads file, beside jf_aligner's coords-out run on the same input.
Prints one JSON line (stage times from --timing).  Usage (GPU box):
  python tools/bench_cmr.py [--reads 50000] [--threads 16]"""
import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _run(cmd):
    t0 = time.perf_counter()
    r = subprocess.run(cmd, capture_output=True, text=True)
    wall = time.perf_counter() - t0
    if r.returncode:
        sys.exit(f"{cmd[0]} failed: {r.stderr[-2000:]}")
    timing = json.loads(r.stderr.strip().splitlines()[-1])
    return wall, timing


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=50000)
    ap.add_argument("--threads", type=int, default=int(os.environ.get("OMP_NUM_THREADS", "16")))
    ap.add_argument("--workdir", default="/tmp")
    a = ap.parse_args()
    from tools.synth import Dataset
    d = tempfile.mkdtemp(prefix="pbgpu_cmr_", dir=a.workdir)
    try:
        ds = Dataset("C2", seed=42, threads=16, n_pb=a.reads)
        ds.write(d)
        ds.close()
        sr, pb, ul = (os.path.join(d, f) for f in ("sr.fa", "pb.fa", "ul.txt"))
        flags = ["-s", "1M", "-m", "17", "--psa-min", "13", "-k", "31", "-l", ul, "-B", "15", "--max-count", "5000",
                 "--stretch-cap", "10000", "-t", str(a.threads), "-r", sr, "-p", pb, "--timing"]
        out = {}
        wall, t = _run([os.path.join(ROOT, "pacbio_amd", "bin", "jf_aligner"), *flags, "-f", "--coords",
                        os.path.join(d, "coords")])
        out["jf_aligner"] = dict(process_wall_s=wall, **t)
        os.unlink(os.path.join(d, "coords"))
        wall, t = _run([os.path.join(ROOT, "pacbio_amd", "bin", "create_mega_reads"), *flags, "-o",
                        os.path.join(d, "mega_reads")])
        out["create_mega_reads"] = dict(process_wall_s=wall, **t)
        mr = open(os.path.join(d, "mega_reads")).read()
        out["create_mega_reads"]["reads_with_mega_reads"] = mr.count(">")
        out["create_mega_reads"]["mega_reads"] = mr.count("\n") - mr.count(">")
        out["create_mega_reads"]["bases_per_s"] = t["bases"] / t["wall_s"]
        out["create_mega_reads"]["graph"] = "device traversal (default)"
        # the same run with the overlap graph traversed on the host: same bytes
        wall, t = _run([os.path.join(ROOT, "pacbio_amd", "bin", "create_mega_reads"), *flags, "--host-graph", "-o",
                        os.path.join(d, "mega_reads_host")])
        out["create_mega_reads_host_graph"] = dict(process_wall_s=wall, **t, bases_per_s=t["bases"] / t["wall_s"])
        out["create_mega_reads_host_graph"]["identical_output"] = open(os.path.join(d, "mega_reads_host")).read() == mr
        out["workload"] = f"C2: {a.reads} PB reads vs 200k SRs, production flags, -t {a.threads}"
        print(json.dumps(out))
    finally:
        shutil.rmtree(d, ignore_errors=True)


if __name__ == "__main__":
    main()
