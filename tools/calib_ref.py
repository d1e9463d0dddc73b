#!/usr/bin/env python3
"""The CPU baseline's speed against the reference itself (calibrate
the restatement on identical inputs in this container).  TEST INFRASTRUCTURE.

The reference's jf_aligner needs Jellyfish (absent), so the whole reference path
cannot run here; two of its components compile from their own sources
(oracle/Makefile `ref`) and are timed against the oracle's restatements on the
same inputs, one thread each:
  * lookup: PSA::search + the walk over every hit (find_pos_size + pos_iterator,
    superread_parser.hpp:110-192) against the oracle's hash lookup, for both
    strands of every 17-mer of the first --reads C2 reads, over the C2 super-reads;
  * lis: lis_align::indices with the production functors (affine_capped(1.3, 10,
    10000), linear(1.3), window 1) against oracle_lis, on the (read, super-read,
    strand) lists the oracle's --details prints for the same reads.
Then the oracle's whole path on those reads (align + format, one thread) is
timed, and the reference's is estimated by swapping the two measured
components' times in: t_ref ~= t_oracle - t_oracle(lookup + lis) + t_ref(lookup +
lis), every other part taken as equal.  Writes profiles/<name>.json.

  python tools/calib_ref.py --reads 200 --out r05_calib_ref
"""
import argparse
import json
import os
import platform
import struct
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

RC = bytes.maketrans(b"ACGT", b"TGCA")


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=200)
    ap.add_argument("--workload", default="C2")
    ap.add_argument("--out", default="r05_calib_ref")
    a = ap.parse_args()
    from oracle.oracle import OracleIndex, params
    from tools.synth import Dataset
    ref_bench = os.path.join(ROOT, "oracle", "_ref", "ref_bench")
    or_bench = os.path.join(ROOT, "oracle", "oracle_bench")
    for p in (ref_bench, or_bench):
        if not os.path.exists(p):
            raise SystemExit(f"{p} missing: make -C oracle all ref")
    wd = tempfile.mkdtemp(prefix="calib_ref_")
    ds = Dataset(a.workload, seed=42, threads=8, n_pb=a.reads)
    ds.write(wd)
    sr = os.path.join(wd, "sr.fa")
    seqs, names = ds.pb_seqs(), ds.pb_names()
    k = 17
    # ---- queries: both strands of every valid 17-mer of the reads
    qs = []
    for s in seqs:
        s = s.upper()
        for i in range(len(s) - k + 1):
            m = s[i:i + k]
            if m.strip(b"ACGT"):
                continue
            qs.append(m)
            qs.append(m.translate(RC)[::-1])
    qpath = os.path.join(wd, "queries.bin")
    with open(qpath, "wb") as f:
        f.write(struct.pack("<II", len(qs), k))
        f.write(b"".join(qs))
    # ---- strands: the oracle's --details lists (production flags), split by strand sign
    akw = dict(k=k, forward=True, unitigs_k=31, unitig_lengths=ds.unitig_lengths, bases_matching=15.0,
               max_count=5000, stretch_cap=10000.0)
    oix = OracleIndex.from_fasta([sr], k, threads=8)
    p = params(**akw)
    _, det = oix.align_format(p, names, seqs, threads=8, details=True)
    strands = []
    for line in det.splitlines():
        f, b = [], []
        for tok in line.split()[2:]:
            x, y = tok.strip("[]").split(":")
            (f if int(y) > 0 else b).append((int(x), int(y)))
        strands += [s for s in (f, b) if s]
    spath = os.path.join(wd, "strands.bin")
    with open(spath, "wb") as fo:
        fo.write(struct.pack("<I", len(strands)))
        for s in strands:
            fo.write(struct.pack("<I", len(s)))
            fo.write(b"".join(struct.pack("<ii", x, y) for x, y in s))
    # ---- the oracle's whole path on the reads, one thread (align + coords text)
    t0 = time.perf_counter()
    oix.align_format(p, names, seqs, threads=1)
    t_or_path = time.perf_counter() - t0
    oix.close()

    def run(cmd):
        r = subprocess.run(cmd, capture_output=True, text=True, check=True)
        return json.loads(r.stdout.strip().splitlines()[-1])

    ref_l = run([ref_bench, "psa", sr, "13", "17", "8", qpath])
    or_l = run([or_bench, "lookup", sr, str(k), qpath])
    ref_s = run([ref_bench, "lis", spath, "1.3", "10", "10000", "1"])
    or_s = run([or_bench, "lis", spath, "1.3", "10", "10000", "1"])
    assert ref_l["hits"] == or_l["hits"] and ref_l["checksum"] == or_l["checksum"], (ref_l, or_l)
    assert ref_s["lis_total"] == or_s["lis_total"], (ref_s, or_s)
    bases = sum(len(s) for s in seqs)
    t_ref_path = t_or_path - or_l["search_s"] - or_s["lis_s"] + ref_l["search_s"] + ref_s["lis_s"]
    out = {
        "what": "the oracle (CPU restatement) against the reference's own compiled components on identical inputs, "
                "one thread each (tools/calib_ref.py)",
        "cpu_model": _cpu_model(), "threads": 1,
        "inputs": {"workload": a.workload, "reads": a.reads, "bases": bases, "super_reads": len(ds.sr_names()),
                   "queries": len(qs), "strands": len(strands), "strand_elements": ref_s["elements"]},
        "lookup": {"reference_s": ref_l["search_s"], "oracle_s": or_l["search_s"],
                   "reference_over_oracle": ref_l["search_s"] / or_l["search_s"], "hits": ref_l["hits"],
                   "reference_build_s": ref_l["build_s"], "oracle_build_s": or_l["build_s"],
                   "note": "PSA::search + position walk (reference) vs the hash lookup (oracle); the same hits "
                           "and position checksum"},
        "lis": {"reference_s": ref_s["lis_s"], "oracle_s": or_s["lis_s"],
                "reference_over_oracle": ref_s["lis_s"] / or_s["lis_s"], "lis_total": ref_s["lis_total"],
                "note": "lis_align::indices vs oracle_lis; the same LIS lengths"},
        "path": {"oracle_s": t_or_path, "oracle_bases_per_s": bases / t_or_path,
                 "reference_estimate_s": t_ref_path, "reference_estimate_bases_per_s": bases / t_ref_path,
                 "ratio_vs_reference": t_ref_path / t_or_path,
                 "note": "reference estimate = the oracle's whole-path time with its lookup and LIS times replaced by "
                         "the reference's; every other component (filters, fit, kmers_info, formatting) taken equal. "
                         "ratio_vs_reference = reference time / oracle time (> 1: the oracle is faster)"},
    }
    dst = os.path.join(ROOT, "profiles", a.out + ".json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))
    ds.close()
    import shutil
    shutil.rmtree(wd, ignore_errors=True)


if __name__ == "__main__":
    main()
