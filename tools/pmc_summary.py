#!/usr/bin/env python3
"""Summarise a tools/pmc_run.sh collection: per kernel, launches, mean
duration (kernel trace), and per-launch PMC counters.  HBM traffic per launch
follows MI355X_MICROARCH.md "HBM [CDNA4]": 2 x FETCH_SIZE (gfx950 tallies
128-B read requests at 64 B) + WRITE_SIZE, both reported in KiB.

  python tools/pmc_summary.py gpurun_out/pmc [--json-out profiles/]
writes pmc_<kernel>.json (hbm_bytes_per_launch, counters) for bench.py.
"""
import argparse
import collections
import csv
import json
import os
import re


def short(name):
    m = re.match(r"(?:void )?(?:pbgpu::)?([A-Za-z_0-9]+)(<[^(]*>)?", name)
    base = m.group(1) if m else name
    tmpl = m.group(2) if m and m.group(2) else ""
    return base + tmpl


def fname(k):
    """file-name form of a (template) kernel name: k_group<false, 256u> -> k_group_false_256u"""
    return re.sub(r"[^A-Za-z0-9]+", "_", k).strip("_")


def load_trace(d):
    p = os.path.join(d, "kt", "run_kernel_trace.csv")
    out = collections.defaultdict(list)
    with open(p) as f:
        for r in csv.DictReader(f):
            out[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
    return out


def load_counters(d):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(lambda: collections.defaultdict(set))
    for sub in sorted(os.listdir(d)):
        p = os.path.join(d, sub, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        with open(p) as f:
            for r in csv.DictReader(f):
                k = short(r["Kernel_Name"])
                c = r["Counter_Name"]
                acc[k][c] += float(r["Counter_Value"])
                disp[k][c].add(r["Dispatch_Id"])
    per = {}
    for k, cs in acc.items():
        per[k] = {c: v / max(1, len(disp[k][c])) for c, v in cs.items()}
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args()
    tr = load_trace(a.dir)
    pc = load_counters(a.dir)
    rows = []
    for k, ds in sorted(tr.items(), key=lambda kv: -sum(kv[1])):
        c = pc.get(k, {})
        hbm = None
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            hbm = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0
        mean = sum(ds) / len(ds)
        rows.append((k, len(ds), sum(ds), mean, hbm, c))
        print(f"{k:40s} n={len(ds):4d} total={sum(ds):9.3f} ms mean={mean:8.3f} ms"
              + (f" hbm/launch={hbm / 1e9:8.3f} GB ({hbm / (mean * 1e-3) / 1e9:7.1f} GB/s)" if hbm else ""))
        for cn in sorted(c):
            print(f"    {cn:28s} {c[cn]:.4g}")
        if a.json_out and hbm is not None:
            os.makedirs(a.json_out, exist_ok=True)
            with open(os.path.join(a.json_out, f"pmc_{fname(k)}.json"), "w") as f:
                json.dump({"kernel": k, "launches": len(ds), "mean_ms": mean, "hbm_bytes_per_launch": hbm,
                           "hbm_formula": "2*FETCH_SIZE + WRITE_SIZE (KiB -> B), MI355X_MICROARCH.md HBM [CDNA4]",
                           "counters_per_launch": c}, f, indent=1)


if __name__ == "__main__":
    main()
