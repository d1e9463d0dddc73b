"""Summary of the round-6 C4 profile (tools/r06/prof.sh: bench.py --only c4 under rocprofv3):
per aligner kernel, launches and mean duration (kernel trace), FETCH_SIZE / WRITE_SIZE per
launch (separate PMC passes, KiB), HBM traffic = 2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md,
gfx950: 128-B read requests tallied at 64 B; k_group's gather shape calibrated to the same
factor) and the rate it moved at; then the C4 leg's own bench object.

python3 tools/r06/c4_summary.py gpurun_out/prof_TAG TAG  ->  profiles/TAG_c4_{kernel_stats.txt,rocprof_summary.json}
"""
import collections
import csv
import json
import os
import re
import sys

KERNELS = re.compile(r"k_seed|k_group|k_lis|k_coords|k_rec|k_len_perm|k_init_slen|k_order")


def short(name):
    n = name.split("(")[0].replace("void ", "").replace("pbgpu::", "")
    return n


def counters(path, cname):
    per = collections.defaultdict(list)
    if not os.path.exists(path):
        return per
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != cname:
                continue
            per[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return per


def main():
    d, tag = sys.argv[1], sys.argv[2]
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "..", "profiles")
    out = os.path.normpath(out)
    stats = {}
    with open(os.path.join(d, "c4_kt", "run_kernel_stats.csv")) as f:
        for r in csv.DictReader(f):
            n = short(r["Name"])
            if KERNELS.search(n):
                stats[n] = {"launches": int(r["Calls"]), "total_ms": float(r["TotalDurationNs"]) / 1e6,
                            "mean_ms": float(r["AverageNs"]) / 1e6}
    fetch = counters(os.path.join(d, "c4_FETCH_SIZE", "run_counter_collection.csv"), "FETCH_SIZE")
    write = counters(os.path.join(d, "c4_WRITE_SIZE", "run_counter_collection.csv"), "WRITE_SIZE")
    rows = []
    for n, s in sorted(stats.items(), key=lambda x: -x[1]["total_ms"]):
        fk = sum(fetch.get(n, [])) / max(1, len(fetch.get(n, []))) if fetch.get(n) else None
        wk = sum(write.get(n, [])) / max(1, len(write.get(n, []))) if write.get(n) else None
        e = dict(s)
        if fk is not None and wk is not None:
            traffic = (2 * fk + wk) * 1024.0
            e.update({"fetch_kib_per_launch": fk, "write_kib_per_launch": wk, "traffic_bytes_per_launch": traffic,
                      "traffic_gbs": traffic / (s["mean_ms"] * 1e-3) / 1e9 if s["mean_ms"] else None})
        rows.append((n, e))
    leg = None
    try:
        leg = json.load(open(os.path.join(d, "c4.json"))).get("c4")
    except (OSError, ValueError):
        pass
    js = {"source": f"tools/r06/prof.sh {tag}: bench.py --only c4 --c4-reads 100000 --device-steps 1 under rocprofv3 "
                    "(kernel trace; FETCH_SIZE and WRITE_SIZE in separate passes)",
          "traffic_formula": "2 x FETCH_SIZE + WRITE_SIZE (KiB)", "kernels": dict(rows), "c4_leg": leg}
    with open(os.path.join(out, f"{tag}_c4_rocprof_summary.json"), "w") as f:
        json.dump(js, f, indent=1)
    with open(os.path.join(out, f"{tag}_c4_kernel_stats.txt"), "w") as f:
        f.write(f"# {js['source']}\n# traffic = {js['traffic_formula']} per launch, rate = traffic / mean duration\n")
        for n, e in rows:
            t = e.get("traffic_bytes_per_launch")
            f.write(f"{n[:44]:44s} n={e['launches']:5d} total={e['total_ms']:10.3f} ms mean={e['mean_ms']:8.3f} ms"
                    + (f" traffic={t / 1e9:8.3f} GB/launch rate={e['traffic_gbs']:7.0f} GB/s" if t else "") + "\n")
        if leg:
            f.write("# C4 leg: value_device %.4g bases/s, stages (ms a step) %s\n"
                    % (leg.get("value_device") or 0, json.dumps(leg.get("stage_ms_per_step"))))
    print(open(os.path.join(out, f"{tag}_c4_kernel_stats.txt")).read())


if __name__ == "__main__":
    main()
