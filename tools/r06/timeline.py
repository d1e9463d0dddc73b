"""Timeline of a rocprofv3 kernel trace (csv): the window from the first k_seed to the
last kernel, union busy time, per-stream busy time, the largest idle gaps (with the
kernels either side) and kernel totals inside the window.

python3 tools/r06/timeline.py run_kernel_trace.csv [--gap-ms 0.3] [--top 25]
"""
import argparse
import collections
import csv


def short(name):
    n = name.split("(")[0]
    return n.replace("void ", "").replace("pbgpu::", "")[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--gap-ms", type=float, default=0.3)
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--start", default="k_seed", help="the window opens at this kernel's first launch")
    ap.add_argument("--last", action="store_true", help="... at its last launch instead")
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                         r.get("Queue_Id"), r.get("Stream_Id")))
    rows.sort()
    starts = [s for s, _, n, _, _ in rows if a.start in n] or [rows[0][0]]
    t0 = starts[-1] if a.last else starts[0]
    rows = [r for r in rows if r[0] >= t0]
    t1 = max(e for _, e, _, _, _ in rows)
    print(f"window {(t1 - t0) / 1e6:.2f} ms, {len(rows)} kernels (from the first {a.start})")
    busy, cur_s, cur_e, gaps = 0, None, None, []
    prev = None
    for s, e, n, q, st in rows:
        if cur_e is None:
            cur_s, cur_e = s, e
        elif s > cur_e:
            busy += cur_e - cur_s
            if s - cur_e > a.gap_ms * 1e6:
                gaps.append(((s - cur_e) / 1e6, (cur_e - t0) / 1e6, prev, n))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        prev = n if cur_e == e or prev is None else prev
        if e >= cur_e:
            prev = n
    busy += cur_e - cur_s
    print(f"busy (any kernel running) {busy / 1e6:.2f} ms = {busy / (t1 - t0):.3f} of the window; "
          f"idle {(t1 - t0 - busy) / 1e6:.2f} ms")
    per_q = collections.defaultdict(int)
    for s, e, n, q, st in rows:
        per_q[(q, st)] += e - s
    for k, v in sorted(per_q.items()):
        print(f"  queue {k[0]} stream {k[1]}: kernel time {v / 1e6:.2f} ms")
    gaps.sort(reverse=True)
    print(f"idle gaps > {a.gap_ms} ms: {len(gaps)}, total {sum(g[0] for g in gaps):.2f} ms")
    for g, at, before, after in gaps[:15]:
        print(f"  {g:7.2f} ms at +{at:8.2f} ms  after {before}  before {after}")
    tot = collections.defaultdict(lambda: [0, 0])
    for s, e, n, q, st in rows:
        tot[n][0] += 1
        tot[n][1] += e - s
    print("kernels in the window (calls, total ms, mean ms):")
    for n, (c, t) in sorted(tot.items(), key=lambda x: -x[1][1])[:a.top]:
        print(f"  {n:70s} {c:6d} {t / 1e6:9.2f} {t / c / 1e6:8.3f}")


if __name__ == "__main__":
    main()
