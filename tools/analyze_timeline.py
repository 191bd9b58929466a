"""GPU timeline of a rocprofv3 --kernel-trace run (round 6: the config-5 step eager vs replayed from a hipGraph).

    python tools/analyze_timeline.py <trace_dir> [--tail FRACTION]

Over the last FRACTION of the dispatches (default 0.5: past warm-up and capture): the span, the union of the kernels'
busy intervals (time with at least one kernel running), the summed kernel time (> union when kernels overlap), the
idle time between kernels split by gap length, and the average concurrency."""
import argparse
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--tail", type=float, default=0.5)
    a = ap.parse_args()
    rows = []
    for f in glob.glob(os.path.join(a.root, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    rows = rows[int(len(rows) * (1 - a.tail)):]
    span = rows[-1][1] - rows[0][0]
    busy, gaps = 0, []
    cs, ce = rows[0][0], rows[0][1]
    for s, e, _ in rows[1:]:
        if s > ce:
            busy += ce - cs
            gaps.append(s - ce)
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    tot = sum(e - s for s, e, _ in rows)
    print(f"{len(rows)} dispatches over {span / 1e6:.2f} ms: busy (union) {busy / 1e6:.2f} ms = {busy / span:.3f} of the span, "
          f"summed kernel time {tot / 1e6:.2f} ms (average concurrency while busy {tot / busy:.2f})")
    for lo, hi in ((0, 2e3), (2e3, 5e3), (5e3, 2e4), (2e4, 1e12)):
        g = [x for x in gaps if lo <= x < hi]
        print(f"  gaps {lo / 1e3:5.0f}-{hi / 1e3 if hi < 1e12 else float('inf'):5.0f} us: {len(g):6d}, "
              f"{sum(g) / 1e6:7.2f} ms")


if __name__ == "__main__":
    main()
