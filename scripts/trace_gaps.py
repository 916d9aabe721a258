"""Per-kernel durations and the idle gaps between consecutive kernels from a
rocprofv3 --kernel-trace CSV (one stream).  Usage:
    python scripts/trace_gaps.py path/to/run_kernel_trace.csv [--last N]
--last N: only the last N kernels (e.g. the timed steps at the end of a bench run)."""

import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--last", type=int, default=0)
    args = ap.parse_args()
    rows = []
    with open(args.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    if args.last:
        rows = rows[-args.last:]
    dur = defaultdict(list)
    gap_after = defaultdict(list)
    for i, (s, e, name) in enumerate(rows):
        short = name.split("(")[0].replace("void ", "").split("<")[0]
        dur[short].append((e - s) / 1e3)
        if i + 1 < len(rows):
            gap_after[short].append((rows[i + 1][0] - e) / 1e3)
    span = (rows[-1][1] - rows[0][0]) / 1e3
    busy = sum(sum(v) for v in dur.values())
    print(f"{len(rows)} kernels, span {span:.1f} us, busy {busy:.1f} us, idle {span - busy:.1f} us")
    for k in sorted(dur, key=lambda k: -sum(dur[k])):
        d, g = dur[k], gap_after[k]
        print(f"{k:40s} n={len(d):5d} avg {sum(d) / len(d):8.2f} us   gap after avg "
              f"{(sum(g) / len(g) if g else 0):6.2f} us")


if __name__ == "__main__":
    main()
