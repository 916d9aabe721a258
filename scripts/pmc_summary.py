"""Per-kernel averages of rocprofv3 --pmc passes (scripts/gpu_pmc.sh layout).

    python scripts/pmc_summary.py gpurun_out/pmc/c1 [gpurun_out/pmc/c2 ...]
"""
import collections
import csv
import glob
import sys


def load(d):
    res = collections.defaultdict(dict)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        acc = collections.defaultdict(float)
        n = collections.defaultdict(set)
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:60]
            acc[(k, r["Counter_Name"])] += float(r["Counter_Value"])
            n[k].add(r["Dispatch_Id"])
        for (k, c), v in acc.items():
            res[k][c] = v / len(n[k])
    return res


def main():
    runs = [load(d) for d in sys.argv[1:]]
    kernels = sorted(set(k for r in runs for k in r))
    for k in kernels:
        print(k)
        ctrs = sorted(set(c for r in runs for c in r.get(k, {})))
        for c in ctrs:
            vals = "  ".join(f"{r.get(k, {}).get(c, float('nan')):12.4g}" for r in runs)
            print(f"   {c:28s} {vals}")


if __name__ == "__main__":
    main()
