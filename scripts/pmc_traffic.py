"""HBM bytes per launch from rocprofv3 FETCH_SIZE / WRITE_SIZE passes.

    python scripts/pmc_traffic.py FETCH_DIR WRITE_DIR OUT.json CONFIG_JSON

CONFIG_JSON names the profiled run ({"size": 4096, "K": 256, "P": 4, "grid": 32},
plus "dpi"/"distance" off the default geometry): bench.py's roofline.traffic
takes the newest file whose config matches its own run, so it is required.

FETCH_DIR / WRITE_DIR are the -d directories of two separate
`rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE` passes
(scripts/gpu_quick.sh pmc).  Both counters are in KiB.  On gfx950
FETCH_SIZE reports half the bytes of wide (16 B/lane) streaming reads
(MI355X_MICROARCH.md, "HBM"), so fetched bytes are doubled; WRITE_SIZE is
exact for 16 B/lane stores and uncalibrated for byte stores (the assign
kernel's index writes), which is recorded alongside.
"""
import collections
import csv
import glob
import json
import sys
import time


def per_kernel(d, counter):
    files = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    acc = collections.defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                name = r["Kernel_Name"].split("(")[0].replace("void ", "")
                acc[name].append(float(r["Counter_Value"]) * 1024.0)
    return {k: (sum(v) / len(v), len(v)) for k, v in acc.items()}


def main():
    fdir, wdir, out = sys.argv[1:4]
    if len(sys.argv) < 5:
        sys.exit("pmc_traffic.py: the config JSON is required (bench.py matches on it)")
    cfg = json.loads(sys.argv[4])
    for key in ("size", "K", "P", "grid"):
        if key not in cfg:
            sys.exit(f"pmc_traffic.py: config needs '{key}'")
    fetch = per_kernel(fdir, "FETCH_SIZE")
    write = per_kernel(wdir, "WRITE_SIZE")
    res = {"config": cfg, "generated": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()),
           "unit": "bytes per launch",
           "correction": "fetch_bytes = 2 x FETCH_SIZE (gfx950 wide-read tally); write as reported",
           "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        fb, fn = fetch.get(k, (0.0, 0))
        wb, wn = write.get(k, (0.0, 0))
        res["kernels"][k] = {"fetch_bytes": 2.0 * fb, "fetch_size_raw_bytes": fb,
                             "write_bytes": wb, "launches": [fn, wn],
                             "traffic_bytes": 2.0 * fb + wb}
    json.dump(res, open(out, "w"), indent=1)
    for k, v in res["kernels"].items():
        print(f"{k:40s} fetch {v['fetch_bytes'] / 1e6:9.1f} MB  write {v['write_bytes'] / 1e6:8.1f} MB")


if __name__ == "__main__":
    main()
