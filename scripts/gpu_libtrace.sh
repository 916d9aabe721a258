# Same-box kernel-trace A/B of library builds ($LIBS under hybridquantization_amd/):
# rocprofv3 --kernel-trace --stats of bench.py ($BENCH_ARGS) per build, twice.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/libtrace
for rep in 1 2; do
  for L in $LIBS; do
    HQ_LIB_PATH=hybridquantization_amd/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/libtrace/$L.$rep -o run -- python3 bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/libtrace/$L.$rep.json 2> gpurun_out/libtrace/$L.$rep.err || { echo "$L rc=$?"; tail -3 gpurun_out/libtrace/$L.$rep.err; exit 1; }
    python3 - "$L" "$rep" <<'PY'
import csv, glob, sys
L, rep = sys.argv[1], sys.argv[2]
f = glob.glob(f"gpurun_out/libtrace/{L}.{rep}/**/run_kernel_stats.csv", recursive=True)[0]
print(L, rep, {r["Name"].split("(")[0].replace("void ", "")[:24]: round(float(r["AverageNs"]) / 1e3, 2)
               for r in csv.DictReader(open(f)) if float(r["Percentage"]) > 0.5})
PY
  done
done
