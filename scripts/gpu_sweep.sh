# parity tests selected by $TESTK, then profile_eval.py over the ';'-separated $CFGS
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/sweep
stop_if_fatal() { if [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; then echo "fatal rc=$1 at $2"; exit "$1"; fi; }
if [ -n "${TESTK:-}" ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "$TESTK" > gpurun_out/sweep/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/sweep/pytest.log; stop_if_fatal $rc pytest
[ $rc -ne 0 ] && exit $rc
fi
IFS=";" read -r -a cfgs <<< "${CFGS:-}"
for cfg in "${cfgs[@]}"; do
  timeout -k 10 300 python scripts/profile_eval.py --evals 20 $cfg > gpurun_out/sweep/eval.log 2>&1
  rc=$?; sed 's/costs.*//; s/libhq.so size=4096 K=256 P=4 grid=32 variant=0//' gpurun_out/sweep/eval.log; stop_if_fatal $rc eval
done
exit 0
