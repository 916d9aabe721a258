# banded assign/cost pipeline: parity tests, then an eval-time sweep over bands / chunks per block
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/bands
stop_if_fatal() { if [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; then echo "fatal rc=$1 at $2"; exit "$1"; fi; }
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "banded or shards or full_size or golden" > gpurun_out/bands/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/bands/pytest.log; stop_if_fatal $rc pytest
[ $rc -ne 0 ] && exit $rc
for cfg in ${CFGS:-"0:2" "2:2" "4:2" "8:2" "8:1" "8:4" "16:1" "16:2"}; do
  b=${cfg%%:*}; c=${cfg##*:}
  timeout -k 10 300 python scripts/profile_eval.py --evals 20 --bands $b --cpb $c > gpurun_out/bands/eval.log 2>&1
  rc=$?; cut -c1-400 gpurun_out/bands/eval.log | grep -v "^$" | sed 's/costs.*//'; stop_if_fatal $rc eval
done
exit 0
