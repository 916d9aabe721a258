# cost16w: pair layout above HB = 10 (32-row layout kept at 10): viewing-geometry
# and pixel tests, then A/B against the previous build at C3, 96/60, 150/30, and
# the HB = 19 channel split on/off (nosplit)
set -u
export TMPDIR=/tmp
O=gpurun_out/g14; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "geometry or pixel or golden or config3 or fast" > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
HQ_LIB_PATH=hybridquantization_amd/libhq_nosplit.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "geometry or pixel" > $O/pytest_nosplit.log 2>&1 || { echo "nosplit tests failed"; tail -30 $O/pytest_nosplit.log; exit 1; }
tail -1 $O/pytest_nosplit.log
for rep in 1 2; do
for L in libhq_prev.so libhq.so libhq_nosplit.so; do
  for cfg in "c3:" "d96:--dpi 96 --distance 60" "d150:--dpi 150 --distance 30"; do
    n=${cfg%%:*}; a=${cfg#*:}
    HQ_LIB_PATH=hybridquantization_amd/$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-full-search $a > $O/${n}_$L.$rep.json 2>> $O/err || exit $?
    python3 -c "import json; d=json.load(open('$O/${n}_$L.$rep.json')); print('$L', '$n', d['ms_per_step'], d['kernel_avg_ms'])"
  done
done
done
