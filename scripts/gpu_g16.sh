# (1) HB = 15 at 4 workgroups per CU ((y, z) table in plane 2, 126 VGPRs) vs 3
# (lb3); (2) cost16w tile total by LDS integer atomics without the closing
# barrier (tsum). GPU suite on the default and on tsum, then A/B.
set -u
export TMPDIR=/tmp
O=gpurun_out/g16; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
HQ_LIB_PATH=hybridquantization_amd/libhq_tsum.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "golden or config3 or pixel or geometry or bitwise or device" > $O/pytest_tsum.log 2>&1 || { echo "tsum tests failed"; tail -30 $O/pytest_tsum.log; exit 1; }
tail -1 $O/pytest_tsum.log
for rep in 1 2; do
for L in libhq.so libhq_lb3.so; do
  HQ_LIB_PATH=hybridquantization_amd/$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-full-search --dpi 150 --distance 30 > $O/d150_$L.$rep.json 2>> $O/err || exit $?
  python3 -c "import json; d=json.load(open('$O/d150_$L.$rep.json')); print('$L d150', d['ms_per_step'], d['kernel_avg_ms'])"
done
for L in libhq.so libhq_tsum.so; do
  for cfg in "c3:" "d96:--dpi 96 --distance 60" "sh8:--shard-of 8 --steps 200"; do
    n=${cfg%%:*}; a=${cfg#*:}
    HQ_LIB_PATH=hybridquantization_amd/$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-full-search $a > $O/${n}_$L.$rep.json 2>> $O/err || exit $?
    python3 -c "import json; d=json.load(open('$O/${n}_$L.$rep.json')); print('$L', '$n', d['ms_per_step'], d['kernel_avg_ms'])"
  done
done
done
# (3) HB = 24 (200 dpi / 30 cm, halfSize 20) at 3 waves per SIMD (92 B spill) vs 2
for rep in 1 2; do
for L in libhq.so libhq_lb24.so; do
  HQ_LIB_PATH=hybridquantization_amd/$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-full-search --dpi 200 --distance 30 > $O/d200_$L.$rep.json 2>> $O/err || exit $?
  python3 -c "import json; d=json.load(open('$O/d200_$L.$rep.json')); print('$L d200', d['ms_per_step'], d['kernel_avg_ms'], d['roofline']['tap_bucket'])"
done
done
