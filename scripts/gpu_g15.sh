# cost16w pair layout above HB = 10, no channel split: full GPU suite; then the
# horizontal chunk sizes at HB = 19 (CH19 6 default, 8, 13) and HB = 15 (CHW 8
# default, 6, 12)
set -u
export TMPDIR=/tmp
O=gpurun_out/g15; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
for L in libhq_prev.so libhq.so libhq_ch8.so libhq_ch13.so; do
  HQ_LIB_PATH=hybridquantization_amd/$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-full-search --dpi 96 --distance 60 > $O/d96_$L.$rep.json 2>> $O/err || exit $?
  python3 -c "import json; d=json.load(open('$O/d96_$L.$rep.json')); print('$L d96', d['ms_per_step'], d['kernel_avg_ms'])"
done
for L in libhq_prev.so libhq.so libhq_chw6.so libhq_chw12.so; do
  HQ_LIB_PATH=hybridquantization_amd/$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-full-search --dpi 150 --distance 30 > $O/d150_$L.$rep.json 2>> $O/err || exit $?
  python3 -c "import json; d=json.load(open('$O/d150_$L.$rep.json')); print('$L d150', d['ms_per_step'], d['kernel_avg_ms'])"
done
HQ_LIB_PATH=hybridquantization_amd/libhq.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-full-search > $O/c3.$rep.json 2>> $O/err || exit $?
python3 -c "import json; d=json.load(open('$O/c3.$rep.json')); print('libhq.so c3', d['ms_per_step'], d['kernel_avg_ms'])"
done
