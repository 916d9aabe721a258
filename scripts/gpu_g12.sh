# A/B on the shard-of-8 step and C2/C3: used colours as bytes (flushed by one wave)
# vs bits
set -u
export TMPDIR=/tmp
O=gpurun_out/g12; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "assign or config3 or golden or chunked or used or pixel or shard" > $O/pytest.log 2>&1 || { echo "tests failed"; tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
for L in libhq.so libhq_ub0.so; do
  HQ_LIB_PATH=hybridquantization_amd/$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-full-search --shard-of 8 --steps 200 > $O/shard8_$L.$rep.json 2>> $O/err || exit $?
  HQ_LIB_PATH=hybridquantization_amd/$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-full-search --size 1024 --K 64 --population 1 --steps 200 > $O/c2_$L.$rep.json 2>> $O/err || exit $?
  HQ_LIB_PATH=hybridquantization_amd/$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-full-search --steps 100 > $O/c3_$L.$rep.json 2>> $O/err || exit $?
  python3 -c "
import json
for c in ('shard8','c2','c3'):
    d=json.load(open('$O/'+c+'_$L.$rep.json')); print('$L', c, d['ms_per_step'], d['kernel_avg_ms'])"
done
done
