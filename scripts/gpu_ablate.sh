# Time the ablation builds of scripts/ablate.py (no tests; timing only).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/ablate
for v in ${VARIANTS:-base novfma nohfma nogather nolab base}; do
  timeout -k 10 200 python scripts/profile_eval.py --evals 20 --lib build_exp/libhq_$v.so ${ARGS:-} > gpurun_out/ablate/$v.log 2>&1
  rc=$?; cut -c1-200 gpurun_out/ablate/$v.log | tail -1
  if [ $rc -ne 0 ]; then echo "rc=$rc at $v"; exit $rc; fi
done
exit 0
