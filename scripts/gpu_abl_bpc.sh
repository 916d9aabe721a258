set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/ablate
run() { timeout -k 10 200 python scripts/profile_eval.py --evals 20 --lib build_exp/libhq_$1.so --bpc $2 > gpurun_out/ablate/x.log 2>&1; rc=$?; echo "$1 bpc=$2 $(grep -o 'assign=[0-9.]*ms' gpurun_out/ablate/x.log)"; return $rc; }
run base 8 && run base 5 && run base 10 && run a_lb8 8 && run a_lb8 16 && run a_lb6 6 && run a_lb6 12 && run base 8 && run a_lb8 8 && run a_lb6 6
