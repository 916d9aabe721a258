# sa_step phase stamps (-DHQ_SA_TIMING build, libhq_sat.so) on the shard-of-8 bench loop
set -u
mkdir -p gpurun_out/sat
HQ_LIB_PATH=hybridquantization_amd/libhq_sat.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-full-search --shard-of 8 --steps 20 > gpurun_out/sat/sat.json 2> gpurun_out/sat/sat.err
