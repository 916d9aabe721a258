# PMC passes (issue/LDS/wait counters) for two cost_tile configurations.
set -u
export TMPDIR=/tmp
CFGS="${CFGS:---tile 6;--tile 7}" bash scripts/gpu_pmc.sh
