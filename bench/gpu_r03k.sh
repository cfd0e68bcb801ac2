#!/bin/bash
# r03k: 131k shard with 16 hardware queues and the bucket pass's shortest chunk 8 / 12 / 16; 262k and 524k shards
# (the N = 4 / N = 2 per-GPU sizes) and 1M with the chosen setting.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
T=${1:-r03k}
B="--no-cpu-baseline --single-call-steps 0"
run() {  # tag, rounds, env...
  local tag=$1 n=$2; shift 2
  env GPU_MAX_HW_QUEUES=16 "$@" timeout -k 10 200 python bench.py --total-rounds $n $B > "$O/s${n}_${T}_$tag.json" 2>> "$O/s_$T.err"
}
run q16l4 131072 DRANDHIP_MSM_LMIN=4
run q16l8 131072 DRANDHIP_MSM_LMIN=8
run q16l12 131072 DRANDHIP_MSM_LMIN=12
run q16l16 131072 DRANDHIP_MSM_LMIN=16
run q16l4 262144 DRANDHIP_MSM_LMIN=4
run q16l8 262144 DRANDHIP_MSM_LMIN=8
run q16l4 524288 DRANDHIP_MSM_LMIN=4
run q16l8 524288 DRANDHIP_MSM_LMIN=8
run q16l8 1048576 DRANDHIP_MSM_LMIN=8
echo "done $T"
