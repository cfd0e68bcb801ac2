#!/bin/bash
# r03j: 131k-shard experiments: hardware queues per process (head-of-line blocking of latency-bound tails), level-0
# window width and the bucket pass's shortest chunk; 1M with more hardware queues.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
T=${1:-r03j}
B="--no-cpu-baseline --single-call-steps 0"
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --total-rounds 131072 $B > "$O/s131k_${T}_$tag.json" 2>> "$O/s131k_$T.err"
}
run base X=0
run q8 GPU_MAX_HW_QUEUES=8
run q16 GPU_MAX_HW_QUEUES=16
run c13 DRANDHIP_MSM_C=13
run c13l16 DRANDHIP_MSM_C=13 DRANDHIP_MSM_LMIN=16
run l8 DRANDHIP_MSM_LMIN=8
GPU_MAX_HW_QUEUES=16 timeout -k 10 200 python bench.py --total-rounds 131072 --streams 16 $B > "$O/s131k_${T}_q16s16.json" 2>> "$O/s131k_$T.err"
timeout -k 10 300 python bench.py $B > "$O/b1m_${T}_base.json" 2>> "$O/b1m_$T.err"
GPU_MAX_HW_QUEUES=16 timeout -k 10 300 python bench.py $B > "$O/b1m_${T}_q16.json" 2>> "$O/b1m_$T.err"
echo "done $T"
