#!/bin/bash
# Per-GPU rate at the shard sizes of the strong-scaling runs (1M rounds over N = 1, 2, 4, 8 GPUs), on one GPU.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/gpu_tests_r02y.log" 2>&1
for n in 131072 262144 524288 1048576; do
  timeout -k 10 200 python bench.py --total-rounds $n --no-cpu-baseline --single-call-steps 0 > "$O/shard_${n}_r02y.json" 2> "$O/shard_${n}_r02y.err"
done
echo shards done
