#!/bin/bash
# r03c: the 28-bit G1 MSM: GPU tests, the headline bench, the 131k shard; then product counts + G2 PMC (r03b)
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
T=${1:-r03c}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > "$O/gpu_tests_$T.log" 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > "$O/bench_$T.json" 2> "$O/bench_$T.err"
timeout -k 10 200 python bench.py --total-rounds 131072 --no-cpu-baseline --single-call-steps 0 > "$O/shard131k_$T.json" 2> "$O/shard131k_$T.err"
bash bench/gpu_r03b.sh r03b
echo "done $T"
