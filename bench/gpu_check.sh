#!/bin/bash
# GPU-box check used during development: Fp microbenchmark, GPU parity tests, smoke, default bench.
# Each GPU step has its own time limit; the first failure ends the script.
#   bash bench/gpu_check.sh <tag>
set -euo pipefail
TAG=${1:-dev}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 120 ./bench/microbench_fp > "$O/microbench_fp_$TAG.txt" 2>&1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$O/gpu_tests_$TAG.log" 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke_$TAG.log" 2>&1
timeout -k 10 300 python bench.py > "$O/bench_$TAG.json" 2> "$O/bench_$TAG.err"
echo "gpu_check $TAG done"
