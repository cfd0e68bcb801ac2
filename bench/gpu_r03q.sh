#!/bin/bash
# r03q: the sigma half of the level-0 MSM queued on the tail stream as soon as the signatures are decoded. GPU tests,
# quicknet bench with the one-call legs, G2 bench with the one-call legs, 131k shard.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
T=${1:-r03q}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > "$O/gpu_tests_$T.log" 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > "$O/bench_$T.json" 2> "$O/bench_$T.err"
timeout -k 10 300 python bench.py --scheme pedersen-bls-unchained --no-cpu-baseline > "$O/bench_unch_$T.json" 2>> "$O/bench_$T.err"
timeout -k 10 200 python bench.py --total-rounds 131072 --no-cpu-baseline --single-call-steps 0 > "$O/shard131k_$T.json" 2>> "$O/bench_$T.err"
echo "done $T"
