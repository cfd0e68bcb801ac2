#!/bin/bash
# r03m: cut keys of the MSM bucket pass resolved inside the wave through LDS; 16 hardware queues in bench.py.
# GPU tests, then quicknet / G2 unchained / 131k shard benches.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
T=${1:-r03m}
B="--no-cpu-baseline --single-call-steps 0"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > "$O/gpu_tests_$T.log" 2>&1
timeout -k 10 300 python bench.py $B > "$O/bench_$T.json" 2> "$O/bench_$T.err"
timeout -k 10 300 python bench.py --scheme pedersen-bls-unchained $B > "$O/bench_unch_$T.json" 2>> "$O/bench_$T.err"
timeout -k 10 200 python bench.py --total-rounds 131072 $B > "$O/shard131k_$T.json" 2>> "$O/bench_$T.err"
timeout -k 10 200 python bench.py --total-rounds 131072 --hw-queues 0 $B > "$O/shard131k_q4_$T.json" 2>> "$O/bench_$T.err"
echo "done $T"
