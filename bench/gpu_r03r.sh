#!/bin/bash
# r03r: bucket pass loads the next entry's affine point one addition ahead; k_lagrange (G2) on the lazy 28-bit chain.
# GPU tests; quicknet, G2 and 131k benches; tbls Recover config.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
T=${1:-r03r}
B="--no-cpu-baseline --single-call-steps 0"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > "$O/gpu_tests_$T.log" 2>&1
timeout -k 10 300 python bench.py $B > "$O/bench_$T.json" 2> "$O/bench_$T.err"
timeout -k 10 300 python bench.py --scheme pedersen-bls-unchained $B > "$O/bench_unch_$T.json" 2>> "$O/bench_$T.err"
timeout -k 10 200 python bench.py --total-rounds 131072 $B > "$O/shard131k_$T.json" 2>> "$O/bench_$T.err"
timeout -k 10 300 python bench/bench_configs.py recover > "$O/cfg_recover_$T.json" 2> "$O/cfg_recover_$T.err"
echo "done $T"
