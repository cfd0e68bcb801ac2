#!/bin/bash
# r03t: Fp2 product operands without the carry pass (f28_add_nc / f28_sub_nc); the bisection's first level from the
# worker's fault-density hint (256-round groups after a dense batch). GPU tests, G2 + quicknet benches, chained 4M.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
T=${1:-r03t}
C=/tmp/drandhip_chain_cache
B="--no-cpu-baseline --single-call-steps 0"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > "$O/gpu_tests_$T.log" 2>&1
timeout -k 10 300 python bench.py --scheme pedersen-bls-unchained $B > "$O/bench_unch_$T.json" 2> "$O/bench_$T.err"
timeout -k 10 300 python bench.py $B > "$O/bench_$T.json" 2>> "$O/bench_$T.err"
timeout -k 10 600 python bench/bench_configs.py chained --rounds 4194304 --window 1048576 --streams 4 --steps 2 \
  --chain-cache $C > "$O/chained4m_$T.json" 2> "$O/chained4m_$T.err"
timeout -k 10 300 python bench/bench_configs.py chained --rounds 4194304 --window 1048576 --streams 1 --steps 1 \
  --chain-cache $C > "$O/chained4m_s1_$T.json" 2>> "$O/chained4m_$T.err"
echo "done $T"
