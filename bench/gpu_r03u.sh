#!/bin/bash
# r03u: no-carry Fp2 product operands only in the G2 subgroup test (opt-in NC template flag); after a dense
# batch the bisection runs 256 -> 32 -> 4 -> leaves. GPU tests, G2 + quicknet benches, chained 4M (4 streams, 1 stream).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
T=${1:-r03u}
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
