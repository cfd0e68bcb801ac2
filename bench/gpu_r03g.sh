#!/bin/bash
# r03g: cost-model MSM windows, lazy G2 cofactor clearing in the VM prep, G2 subgroup kernel occupancy 1 vs 2,
# 64-entry G2 chunks: tests, benches, 131k shard, chained 4M replay (4 x 1M on 4 streams, 8 x 512k on 8 streams)
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
T=${1:-r03g}
C=/tmp/drandhip_chain_cache
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > "$O/gpu_tests_$T.log" 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --single-call-steps 0 > "$O/bench_$T.json" 2> "$O/bench_$T.err"
timeout -k 10 300 python bench.py --scheme pedersen-bls-unchained --no-cpu-baseline --single-call-steps 0 > "$O/bench_unch_$T.json" 2> "$O/bench_unch_$T.err"
DRANDHIP_SUBG2_OCC=2 timeout -k 10 300 python bench.py --scheme pedersen-bls-unchained --no-cpu-baseline --single-call-steps 0 \
  > "$O/bench_unch_occ2_$T.json" 2> "$O/bench_unch_occ2_$T.err"
timeout -k 10 200 python bench.py --total-rounds 131072 --no-cpu-baseline --single-call-steps 0 > "$O/shard131k_$T.json" 2> "$O/shard131k_$T.err"
timeout -k 10 600 python bench/bench_configs.py chained --rounds 4194304 --window 1048576 --streams 4 --steps 2 \
  --chain-cache $C > "$O/chained4m_$T.json" 2> "$O/chained4m_$T.err"
timeout -k 10 300 python bench/bench_configs.py chained --rounds 4194304 --window 524288 --streams 8 --steps 2 \
  --chain-cache $C > "$O/chained4m_w512k_$T.json" 2>> "$O/chained4m_$T.err"
echo "done $T"
