#!/bin/bash
# r03p: tbls Recover config (n = 64, t = 33, 100k rounds) on the r03 build; chained 4M replay with the one-lane pairing
# path for group checks and leaves (DRANDHIP_LANE_PAIRING=1) against the VM, one stream and 4 streams.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
T=${1:-r03p}
C=/tmp/drandhip_chain_cache
timeout -k 10 300 python bench/bench_configs.py recover > "$O/cfg_recover_$T.json" 2> "$O/cfg_recover_$T.err"
timeout -k 10 500 python bench/bench_configs.py chained --rounds 4194304 --window 1048576 --streams 1 --steps 1 \
  --chain-cache $C > "$O/chained4m_s1_vm_$T.json" 2> "$O/chained4m_$T.err"
DRANDHIP_LANE_PAIRING=1 timeout -k 10 300 python bench/bench_configs.py chained --rounds 4194304 --window 1048576 --streams 1 \
  --steps 1 --chain-cache $C > "$O/chained4m_s1_lane_$T.json" 2>> "$O/chained4m_$T.err"
DRANDHIP_LANE_PAIRING=1 timeout -k 10 300 python bench/bench_configs.py chained --rounds 4194304 --window 1048576 --streams 4 \
  --steps 2 --chain-cache $C > "$O/chained4m_lane_$T.json" 2>> "$O/chained4m_$T.err"
echo "done $T"
