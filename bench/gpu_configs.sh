#!/bin/bash
# Secondary BASELINE configs on a given build (tag = first argument) (one GPU call; each step with its own limit).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
T=${1:-r02x}
timeout -k 10 300 python bench/bench_configs.py unchained --streams 8 > "$O/cfg_unchained_${T}.json" 2> "$O/cfg_unchained_${T}.err"
timeout -k 10 400 python bench/bench_configs.py chained --rounds 4194304 --streams 4 --chain-cache /tmp/dh_chain > "$O/cfg_chained_${T}.json" 2> "$O/cfg_chained_${T}.err"
timeout -k 10 300 python bench/bench_configs.py recover > "$O/cfg_recover_${T}.json" 2> "$O/cfg_recover_${T}.err"
echo configs done
