#!/bin/bash
# Secondary BASELINE configs after the r02 arithmetic changes (one GPU call; each step with its own limit).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python bench/bench_configs.py unchained --streams 8 > "$O/cfg_unchained_r02w.json" 2> "$O/cfg_unchained_r02w.err"
timeout -k 10 400 python bench/bench_configs.py chained --rounds 4194304 --streams 4 --chain-cache /tmp/dh_chain > "$O/cfg_chained_r02w.json" 2> "$O/cfg_chained_r02w.err"
timeout -k 10 300 python bench/bench_configs.py recover > "$O/cfg_recover_r02w.json" 2> "$O/cfg_recover_r02w.err"
echo configs done
