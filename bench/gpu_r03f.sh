#!/bin/bash
# r03f: chained replay (Cfg5) on the r03 build: one 1M window single-stream with ladder / pairing-path variants
# (stage times), then the 4M config on 4 streams. The signed chains are cached under /tmp for the call.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
T=${1:-r03f}
C=/tmp/drandhip_chain_cache
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 400 python bench/bench_configs.py chained --rounds 1048576 --window 1048576 --streams 1 --steps 2 \
    --cpu-sample 10 --cpu-threads 4 --chain-cache $C > "$O/chained1m_${T}_$tag.json" 2>> "$O/chained1m_$T.err"
}
run adaptive DRANDHIP_X=0
run lane DRANDHIP_LANE_PAIRING=1
run l64_4 DRANDHIP_BISECT=64,4
run l256_16_2 DRANDHIP_BISECT=256,16,2
timeout -k 10 600 python bench/bench_configs.py chained --rounds 4194304 --window 1048576 --streams 4 --steps 2 \
  --chain-cache $C > "$O/chained4m_$T.json" 2> "$O/chained4m_$T.err"
echo "done $T"
