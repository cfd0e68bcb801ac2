#!/bin/bash
# r03i: adaptive rounds-per-inversion in k_msm_prep28; headline + 131k shard benches, rocprofv3 kernel trace of the
# 131k shard, then the chained 4M replay (Cfg5) on the r03 build.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
T=${1:-r03i}
C=/tmp/drandhip_chain_cache
timeout -k 10 300 python bench.py --no-cpu-baseline --single-call-steps 2 > "$O/bench_$T.json" 2> "$O/bench_$T.err"
timeout -k 10 300 python bench.py --total-rounds 131072 --no-cpu-baseline --single-call-steps 0 > "$O/shard131k_$T.json" 2> "$O/shard131k_$T.err"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof131k_$T" -o run --output-format csv -- \
  python3 "$R/bench.py" --total-rounds 131072 --steps 8 --warmup 8 --single-call-steps 0 --no-cpu-baseline > "$O/prof131k_$T.log" 2>&1
cd "$R"
timeout -k 10 700 python bench/bench_configs.py chained --rounds 4194304 --window 1048576 --streams 4 --steps 2 \
  --chain-cache $C > "$O/chained4m_$T.json" 2> "$O/chained4m_$T.err"
echo "done $T"
