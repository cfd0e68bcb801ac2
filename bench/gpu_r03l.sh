#!/bin/bash
# r03l: new defaults (bucket-pass chunks >= 8 entries, 16 hardware queues in the benches): headline bench with the
# CPU baseline, 131k shard, G2 unchained bench and its rocprofv3 kernel trace, chained 4M replay and the kernel
# trace of one single-stream pass over it.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
T=${1:-r03l}
C=/tmp/drandhip_chain_cache
timeout -k 10 300 python bench.py > "$O/bench_$T.json" 2> "$O/bench_$T.err"
timeout -k 10 200 python bench.py --total-rounds 131072 --no-cpu-baseline --single-call-steps 0 > "$O/shard131k_$T.json" 2>> "$O/bench_$T.err"
timeout -k 10 300 python bench.py --scheme pedersen-bls-unchained --no-cpu-baseline --single-call-steps 0 > "$O/bench_unch_$T.json" 2>> "$O/bench_$T.err"
timeout -k 10 600 python bench/bench_configs.py chained --rounds 4194304 --window 1048576 --streams 4 --steps 2 \
  --chain-cache $C > "$O/chained4m_$T.json" 2> "$O/chained4m_$T.err"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_unch_$T" -o run --output-format csv -- \
  python3 "$R/bench.py" --scheme pedersen-bls-unchained --steps 4 --warmup 8 --single-call-steps 0 --no-cpu-baseline > "$O/prof_unch_$T.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_chained_$T" -o run --output-format csv -- \
  python3 "$R/bench/bench_configs.py" chained --rounds 4194304 --window 1048576 --streams 1 --steps 1 --cpu-sample 10 \
  --chain-cache $C > "$O/prof_chained_$T.log" 2>&1
echo "done $T"
