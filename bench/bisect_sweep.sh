#!/bin/bash
# Bisection-ladder sweep on the chained-replay config (a real sequential chain, Cfg5 corruption classes), one
# stream, one 1M window: the adaptive ladder (next_group_size) against fixed ladders set through DRANDHIP_BISECT
# (read when the library loads, so one process per ladder; the chain is signed once and cached).
#   bash bench/bisect_sweep.sh <tag> [rounds] [densities] [ladders]
set -euo pipefail
TAG=${1:-dev}
N=${2:-1048576}
DENS=${3:-"0.001"}
LADDERS=${4:-"adaptive 256,16,2 64,4 512,32,4"}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
CACHE=${TMPDIR:-/tmp}/drandhip_chain_cache  # ~100 MB per 1M chain: outside gpurun_out
cd "$R"
for C in $DENS; do
  for L in $LADDERS; do
    if [ "$L" = adaptive ]; then unset DRANDHIP_BISECT; else export DRANDHIP_BISECT=$L; fi
    echo "corrupt $C ladder $L" >> "$O/bisect_$TAG.txt"
    timeout -k 10 240 python bench/bench_configs.py chained --rounds $N --window $N --streams 1 --steps 2 \
      --cpu-sample 10 --cpu-threads 4 --corrupt $C --chain-cache "$CACHE" >> "$O/bisect_$TAG.txt" 2>> "$O/bisect_$TAG.err"
  done
done
rm -rf "$CACHE"
echo "sweep $TAG done"
