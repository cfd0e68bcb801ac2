#!/bin/bash
# Bisection-ladder sweep over 1M corrupted rounds (chained replay by default; quicknet / unchained), one stream:
#   bash bench/bisect_sweep.sh <tag> [chained|quicknet|unchained]
# adaptive (default) vs the fixed r01 ladder at three fault densities set through DRANDHIP_BISECT; one JSON line per ladder.
set -euo pipefail
TAG=${1:-dev}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
CFG=${2:-chained}
ARGS="$CFG --streams 1 --steps 2 --warmup 1 --cpu-sample 100 --cpu-threads 4"
for C in 0.001 0.000001 0.01; do
  for L in adaptive 4096,256,16,2; do
    if [ "$L" = adaptive ]; then unset DRANDHIP_BISECT; else export DRANDHIP_BISECT=$L; fi
    echo "corrupt $C ladder $L" >> "$O/bisect_$TAG.txt"
    timeout -k 10 150 python bench/bench_configs.py $ARGS --corrupt $C >> "$O/bisect_$TAG.txt" 2>> "$O/bisect_$TAG.err"
  done
done
echo "sweep $TAG done"
