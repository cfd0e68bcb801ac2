#!/bin/bash
# r03n: G2 bucket chunks sized to the pass's occupancy (64 entries at 1M); G2 + quicknet benches; PMC passes of both
# schemes (bench/pmc.sh) on the current build.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
T=${1:-r03n}
B="--no-cpu-baseline --single-call-steps 0"
timeout -k 10 300 python bench.py --scheme pedersen-bls-unchained $B > "$O/bench_unch_$T.json" 2> "$O/bench_$T.err"
timeout -k 10 300 python bench.py $B > "$O/bench_$T.json" 2>> "$O/bench_$T.err"
timeout -k 10 700 bash bench/pmc.sh $T > "$O/pmc_$T.out" 2>&1
timeout -k 10 700 bash bench/pmc.sh ${T}_g2 pedersen-bls-unchained > "$O/pmc_${T}_g2.out" 2>&1
echo "done $T"
