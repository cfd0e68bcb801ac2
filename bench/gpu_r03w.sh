#!/bin/bash
# r03w: PMC passes of both schemes on the final r03 build (bench/pmc.sh), for bench.py's traffic field.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
T=${1:-r03w}
timeout -k 10 700 bash bench/pmc.sh $T > "$O/pmc_$T.out" 2>&1
timeout -k 10 700 bash bench/pmc.sh ${T}_g2 pedersen-bls-unchained > "$O/pmc_${T}_g2.out" 2>&1
echo "done $T"
