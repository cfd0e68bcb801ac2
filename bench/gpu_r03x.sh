#!/bin/bash
# r03x: carry-free product operands in the G2 bucket pass's mixed additions. GPU tests, G2 bench, then the PMC
# passes of both schemes on this build (bench/pmc.sh) for bench.py's traffic field.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
T=${1:-r03x}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > "$O/gpu_tests_$T.log" 2>&1
timeout -k 10 300 python bench.py --scheme pedersen-bls-unchained --no-cpu-baseline --single-call-steps 0 > "$O/bench_unch_$T.json" 2> "$O/bench_$T.err"
timeout -k 10 700 bash bench/pmc.sh $T > "$O/pmc_$T.out" 2>&1
timeout -k 10 700 bash bench/pmc.sh ${T}_g2 pedersen-bls-unchained > "$O/pmc_${T}_g2.out" 2>&1
echo "done $T"
