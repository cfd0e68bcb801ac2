#!/bin/bash
# r03final: the committed final tree as the driver runs it: GPU tests, smoke, bench.py with its defaults.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
T=${1:-r03final}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > "$O/gpu_tests_$T.log" 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke_$T.log" 2>&1
timeout -k 10 300 python bench.py > "$O/bench_$T.json" 2> "$O/bench_$T.err"
echo "done $T"
