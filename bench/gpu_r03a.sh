#!/bin/bash
# r03a: GPU tests (new node-wide / two-process / tryNode / relay tests included), then the 131k-round shard shape
# (the per-GPU size of the 8-GPU strong-scaling run) with a kernel trace. First failure ends it.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
T=${1:-r03a}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > "$O/gpu_tests_$T.log" 2>&1
timeout -k 10 200 python bench.py --total-rounds 131072 --no-cpu-baseline --single-call-steps 0 > "$O/shard131k_$T.json" 2> "$O/shard131k_$T.err"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/prof131k_$T" -o run --output-format csv -- \
  python3 "$R/bench.py" --total-rounds 131072 --steps 8 --warmup 8 --single-call-steps 0 --no-cpu-baseline > "$O/prof131k_$T.log" 2>&1
echo "done $T"
