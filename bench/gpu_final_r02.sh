#!/bin/bash
# End-of-round check of the committed tree: GPU parity tests, smoke, the default bench (CPU baseline included),
# a gloo 2-rank rehearsal and the profiling recipe (rocprofv3 kernel stats + PMC passes). First failure ends it.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
T=${1:-r02f}
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/gpu_tests_$T.log" 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke_$T.log" 2>&1
timeout -k 10 300 python bench.py > "$O/bench_$T.json" 2> "$O/bench_$T.err"
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --total-rounds 262144 --steps 4 --warmup 2 --backend gloo --no-cpu-baseline --single-call-steps 0 \
  > "$O/gloo2_$T.json" 2> "$O/gloo2_$T.err"
bash bench/profile.sh "$T"
echo "final $T done"
