#!/bin/bash
# r03zc: verify_node_batch waits for torch's gathered sums with an event (none with one rank) instead of a stream sync.
# and evicted the batch path's cache). GPU tests, then the per-rank shapes of the strong-scaling run (node-wide check
# on, one GPU) against the local check.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
T=${1:-r03zc}
B="--no-cpu-baseline --single-call-steps 0"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > "$O/gpu_tests_$T.log" 2>&1
for n in 131072 262144 524288; do
  timeout -k 10 200 python bench.py --total-rounds $n --node-check on $B > "$O/node_${n}_$T.json" 2>> "$O/node_$T.err"
done
timeout -k 10 200 python bench.py --total-rounds 131072 $B > "$O/local_131072_$T.json" 2>> "$O/node_$T.err"
timeout -k 10 200 python bench.py --total-rounds 131072 --node-check on $B > "$O/node_131072b_$T.json" 2>> "$O/node_$T.err"
for S in 12 16; do
  timeout -k 10 200 python bench.py --total-rounds 131072 --node-check on --streams $S $B > "$O/node_131072_s${S}_$T.json" 2>> "$O/node_$T.err"
done
echo "done $T"
