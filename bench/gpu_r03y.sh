#!/bin/bash
# r03y: the per-rank shape of the 8-GPU strong-scaling run on one GPU (131,072 rounds under the node-wide check:
# dh_batch_begin -> dh_check_partials -> dh_batch_finish, minus the collective), twice, against the local check;
# and the 262k / 524k shapes (N = 4 / 2).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
T=${1:-r03y}
B="--no-cpu-baseline --single-call-steps 0"
for n in 131072 262144 524288; do
  timeout -k 10 200 python bench.py --total-rounds $n --node-check on $B > "$O/node_${n}_$T.json" 2>> "$O/node_$T.err"
  timeout -k 10 200 python bench.py --total-rounds $n --node-check off $B > "$O/local_${n}_$T.json" 2>> "$O/node_$T.err"
done
timeout -k 10 200 python bench.py --total-rounds 131072 --node-check on $B > "$O/node_131072b_$T.json" 2>> "$O/node_$T.err"
echo "done $T"
