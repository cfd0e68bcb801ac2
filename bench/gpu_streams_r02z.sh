#!/bin/bash
# Streams in flight at the 8-GPU strong-scaling shard size (131072 rounds per GPU), on one GPU.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
for s in 4 12 16; do
  timeout -k 10 200 python bench.py --total-rounds 131072 --streams $s --no-cpu-baseline --single-call-steps 0 > "$O/streams_${s}_131k.json" 2> "$O/streams_${s}_131k.err"
done
echo streams done
