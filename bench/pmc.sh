#!/bin/bash
# PMC passes (one counter group per run, MI355X_MICROARCH.md) over one single-stream 262144-round batch of bench.py
# for any scheme:  bash bench/pmc.sh <tag> [scheme]
# FETCH_SIZE, WRITE_SIZE, the SQ instruction mix, and the VALU-busy pass; summarise with bench/pmc_summary.py.
set -euo pipefail
TAG=${1:-dev}
SCHEME=${2:-bls-unchained-g1-rfc9380}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
SMALL="--scheme $SCHEME --total-rounds 262144 --steps 1 --warmup 0 --streams 1 --roofline-steps 0 --single-call-steps 0 --single-beacon-reps 0 --no-cpu-baseline"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_fetch_$TAG" -o pmc --output-format csv -- python3 "$R/bench.py" $SMALL \
  > "$O/pmc_fetch_$TAG.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d "$O/pmc_write_$TAG" -o pmc --output-format csv -- python3 "$R/bench.py" $SMALL \
  > "$O/pmc_write_$TAG.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
  SQ_INSTS_LDS SQ_INSTS_FLAT SQ_INSTS_SMEM -d "$O/pmc_sq_$TAG" -o pmc --output-format csv -- python3 "$R/bench.py" $SMALL \
  > "$O/pmc_sq_$TAG.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY \
  SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE -d "$O/pmc_busy_$TAG" -o pmc --output-format csv -- python3 "$R/bench.py" $SMALL \
  > "$O/pmc_busy_$TAG.log" 2>&1
echo "pmc $TAG $SCHEME done"
