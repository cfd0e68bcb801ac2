#!/bin/bash
# Profiling recipe for the headline bench (run on the GPU box from the repo root):
#   bash bench/profile.sh <tag>
# 1. rocprofv3 --kernel-trace --stats over the default bench command (1M quicknet rounds, 8 batches in flight,
#    then bench.py's 2 single-stream roofline batches) -> bench/rocpd_stats.py --last 2 gives the per-kernel
#    average over exactly the launches bench.py's HIP-event roofline measures;
# 2. --pmc passes over one single-stream 262144-round batch, one counter group per run as MI355X_MICROARCH.md
#    prescribes (TCC: FETCH_SIZE uses 3 of 4 counters, WRITE_SIZE 2; SQ: at most 8): FETCH_SIZE, WRITE_SIZE, the SQ
#    instruction mix, and the VALU-busy pass (SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES / SQ_BUSY_CYCLES in quad-cycles,
#    GRBM_GUI_ACTIVE in cycles summed over the 8 XCDs).
# Each step has its own time limit; the first failure ends the script.
set -euo pipefail
TAG=${1:-r02}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_$TAG" -o run --output-format csv -- \
  python3 "$R/bench.py" --steps 8 --warmup 8 --single-call-steps 0 --single-beacon-reps 0 --no-cpu-baseline > "$O/prof_$TAG.log" 2>&1
SMALL="--total-rounds 262144 --steps 1 --warmup 0 --streams 1 --roofline-steps 0 --single-call-steps 0 --single-beacon-reps 0 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_fetch_$TAG" -o pmc --output-format csv -- python3 "$R/bench.py" $SMALL \
  > "$O/pmc_fetch_$TAG.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$O/pmc_write_$TAG" -o pmc --output-format csv -- python3 "$R/bench.py" $SMALL \
  > "$O/pmc_write_$TAG.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
  SQ_INSTS_LDS SQ_INSTS_FLAT SQ_INSTS_SMEM -d "$O/pmc_sq_$TAG" -o pmc --output-format csv -- python3 "$R/bench.py" $SMALL \
  > "$O/pmc_sq_$TAG.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY \
  SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE -d "$O/pmc_busy_$TAG" -o pmc --output-format csv -- python3 "$R/bench.py" $SMALL \
  > "$O/pmc_busy_$TAG.log" 2>&1
echo "profile $TAG done"
