#!/bin/bash
# PMC passes for the instruction-level accounting of the per-round kernels (bench/isa_account.py): the VALU
# instruction classes (INT64 = v_mad_u64_u32 and the 64-bit shifts/adds, INT32 = the rest of the integer VALU) and the
# VALU busy cycles, over one single-stream 262144-round batch of bench.py; one counter group per run.
#   bash bench/pmc_isa.sh <tag> [scheme]
set -euo pipefail
TAG=${1:-dev}
SCHEME=${2:-bls-unchained-g1-rfc9380}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
SMALL="--scheme $SCHEME --total-rounds 262144 --steps 1 --warmup 0 --streams 1 --roofline-steps 0 --single-call-steps 0 --single-beacon-reps 0 --no-cpu-baseline"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_SALU \
  SQ_INSTS_VALU_CVT SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU -d "$O/pmc_isa_$TAG" -o pmc --output-format csv -- \
  python3 "$R/bench.py" $SMALL > "$O/pmc_isa_$TAG.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY \
  SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE -d "$O/pmc_isabusy_$TAG" -o pmc --output-format csv -- python3 "$R/bench.py" $SMALL \
  > "$O/pmc_isabusy_$TAG.log" 2>&1
echo "pmc_isa $TAG $SCHEME done"
