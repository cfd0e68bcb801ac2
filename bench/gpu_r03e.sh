#!/bin/bash
# r03e: 28-bit MSM for G1 and G2 (affine hash points, fast-then-exact reductions), lazy G2 subgroup test:
# GPU tests, single-stream kernel traces, quicknet + unchained benches
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
T=${1:-r03e}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > "$O/gpu_tests_$T.log" 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline --single-call-steps 0 > "$O/bench_$T.json" 2> "$O/bench_$T.err"
timeout -k 10 300 python bench.py --scheme pedersen-bls-unchained --no-cpu-baseline --single-call-steps 0 > "$O/bench_unch_$T.json" 2> "$O/bench_unch_$T.err"
cd /tmp && export TMPDIR=/tmp
for S in bls-unchained-g1-rfc9380 pedersen-bls-unchained; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/prof1s_${T}_$S" -o run --output-format csv -- \
    python3 "$R/bench.py" --scheme $S --streams 1 --steps 3 --warmup 1 --roofline-steps 0 --single-call-steps 0 --no-cpu-baseline \
    > "$O/prof1s_${T}_$S.log" 2>&1
done
echo "done $T"
