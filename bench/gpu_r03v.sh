#!/bin/bash
# r03v: carry-free operands in the G1 subgroup test's inlined doubling. GPU tests, the headline bench as the driver
# runs it (defaults, CPU baseline), its rocprofv3 kernel trace, the 131k shard, smoke, and the product counts of the
# current build (counting library).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
T=${1:-r03v}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > "$O/gpu_tests_$T.log" 2>&1
timeout -k 10 300 python bench.py > "$O/bench_$T.json" 2> "$O/bench_$T.err"
timeout -k 10 200 python bench.py --total-rounds 131072 --no-cpu-baseline --single-call-steps 0 > "$O/shard131k_$T.json" 2>> "$O/bench_$T.err"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke_$T.log" 2>&1
DRANDHIP_LIB=$R/drand_amd/libdrandhip_count.so timeout -k 10 400 python -u bench/count_products.py --rounds 1048576 \
  --out "$O/count_products_$T.json" > "$O/count_products_$T.log" 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_$T" -o run --output-format csv -- \
  python3 "$R/bench.py" --steps 8 --warmup 8 --single-call-steps 0 --no-cpu-baseline > "$O/prof_$T.log" 2>&1
echo "done $T"
