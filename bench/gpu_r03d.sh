#!/bin/bash
# r03d: executed products with the 28-bit G1 MSM; single-stream kernel traces of quicknet and unchained batches
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
T=${1:-r03d}
DRANDHIP_LIB=$R/drand_amd/libdrandhip_count.so timeout -k 10 300 python -u bench/count_products.py --rounds 131072 1048576 \
  --out "$O/count_products_$T.json" > "$O/count_products_$T.log" 2>&1
cd /tmp && export TMPDIR=/tmp
for S in bls-unchained-g1-rfc9380 pedersen-bls-unchained; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/prof1s_${T}_$S" -o run --output-format csv -- \
    python3 "$R/bench.py" --scheme $S --streams 1 --steps 3 --warmup 1 --roofline-steps 0 --single-call-steps 0 --no-cpu-baseline \
    > "$O/prof1s_${T}_$S.log" 2>&1
done
echo "done $T"
