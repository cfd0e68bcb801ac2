#!/bin/bash
# r03b: executed field products per kernel (counting build) + the G2 PMC passes (work-model evidence)
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
T=${1:-r03b}
DRANDHIP_LIB=$R/drand_amd/libdrandhip_count.so timeout -k 10 400 python -u bench/count_products.py --rounds 131072 1048576 \
  --out "$O/count_products_$T.json" > "$O/count_products_$T.log" 2>&1
bash bench/pmc.sh "${T}_g2" pedersen-bls-unchained
echo "done $T"
