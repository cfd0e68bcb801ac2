#!/bin/bash
# r03p: tbls Recover config (n = 64, t = 33, 100k rounds) on the r03 build; chained 4M replay with the one-lane pairing
# path for group checks and leaves (DRANDHIP_LANE_PAIRING=1) against the VM, one stream and 4 streams.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
T=${1:-r03p}
C=/tmp/drandhip_chain_cache
timeout -k 10 300 python bench/bench_configs.py recover > "$O/cfg_recover_$T.json" 2> "$O/cfg_recover_$T.err"
timeout -k 10 500 python bench/bench_configs.py chained --rounds 4194304 --window 1048576 --streams 1 --steps 1 \
  --chain-cache $C > "$O/chained4m_s1_vm_$T.json" 2> "$O/chained4m_$T.err"
DRANDHIP_LANE_PAIRING=1 timeout -k 10 300 python bench/bench_configs.py chained --rounds 4194304 --window 1048576 --streams 1 \
  --steps 1 --chain-cache $C > "$O/chained4m_s1_lane_$T.json" 2>> "$O/chained4m_$T.err"
DRANDHIP_LANE_PAIRING=1 timeout -k 10 300 python bench/bench_configs.py chained --rounds 4194304 --window 1048576 --streams 4 \
  --steps 2 --chain-cache $C > "$O/chained4m_lane_$T.json" 2>> "$O/chained4m_$T.err"
echo "done $T"
# smoke and a 2-rank gloo rehearsal of the multi-GPU bench path on the one GPU (both ranks on GPU 0)
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke_$T.log" 2>&1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --backend gloo --steps 4 --warmup 4 --streams 2 > "$O/gloo2_$T.json" 2> "$O/gloo2_$T.err"
echo "smoke + gloo done $T"
