set -euo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python bench.py > $O/bench_r02u.json 2> $O/bench_r02u.err
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --total-rounds 262144 --steps 4 --warmup 2 --backend gloo --no-cpu-baseline --single-call-steps 0 > $O/gloo2_r02u.json 2> $O/gloo2_r02u.err
bash bench/profile.sh r02u
echo done
