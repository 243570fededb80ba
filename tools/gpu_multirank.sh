# Rehearse the sharded bench path on a 1-GPU box: 2 ranks share cuda:0 over gloo.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --backend gloo > gpurun_out/bench_2rank.json 2> gpurun_out/bench_2rank.err
