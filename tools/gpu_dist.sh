# The driver's multi-GPU launch path, rehearsed on a 1-GPU box:
#   1. torchrun world 1 with the nccl (RCCL) backend: the exact N>1 command shape,
#      barrier + max-over-ranks timing and the end-of-batch all_gather over RCCL;
#   2. torchrun world 2 with gloo, both ranks sharing cuda:0 (control flow and
#      sharding only, timing not meaningful);
#   3. `python bench.py --gpus 2` without torchrun (the script's own launcher).
# Results: gpurun_out/dist/
set -o pipefail
mkdir -p gpurun_out/dist
A="--steps 3 --warmup 1 --no-cpu"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 \
  bench.py --gpus 1 $A > gpurun_out/dist/w1_nccl.json 2> gpurun_out/dist/w1_nccl.err || exit $?
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 \
  bench.py --gpus 2 --dist-backend gloo $A > gpurun_out/dist/w2_gloo.json 2> gpurun_out/dist/w2_gloo.err || exit $?
# 3. the bare `bench.py --gpus 2` (no launcher): the script starts its two ranks itself
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo $A > gpurun_out/dist/w2_launcher.json 2> gpurun_out/dist/w2_launcher.err || exit $?
echo dist done
