set -e -o pipefail
TAG=${1:-x}
O=gpurun_out/$TAG; mkdir -p $O
CONCRETE_HIP_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --batch 1024 > $O/bench_n2.log 2>&1
echo done
