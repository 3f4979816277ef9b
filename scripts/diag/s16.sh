set -o pipefail
O=gpurun_out/s16
mkdir -p $O
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29502 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo > $O/gloo_2.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_multiproc.py tests/test_gpu_dist.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit $?
