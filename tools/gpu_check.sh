#!/bin/bash
# quick check: GPU tests, the default bench line, the 1-rank torchrun bench (RCCL group + gather)
source "$(dirname "$0")/gpu_lib.sh"
run pytest_gpu 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run bench_default 500 python -u bench.py
run bench_torchrun1 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --fuse-envs 0
echo ALL_DONE
