#!/bin/bash
source "$(dirname "$0")/gpu_lib.sh"
run bt_default 300 python -u tools/bench_train.py --task Humanoid --epochs 4 --warmup 3
TORCH_BLAS_PREFER_HIPBLASLT=0 run bt_rocblas 300 python -u tools/bench_train.py --task Humanoid --epochs 4 --warmup 3
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_results.csv run bt_tunable 600 python -u tools/bench_train.py --task Humanoid --epochs 4 --warmup 3
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_results.csv run bt_tuned 300 python -u tools/bench_train.py --task Humanoid --epochs 4 --warmup 3
echo ALL_DONE
