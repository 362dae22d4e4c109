#!/bin/bash
source "$(dirname "$0")/gpu_lib.sh"
run prof_train 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_train -o run -- python3 tools/bench_train.py --task Humanoid --epochs 4 --warmup 3
echo ALL_DONE
