#!/bin/bash
# round 6: PPO learner profile — bench_train (frames/s) and its rocprofv3 kernel trace
export TMPDIR=/tmp
mkdir -p gpurun_out/r06/train
timeout -k 10 300 python -u tools/bench_train.py > gpurun_out/r06/train/bench_train.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --output-format csv --kernel-trace --stats -d gpurun_out/r06/train/prof -o run -- \
  python3 tools/bench_train.py --epochs 4 --warmup 2 > gpurun_out/r06/train/prof.log 2>&1 || exit $?
