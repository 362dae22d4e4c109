#!/bin/bash
# learner: GPU tests of libmi_rl + learner, training throughput (graphed rollout + graphed
# updates, graphed rollout + eager updates, all eager)
source "$(dirname "$0")/gpu_lib.sh"
run pytest_rl 300 python -u -m pytest tests/test_rl_gpu.py -x -v --timeout 240 --timeout-method thread
run bench_train 300 python -u tools/bench_train.py --task Humanoid --epochs 6 --warmup 3
run bench_train_eager_update 300 python -u tools/bench_train.py --task Humanoid --epochs 4 --warmup 2 --no-graph-update
run bench_train_eager 300 python -u tools/bench_train.py --task Humanoid --epochs 4 --warmup 2 --no-graph
echo ALL_DONE
