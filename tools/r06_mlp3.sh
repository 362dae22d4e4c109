#!/bin/bash
# round 6: fused training MLP in the learner — loss parity, rocprofv3 kernel trace of the
# PPO epoch, reference-schedule training curves (Humanoid, Ant)
export TMPDIR=/tmp
O=gpurun_out/r06/mlp3
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_rl_gpu.py -m gpu -k "fused_loss or graph_update" > $O/tests.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --output-format csv --kernel-trace --stats -d $O/prof -o run -- \
  python3 tools/bench_train.py --epochs 4 --warmup 2 > $O/prof.log 2>&1 || exit $?
timeout -k 10 900 python -u tools/train_curve.py --task Humanoid --out $O/train_curve_humanoid.jsonl > $O/curve_Humanoid.log 2>&1 || exit $?
timeout -k 10 900 python -u tools/train_curve.py --task Ant --out $O/train_curve_ant.jsonl > $O/curve_Ant.log 2>&1 || exit $?
