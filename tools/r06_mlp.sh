#!/bin/bash
# round 6: fused fp16-MFMA training MLP — parity tests, then bench_train with it on / off
export TMPDIR=/tmp
mkdir -p gpurun_out/r06/mlp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_train_mlp.py -m gpu > gpurun_out/r06/mlp/tests.log 2>&1 || exit $?
for k in 1 2; do
  for f in 1 0; do
    MI_RL_FUSED_MLP=$f timeout -k 10 300 python -u tools/bench_train.py > gpurun_out/r06/mlp/bench_train_f${f}_$k.log 2>&1 || exit $?
  done
done
timeout -k 10 400 rocprofv3 --output-format csv --kernel-trace --stats -d gpurun_out/r06/mlp/prof -o run -- \
  python3 tools/bench_train.py --epochs 4 --warmup 2 > gpurun_out/r06/mlp/prof.log 2>&1 || exit $?
