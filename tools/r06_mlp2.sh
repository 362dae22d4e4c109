#!/bin/bash
# round 6: fused training MLP — parity tests, kernel times, bench_train
export TMPDIR=/tmp
mkdir -p gpurun_out/r06/mlp2
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_train_mlp.py -m gpu > gpurun_out/r06/mlp2/tests.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/mlp_bench.py > gpurun_out/r06/mlp2/mlp_bench.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/bench_train.py > gpurun_out/r06/mlp2/bench_train.log 2>&1 || exit $?
