#!/bin/bash
# DR + zero-copy rollout GPU tests, full GPU suite, Humanoid bench (perf regression check)
source "$(dirname "$0")/gpu_lib.sh"
run pytest_new 300 python -u -m pytest tests/test_gpu_dr.py tests/test_gpu_rollout.py -x -v --timeout 120 --timeout-method thread
run pytest_gpu 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run bench_humanoid 200 python -u bench.py --steps 300 --warmup 50 --no-cpu-baseline
run bench_ant 150 python -u bench.py --task Ant --steps 300 --warmup 50 --no-cpu-baseline
echo ALL_DONE
