#!/bin/bash
# learner GPU tests only
source "$(dirname "$0")/gpu_lib.sh"
run pytest_rl 400 python -u -m pytest tests/test_rl_gpu.py -x -v --timeout 300 --timeout-method thread
echo ALL_DONE
