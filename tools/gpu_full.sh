#!/bin/bash
source "$(dirname "$0")/gpu_lib.sh"
run pytest_full 400 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 200 --timeout-method thread
echo ALL_DONE
