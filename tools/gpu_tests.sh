#!/bin/bash
# the GPU test suite (what the driver runs at round end)
source "$(dirname "$0")/gpu_lib.sh"
run pytest_gpu 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread
grep -E "^FAILED|^E  .*Error|passed|failed" gpurun_out/pytest_gpu.log | head -30
echo ALL_DONE
