#!/bin/bash
# GPU tests + free-running distribution stats
source "$(dirname "$0")/gpu_lib.sh"
run pytest_gpu 500 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread
run fr_h 300 python -u tools/free_run.py Humanoid 4096 200
run fr_a 300 python -u tools/free_run.py Ant 4096 200
run fr_c 300 python -u tools/free_run.py Cartpole 4096 300
grep -h '"task"' gpurun_out/fr_h.log gpurun_out/fr_a.log gpurun_out/fr_c.log
echo ALL_DONE
