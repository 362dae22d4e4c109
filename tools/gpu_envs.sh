#!/bin/bash
# multi-env workgroups: GPU tests at E=1 (default) and E=4, bench at E=1/2/4
source "$(dirname "$0")/gpu_lib.sh"
B="python -u bench.py --steps 200 --warmup 30 --no-cpu-baseline --fuse-envs 0 --no-side"
run pytest_gpu 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run pytest_gpu_e4 400 env MI_WAVE_ENVS=4 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run hum_e1 120 $B
run hum_e2 120 env MI_WAVE_ENVS=2 $B
run hum_e4 120 env MI_WAVE_ENVS=4 $B
for f in hum_e1 hum_e2 hum_e4; do echo $f; grep -o '"lds_bytes_per_env": [0-9]*\|"kernel_ms": [0-9.]*' gpurun_out/$f.log; done
echo ALL_DONE
