#!/bin/bash
# quick iteration: parity tests, Humanoid/Ant bench, phase timers
source "$(dirname "$0")/gpu_lib.sh"
run pytest_gpu 300 python -u -m pytest tests -m gpu -x -q
run bench_humanoid 200 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline
run bench_ant 150 python -u bench.py --task Ant --steps 200 --warmup 20 --no-cpu-baseline
run stamps_humanoid 150 python -u tools/phase_stamps.py Humanoid 4096
run stamps_ant 150 python -u tools/phase_stamps.py Ant 4096
echo ALL_DONE
