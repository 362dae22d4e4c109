#!/bin/bash
# quick GPU check: parity tests + Humanoid bench
source "$(dirname "$0")/gpu_lib.sh"
run pytest_gpu 300 python -u -m pytest tests -m gpu -x -q
run bench_humanoid 200 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline
echo ALL_DONE
