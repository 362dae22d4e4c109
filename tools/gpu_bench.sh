#!/bin/bash
# default bench line + its rocprofv3 kernel-trace stats (+ the events diagnostic)
source "$(dirname "$0")/gpu_lib.sh"
run ev_h 120 python -u bench.py --steps 300 --warmup 50 --no-cpu-baseline --fuse-envs 0 --no-side --events-apart
grep -h events_apart gpurun_out/ev_h.log
run bench_default 500 python -u bench.py
run prof_bench 500 rocprofv3 --output-format csv --kernel-trace --stats -d gpurun_out/prof_bench -o run -- python3 bench.py
echo ALL_DONE
