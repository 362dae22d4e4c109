#!/bin/bash
source "$(dirname "$0")/gpu_lib.sh"
B="python -u bench.py --steps 300 --warmup 50 --no-cpu-baseline --fuse-envs 0 --no-side --events-apart"
run ev_h 120 $B
run ev_a 120 $B --task Ant
grep -h events_apart gpurun_out/ev_h.log gpurun_out/ev_a.log
echo ALL_DONE
