#!/bin/bash
# launch-timing tests, the events diagnostic (plain / torch events / dispatch events) and the bench
source "$(dirname "$0")/gpu_lib.sh"
run pytest_timing 200 python -u -m pytest tests/test_gpu_timing.py -x -v --timeout 120 --timeout-method thread
B="python -u bench.py --steps 300 --warmup 50 --no-cpu-baseline --fuse-envs 0 --no-side --events-apart"
run ev_h 120 $B
run ev_a 120 $B --task Ant
grep -h events_apart gpurun_out/ev_h.log gpurun_out/ev_a.log
run fuse_h 200 python -u tools/fuse_roofline.py Humanoid 262144,1048576
run fuse_a 200 python -u tools/fuse_roofline.py Ant 1048576
grep -h '^{' gpurun_out/fuse_h.log gpurun_out/fuse_a.log
echo ALL_DONE
