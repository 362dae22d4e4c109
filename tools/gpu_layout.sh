#!/bin/bash
# full GPU suite, fuse sweeps and Humanoid / Ant bench lines
source "$(dirname "$0")/gpu_lib.sh"
run pytest_gpu 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run fuse_h 200 python -u tools/fuse_roofline.py Humanoid 262144,1048576,2097152
run fuse_a 200 python -u tools/fuse_roofline.py Ant 262144,1048576,2097152
grep -h '^{' gpurun_out/fuse_h.log gpurun_out/fuse_a.log
B="python -u bench.py --steps 300 --warmup 50 --no-cpu-baseline --fuse-envs 0 --no-side"
run hum 120 $B
run ant 120 $B --task Ant
grep -h -o '"value": [0-9.]*, "unit\|"kernel_ms": [0-9.]*' gpurun_out/hum.log gpurun_out/ant.log
echo ALL_DONE
