#!/bin/bash
# obs/reward fuse iteration: GPU suite, Humanoid / Ant fuse sweeps (two passes each)
source "$(dirname "$0")/gpu_lib.sh"
run pytest_gpu 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
for k in 1 2; do
run fuse_h$k 200 python -u tools/fuse_roofline.py Humanoid 262144,1048576,2097152
run fuse_a$k 200 python -u tools/fuse_roofline.py Ant 1048576,2097152
done
cat gpurun_out/fuse_roofline_humanoid.json > /dev/null
grep -h '^{' gpurun_out/fuse_h1.log gpurun_out/fuse_h2.log gpurun_out/fuse_a1.log gpurun_out/fuse_a2.log | cut -c1-200
echo ALL_DONE
