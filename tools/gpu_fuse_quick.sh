#!/bin/bash
# obs/reward fuse iteration: GPU parity tests, then the Humanoid / Ant fuse roofline sweeps of
# the pipelined kernel (default 32p) and the one-tile kernel (32s)
source "$(dirname "$0")/gpu_lib.sh"
run pytest_gpu 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run fuse_a_32s 300 env MI_POST_TILE=32s python -u tools/fuse_roofline.py Ant 65536,262144,1048576
cp gpurun_out/fuse_roofline_ant.json gpurun_out/fuse_roofline_ant_32s.json
run fuse_h_32s 300 env MI_POST_TILE=32s python -u tools/fuse_roofline.py Humanoid 65536,262144,1048576
cp gpurun_out/fuse_roofline_humanoid.json gpurun_out/fuse_roofline_humanoid_32s.json
run fuse_a 300 python -u tools/fuse_roofline.py Ant 4096,65536,262144,1048576
run fuse_h 300 python -u tools/fuse_roofline.py Humanoid 4096,65536,262144,1048576
echo ALL_DONE
