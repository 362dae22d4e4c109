#!/bin/bash
# obs/reward fuse iteration: GPU parity tests, then the Humanoid / Ant fuse roofline sweeps
# (default selection: pipelined kernel at >= 8 tiles per resident workgroup, else one-tile)
source "$(dirname "$0")/gpu_lib.sh"
run pytest_gpu 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run fuse_a 300 python -u tools/fuse_roofline.py Ant 65536,262144,1048576,2097152
run fuse_h 300 python -u tools/fuse_roofline.py Humanoid 65536,262144,1048576,2097152
echo ALL_DONE
