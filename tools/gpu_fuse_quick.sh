#!/bin/bash
# obs/reward fuse iteration: GPU parity tests (incl. the fuse-vs-oracle full-size cases), then the
# Humanoid / Ant fuse roofline sweeps
source "$(dirname "$0")/gpu_lib.sh"
run pytest_gpu 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
run fuse_a 300 python -u tools/fuse_roofline.py Ant 65536,262144,1048576,2097152
run fuse_h 300 python -u tools/fuse_roofline.py Humanoid 65536,262144,1048576,2097152
echo ALL_DONE
