#!/bin/bash
source "$(dirname "$0")/gpu_lib.sh"
run pytest_post 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread
for V in 64s 64d 32s 32d; do
  MI_POST_TILE=$V run fuse_h_$V 300 python -u tools/fuse_roofline.py Humanoid 65536,262144,1048576
done
echo ALL_DONE
