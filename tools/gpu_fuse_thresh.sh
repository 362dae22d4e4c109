#!/bin/bash
# pipelined-vs-one-tile crossover of the obs/reward fuse: MI_POST_PIPE_MIN = tiles per workgroup
source "$(dirname "$0")/gpu_lib.sh"
for m in 1 2 4 1000000; do
  run fuse_h_min$m 200 env MI_POST_PIPE_MIN=$m python -u tools/fuse_roofline.py Humanoid 131072,262144,524288
  run fuse_a_min$m 200 env MI_POST_PIPE_MIN=$m python -u tools/fuse_roofline.py Ant 131072,262144,524288
done
echo ALL_DONE
