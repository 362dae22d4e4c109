#!/bin/bash
# obs/reward fuse kernel: GPU tests, HBM roofline sweeps (Humanoid, Ant), Humanoid bench
source "$(dirname "$0")/gpu_lib.sh"
run pytest_gpu 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
run fuse_h 300 python -u tools/fuse_roofline.py Humanoid 65536,262144,1048576
run fuse_a 300 python -u tools/fuse_roofline.py Ant 65536,262144,1048576
run bench_humanoid 200 python -u bench.py --steps 300 --warmup 50 --no-cpu-baseline --fuse-envs 0
echo ALL_DONE
