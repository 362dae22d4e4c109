#!/bin/bash
# round-end: GPU suite, smoke, fuse sweeps + rocprof, bench + rocprof (TRAFFIC=1: traffic sweeps)
source "$(dirname "$0")/gpu_lib.sh"
run pytest_gpu 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
if [ -n "$TRAFFIC" ]; then
TASK=Humanoid bash tools/gpu_traffic_sweep.sh
TASK=Ant bash tools/gpu_traffic_sweep.sh
fi
RP="rocprofv3 --output-format csv"
run fuse_h 300 python -u tools/fuse_roofline.py Humanoid 4096,65536,131072,262144,1048576,2097152
cp gpurun_out/fuse_roofline_humanoid.json gpurun_out/sweep_fuse_humanoid.json
run fuse_a 300 python -u tools/fuse_roofline.py Ant 4096,65536,131072,262144,1048576,2097152
cp gpurun_out/fuse_roofline_ant.json gpurun_out/sweep_fuse_ant.json
run prof_fuse 300 $RP --kernel-trace --stats -d gpurun_out/prof_fuse -o run -- python3 tools/fuse_roofline.py Humanoid 1048576 20
run bench_default 500 python -u bench.py
run prof_bench 500 $RP --kernel-trace --stats -d gpurun_out/prof_bench -o run -- python3 bench.py
echo ALL_DONE
