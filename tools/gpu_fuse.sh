#!/bin/bash
# obs/reward fuse kernel: parity (modular path), HBM roofline sweep, rocprof stats + PMC traffic
source "$(dirname "$0")/gpu_lib.sh"
RP="rocprofv3 --output-format csv"
run pytest_post 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dr.py -x -q --timeout 120 --timeout-method thread
run fuse_h 300 python -u tools/fuse_roofline.py Humanoid 4096,65536,262144,1048576
run fuse_a 300 python -u tools/fuse_roofline.py Ant 4096,65536,262144,1048576
run prof_fuse 300 $RP --kernel-trace --stats -d gpurun_out/prof_fuse -o run -- python3 tools/fuse_roofline.py Humanoid 1048576 20
run pmcf_fuse 300 $RP --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmcf_fuse -o run -- python3 tools/fuse_roofline.py Humanoid 1048576 10
run pmcw_fuse 300 $RP --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmcw_fuse -o run -- python3 tools/fuse_roofline.py Humanoid 1048576 10
echo ALL_DONE
