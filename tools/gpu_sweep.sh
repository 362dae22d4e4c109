#!/bin/bash
source "$(dirname "$0")/gpu_lib.sh"
run sweep_h 500 python -u tools/bw_sweep.py Humanoid 1024,2048,3072,4096,6144,8192,16384,65536
echo ALL_DONE
