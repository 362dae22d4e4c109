#!/bin/bash
# Cartpole fused env step (one lane per env) across N: HBM roofline of BASELINE config 1's kernel
source "$(dirname "$0")/gpu_lib.sh"
run sweep_cartpole 600 python -u tools/bw_sweep.py Cartpole 4096,65536,1048576,4194304,16777216
echo ALL_DONE
