#!/bin/bash
source "$(dirname "$0")/gpu_lib.sh"
run stamps_humanoid 150 python -u tools/phase_stamps.py Humanoid 4096
run stamps_ant 150 python -u tools/phase_stamps.py Ant 4096
echo ALL_DONE
