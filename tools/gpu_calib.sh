#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration of the fused env-step kernel's access widths and of the
# instruction fetch (tools/fetch_calib.hip), at the bench size and past the Infinity Cache
source "$(dirname "$0")/gpu_lib.sh"
RP="rocprofv3 --output-format csv"
for N in ${NS:-4096 1048576}; do
  run calf_$N 60 $RP --pmc FETCH_SIZE --kernel-trace -d gpurun_out/calf_$N -o run -- tools/fetch_calib $N 6
  [ -z "$NOWRITE" ] && run calw_$N 60 $RP --pmc WRITE_SIZE --kernel-trace -d gpurun_out/calw_$N -o run -- tools/fetch_calib $N 6
done
echo ALL_DONE
