#!/bin/bash
# round 6: PMC traffic of the fused Humanoid step, staged outputs on (default) over the env-count
# sweep, then MI_STAGE_OUT=0 at 4096 envs for the A/B (tools/gpu.sh traffic recipe)
set -o pipefail
bash tools/gpu.sh traffic || exit $?
mkdir -p gpurun_out/r06/tr_on gpurun_out/r06/tr_off
mv gpurun_out/ts[fw]_Humanoid_* gpurun_out/r06/tr_on/ || exit 1
MI_STAGE_OUT=0 NS=4096 bash tools/gpu.sh traffic || exit $?
mv gpurun_out/ts[fw]_Humanoid_* gpurun_out/r06/tr_off/
