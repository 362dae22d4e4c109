#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the fused env-step kernel over the env count: the per-env slope and
# the per-launch intercept split the traffic into per-env bytes and fixed per-launch bytes
source "$(dirname "$0")/gpu_lib.sh"
RP="rocprofv3 --output-format csv --kernel-trace"
T=${TASK:-Humanoid}
for N in ${NS:-1024 2048 4096 8192 16384}; do
  B="python3 bench.py --task $T --num-envs $N --steps 30 --warmup 5 --no-cpu-baseline --no-side --fuse-envs 0"
  run tsf_${T}_$N 100 timeout -s KILL 90 $RP --pmc FETCH_SIZE -d gpurun_out/tsf_${T}_$N -o run -- $B
  run tsw_${T}_$N 100 timeout -s KILL 90 $RP --pmc WRITE_SIZE -d gpurun_out/tsw_${T}_$N -o run -- $B
done
echo ALL_DONE
