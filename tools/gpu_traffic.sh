#!/bin/bash
# parity tests, per-task bench, and the FETCH/WRITE PMC passes of the fused env-step kernel
source "$(dirname "$0")/gpu_lib.sh"
RP="rocprofv3 --output-format csv"
[ -z "$NOTEST" ] && run pytest_gpu 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
for T in ${TASKS:-Humanoid Ant Cartpole}; do
  run bench_$T 200 python -u bench.py --task $T --steps 200 --warmup 20 --no-cpu-baseline --no-side --fuse-envs 0
  run pmcf_$T 120 $RP --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmcf_$T -o run -- \
      python3 bench.py --task $T --steps 40 --warmup 5 --no-cpu-baseline --no-side --fuse-envs 0
  run pmcw_$T 120 $RP --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmcw_$T -o run -- \
      python3 bench.py --task $T --steps 40 --warmup 5 --no-cpu-baseline --no-side --fuse-envs 0
done
echo ALL_DONE
