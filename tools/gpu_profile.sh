#!/bin/bash
# GPU-box profiling pass: phase stamps, rocprofv3 kernel-trace stats, PMC HBM traffic passes
# (FETCH_SIZE and WRITE_SIZE in separate runs: they do not fit one TCC pass), then the
# default bench line (with the CPU baseline). Every step under its own time limit.
source "$(dirname "$0")/gpu_lib.sh"
run stamps_humanoid 150 python -u tools/phase_stamps.py Humanoid 4096
run stamps_ant 150 python -u tools/phase_stamps.py Ant 4096
for T in Humanoid Ant Cartpole; do
  run prof_$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o run -- \
      python3 bench.py --task $T --steps 200 --warmup 20 --no-cpu-baseline
  run pmcf_$T 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmcf_$T -o run -- \
      python3 bench.py --task $T --steps 40 --warmup 5 --no-cpu-baseline
  run pmcw_$T 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmcw_$T -o run -- \
      python3 bench.py --task $T --steps 40 --warmup 5 --no-cpu-baseline
done
run bench_default 500 python -u bench.py
echo ALL_DONE
