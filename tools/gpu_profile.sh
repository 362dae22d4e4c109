#!/bin/bash
# GPU-box profiling pass: phase stamps, rocprofv3 kernel-trace stats, PMC HBM traffic passes
# (FETCH_SIZE and WRITE_SIZE in separate runs: they do not fit one TCC pass), SQ issue/wait
# counters, then the default bench line (with the CPU baseline). Each step time-limited.
source "$(dirname "$0")/gpu_lib.sh"
RP="rocprofv3 --output-format csv"
run stamps_humanoid 150 python -u tools/phase_stamps.py Humanoid 4096
run stamps_ant 150 python -u tools/phase_stamps.py Ant 4096
for T in Humanoid Ant Cartpole; do
  run prof_$T 300 $RP --kernel-trace --stats -d gpurun_out/prof_$T -o run -- \
      python3 bench.py --task $T --steps 200 --warmup 20 --no-cpu-baseline --fuse-envs 0
  run pmcf_$T 300 $RP --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmcf_$T -o run -- \
      python3 bench.py --task $T --steps 40 --warmup 5 --no-cpu-baseline --fuse-envs 0
  run pmcw_$T 300 $RP --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmcw_$T -o run -- \
      python3 bench.py --task $T --steps 40 --warmup 5 --no-cpu-baseline --fuse-envs 0
done
run sq1 300 $RP --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-trace -d gpurun_out/sq1 -o run -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --fuse-envs 0
run sq2 300 $RP --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/sq2 -o run -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --fuse-envs 0
run fuse_h 300 python -u tools/fuse_roofline.py Humanoid 4096,65536,262144,1048576
run fuse_a 300 python -u tools/fuse_roofline.py Ant 4096,65536,262144,1048576
run prof_fuse 300 $RP --kernel-trace --stats -d gpurun_out/prof_fuse -o run -- python3 tools/fuse_roofline.py Humanoid 1048576 20
run pmcf_fuse 300 $RP --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmcf_fuse -o run -- python3 tools/fuse_roofline.py Humanoid 1048576 10
run pmcw_fuse 300 $RP --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmcw_fuse -o run -- python3 tools/fuse_roofline.py Humanoid 1048576 10
run bench_default 500 python -u bench.py
echo ALL_DONE
