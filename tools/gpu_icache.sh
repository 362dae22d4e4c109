#!/bin/bash
# instruction-cache and issue counters of the fused env-step kernel (Humanoid bench), one PMC
# pass per block: SQC (I-cache), SQ (wave-cycle split, instruction fetch)
source "$(dirname "$0")/gpu_lib.sh"
B="python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --fuse-envs 0 --no-side ${BARGS:-}"
RP="rocprofv3 --output-format csv --kernel-trace"
T=${TAG:-cur}
run ic1_$T 90 timeout -s KILL 80 $RP --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE -d gpurun_out/ic1_$T -o run -- $B
run ic2_$T 90 timeout -s KILL 80 $RP --pmc SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU -d gpurun_out/ic2_$T -o run -- $B
echo ALL_DONE
