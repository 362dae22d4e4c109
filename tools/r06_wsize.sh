#!/bin/bash
# round 6: WRITE_SIZE of the fused Humanoid step at 4096 envs under {pairing by load, index
# pairing} x {TGS, PGS} (one rocprofv3 PMC pass each)
export TMPDIR=/tmp
mkdir -p gpurun_out/r06/wsize
for sv in tgs pgs; do
  for pl in 1 0; do
    B="python3 bench.py --task Humanoid --num-envs 4096 --steps 30 --warmup 5 --no-cpu-baseline --no-side --fuse-envs 0 --solver $sv"
    MI_PAIR_LOAD=$pl timeout -s KILL 90 rocprofv3 --output-format csv --pmc WRITE_SIZE --kernel-trace \
      -d gpurun_out/r06/wsize/w_${sv}_pl$pl -o run -- $B > gpurun_out/r06/wsize/w_${sv}_pl$pl.log 2>&1 || exit $?
  done
done
