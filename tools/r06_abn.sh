#!/bin/bash
# round 6: bench A/B/C.. of library builds (LIBS="name:path ..."), alternating passes
export TMPDIR=/tmp
O=gpurun_out/r06/${ABN_TAG:-abn}
mkdir -p $O
B="python3 -u bench.py --task ${TASK:-Humanoid} --steps 300 --warmup 30 --no-cpu-baseline --no-side --fuse-envs 0"
for k in 1 2 3; do
  for e in $LIBS; do
    n=${e%%:*}; l=${e#*:}
    MI_SIM_LIB=$l timeout -k 10 200 $B > $O/${n}_$k.log 2>&1 || exit $?
  done
done
for e in $LIBS; do n=${e%%:*}; echo "$n $(grep -ho '"kernel_ms": [0-9.]*' $O/${n}_*.log | awk '{printf "%s ", $2}')"; done
