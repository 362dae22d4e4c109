#!/bin/bash
# round 6: device-vs-oracle error distribution with 4 oracle-side sensitivity probes, per-env dumps
# (tools/parity_stats.py), Humanoid / Ant under TGS and PGS, 8 steps x 4096 envs each
mkdir -p gpurun_out/r06
for t in Humanoid Ant; do
  for s in tgs pgs; do
    echo "== $t $s"
    PARITY_PROBES=${PROBES:-4} PARITY_DUMP=gpurun_out/r06/pp8_${t}_${s}.npz timeout -k 10 600 \
      python -u tools/parity_stats.py $t 4096 ${STEPS:-8} $s > gpurun_out/r06/pp8_${t}_${s}.log 2>&1 || exit 1
  done
done
