#!/bin/bash
# round 6: PGS row step as two FMAs around the projection (MI_PAIR_SWEEP_FMA) — parity /
# pairing / free-run tests on the new library, then bench A/B against the previous build
export TMPDIR=/tmp
O=gpurun_out/r06/sweep
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_pairing.py tests/test_gpu_parity.py tests/test_gpu_freerun.py tests/test_gpu_fullsize.py > $O/tests.log 2>&1 || exit $?
B="python3 -u bench.py --task Humanoid --steps 300 --warmup 30 --no-cpu-baseline --no-side --fuse-envs 0"
for k in 1 2 3; do
  timeout -k 10 200 $B > $O/ab_new_$k.log 2>&1 || exit $?
  MI_SIM_LIB=ab/libmi_sim_base.so timeout -k 10 200 $B > $O/ab_base_$k.log 2>&1 || exit $?
done
grep -h '"kernel_ms"' $O/ab_*.log | sed 's/.*"kernel_ms": \([0-9.]*\).*/\1/' > /dev/null
