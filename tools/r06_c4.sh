#!/bin/bash
# round 6: spill-free paired kernel (wide AREG 28) — bit-identity, GPU suite, traffic sweep,
# kernel-trace stats and the default bench line
export TMPDIR=/tmp
mkdir -p gpurun_out/r06/c4
timeout -k 10 300 python -u tools/hash_run.py > gpurun_out/r06/c4/hash.log 2>&1 || exit $?
PYTEST_X= bash tools/gpu.sh tests || exit $?
bash tools/gpu.sh traffic || exit $?
bash tools/gpu.sh prof || exit $?
bash tools/gpu.sh bench || exit $?
