#!/bin/bash
# round 6: the default library's parity / pairing / free-run / full-size tests, then
# tools/r06_abn.sh over LIBS
export TMPDIR=/tmp
O=gpurun_out/r06/${ABN_TAG:-abn}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_pairing.py tests/test_gpu_parity.py tests/test_gpu_freerun.py tests/test_gpu_fullsize.py > $O/tests.log 2>&1 || exit $?
tail -1 $O/tests.log
bash tools/r06_abn.sh
