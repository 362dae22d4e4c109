#!/bin/bash
# round 6 final measurements at HEAD: the GPU suite, smoke, the default bench line and its
# rocprofv3 kernel statistics, the PMC traffic sweep, SQ counters and the slowest-wave stamps
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}"
PYTEST_X= bash tools/gpu.sh tests smoke bench prof || exit $?
TAG=r06 bash tools/gpu.sh traffic sq tail || exit $?
echo ALL_FINAL_DONE
