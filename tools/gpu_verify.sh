#!/bin/bash
# Full round-end rehearsal: every GPU test, smoke, default bench line.
source "$(dirname "$0")/gpu_lib.sh"
run pytest_gpu 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
run smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
run bench_default 500 python -u bench.py
echo ALL_DONE
