#!/bin/bash
# iteration loop: GPU tests, Humanoid / Ant bench, phase stamps, Humanoid PMC traffic passes
source "$(dirname "$0")/gpu_lib.sh"
run pytest_gpu 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run bench_humanoid 200 python -u bench.py --steps 300 --warmup 50 --no-cpu-baseline --fuse-envs 0
run bench_ant 150 python -u bench.py --task Ant --steps 300 --warmup 50 --no-cpu-baseline --fuse-envs 0
run stamps_humanoid 150 python -u tools/phase_stamps.py Humanoid 4096
RP="rocprofv3 --output-format csv"
run pmcf_Humanoid 120 $RP --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmcf_Humanoid -o run -- python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline --fuse-envs 0
run pmcw_Humanoid 120 $RP --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmcw_Humanoid -o run -- python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline --fuse-envs 0
echo ALL_DONE
