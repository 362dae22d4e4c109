#!/bin/bash
# First GPU pass: parity tests, smoke, bench (Humanoid 4096), rocprofv3 kernel stats.
source "$(dirname "$0")/gpu_lib.sh"
python -c "import torch; print(torch.cuda.get_device_name(0))" > gpurun_out/device.txt 2>&1
run pytest_gpu 300 python -u -m pytest tests -m gpu -x -q
run smoke 150 python -u -c "import __graft_entry__ as g; g.smoke()"
run bench_humanoid 250 python -u bench.py --steps 200 --warmup 20 --cpu-seconds 6
run bench_ant 120 python -u bench.py --task Ant --steps 200 --warmup 20 --no-cpu-baseline
run bench_cartpole 100 python -u bench.py --task Cartpole --steps 200 --warmup 20 --no-cpu-baseline
run rocprof_humanoid 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_humanoid -o run -- python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline
echo ALL_DONE
