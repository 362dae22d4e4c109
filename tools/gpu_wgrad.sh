#!/bin/bash
source tools/gpu_lib.sh
run wgrad 200 python -u tools/wgrad_bench.py
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tun_wg.csv run wgrad_tuned 400 python -u tools/wgrad_bench.py
echo ALL_DONE
