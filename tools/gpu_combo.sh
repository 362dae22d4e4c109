set -e
bash tools/gpu_calib.sh
TASK=Ant bash tools/gpu_traffic_sweep.sh
TASK=Cartpole bash tools/gpu_traffic_sweep.sh
