source tools/gpu_lib.sh
run st_h 150 python -u tools/phase_stamps.py Humanoid 4096
grep -v "^{" gpurun_out/st_h.log | tail -20
