set -o pipefail
mkdir -p gpurun_out
R=$PWD/omniisaacgymenvs_amd
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -k "write_batching or setters or mirrors or deferred" > gpurun_out/pytest_view.log 2>&1 && tail -2 gpurun_out/pytest_view.log && \
timeout -k 10 120 python -u tools/hash_run.py > gpurun_out/hash_a.log 2>&1 && \
MI_SIM_LIB=$R/libmi_sim_b.so timeout -k 10 120 python -u tools/hash_run.py > gpurun_out/hash_b.log 2>&1 && \
grep HASH gpurun_out/hash_a.log > gpurun_out/ha.txt && grep HASH gpurun_out/hash_b.log > gpurun_out/hb.txt && \
(cmp gpurun_out/ha.txt gpurun_out/hb.txt && echo HASH_SAME || echo HASH_DIFF) && \
timeout -k 10 200 python -u tools/path_a_timing.py Humanoid 4096 200 > gpurun_out/path_a.log 2>&1 && tail -c 600 gpurun_out/path_a.log && \
MI_SIM_BATCH_WRITES=0 timeout -k 10 200 python -u tools/path_a_timing.py Humanoid 4096 200 > gpurun_out/path_a_nobatch.log 2>&1 && tail -c 600 gpurun_out/path_a_nobatch.log && \
LIBS="$R/libmi_sim_b.so $R/libmi_sim_ap16.so $R/libmi_sim_wpd8.so" TAG=upd TASK=Humanoid bash tools/gpu.sh abn && \
TAG=upd bash tools/gpu.sh tail
