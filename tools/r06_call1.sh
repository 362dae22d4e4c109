set -o pipefail
mkdir -p gpurun_out/r06/c1
O=gpurun_out/r06/c1
true && \
true && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pairing.py tests/test_gpu_shard_world2.py tests/test_gpu_policy.py tests/test_gpu_dp_world2.py tests/test_cpu_pipeline_cartpole.py -m gpu > $O/new_tests.log 2>&1 && \
for k in 1 2; do for st in 1 0; do MI_STAGE_OUT=$st timeout -k 10 300 python -u bench.py > $O/bench_stage${st}_$k.log 2>&1 || exit 1; done; done
