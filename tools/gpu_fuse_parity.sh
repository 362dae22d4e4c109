source tools/gpu_lib.sh
run pytest_fuse 300 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 200 --timeout-method thread -k "fuse"
echo ALL_DONE
