set -u
mkdir -p gpurun_out/r5y
timeout -k 10 300 python -u -m pytest tests/test_gpu_lds_staging.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/r5y/pytest_lds.log 2>&1 || { tail -n 40 gpurun_out/r5y/pytest_lds.log; exit 1; }
tail -n 3 gpurun_out/r5y/pytest_lds.log
bash tools/gpu/ab_scenes.sh r5y tools/gpu/specs/r5y.txt --no-suite
