set -u
mkdir -p gpurun_out/r6c
timeout -k 10 300 python -u -m pytest tests/test_gpu_lists.py tests/test_gpu_list_margins.py tests/test_gpu_instance_masks.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6c/pytest.log 2>&1 || { tail -n 30 gpurun_out/r6c/pytest.log; exit 1; }
tail -n 1 gpurun_out/r6c/pytest.log
bash tools/gpu/ab_scenes.sh r6c tools/gpu/specs/r6c.txt --no-suite
