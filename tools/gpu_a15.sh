set -u
OUT=gpurun_out/a15
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_lists.py -v -s --timeout 240 --timeout-method thread > $OUT/lists.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|bit-exact|passed|failed" $OUT/lists.log | tail -30; if [ $rc -ne 0 ]; then tail -60 $OUT/lists.log; exit $rc; fi
