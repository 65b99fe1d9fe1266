set -u
mkdir -p gpurun_out/a1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/a1/pytest.log 2>&1
rc=$?; tail -n 3 gpurun_out/a1/pytest.log; if [ $rc -ne 0 ]; then exit $rc; fi
AB_LIBS="base bfs l255 l511 l1023 w6 w7 h16" PMC_LIBS="bfs l1023 w6" bash tools/gpu_ab_pmc.sh a1 instance10000 instance100k
