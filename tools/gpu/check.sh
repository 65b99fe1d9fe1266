#!/bin/bash
# GPU box: the -m gpu suite, then (unless it faulted) the default bench line.
#   bash tools/gpu/check.sh TAG [bench args...]
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -n 3 $OUT/pytest.log
# no further GPU step after a fault, an abort or a time limit
if grep -q "illegal memory\|Aborted\|Segmentation\|Timeout" $OUT/pytest.log || [ $rc -ge 124 ]; then
  exit 1
fi
timeout -k 10 300 python bench.py --cpu-seconds 0 "$@" > $OUT/bench.json 2> $OUT/bench.err
