#!/bin/bash
# GPU box, one call: the -m gpu suite, the default bench line (CPU baselines included),
# then the roofline counter passes. Every GPU step has its own time limit; after a fault,
# an abort or a time limit nothing else runs.
#   bash tools/gpu_round.sh TAG [pytest selection...]
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" > $OUT/pytest.log 2>&1
rc=$?
tail -n 5 $OUT/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?
cat $OUT/bench.json
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_issue_pmc.sh $TAG/pmc_c4
