#!/bin/bash
# GPU box: the -m gpu suite + smoke, an in-process A/B of library variants at c4
# (tools/ab_variants.py: per-phase ms and the image digest of each), then the default
# bench line. Every GPU step has its own time limit; a failing step ends the script.
#   bash tools/gpu_ab.sh TAG [lib.so ...]
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
run() { "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "FAILED (rc=$rc): $*"; exit $rc; fi; }
run timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
tail -n 2 $OUT/pytest.log
run timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
cat $OUT/smoke.log
if [ $# -gt 0 ]; then
  run timeout -k 10 400 python tools/ab_variants.py --rounds ${AB_ROUNDS:-5} "$@" > $OUT/ab.txt 2>&1
  grep -v '^{' $OUT/ab.txt
fi
run timeout -k 10 300 python bench.py --cpu-seconds 0 > $OUT/bench.json 2> $OUT/bench.err
cut -c1-600 $OUT/bench.json
