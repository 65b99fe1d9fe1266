#!/bin/bash
# GPU box: the -m gpu suite, then in-process A/B of the given libraries at c4, instance1k and
# instance100k (tools/ab_variants.py). Stops at the first failing GPU step.
#   bash tools/gpu/ab_quick.sh TAG ROUNDS lib1.so lib2.so ...
set -u
TAG=$1; ROUNDS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -n 30 $OUT/pytest.log; exit 1; }
tail -n 2 $OUT/pytest.log
for sc in instance10000 instance1k instance100k; do
  timeout -k 10 240 python -u tools/ab_variants.py --rounds $ROUNDS --scene $sc "$@" > $OUT/ab_$sc.txt 2>&1 || { tail -n 20 $OUT/ab_$sc.txt; exit 1; }
  grep image $OUT/ab_$sc.txt
done
