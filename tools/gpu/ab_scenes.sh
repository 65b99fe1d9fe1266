#!/bin/bash
# GPU box: the -m gpu suite, then in-process A/B runs (tools/ab_variants.py), one per line of
# the spec file: "<name> <ab_variants.py args...>" (libraries and their @lists modes included).
# Stops at the first failing GPU step.
#   bash tools/gpu/ab_scenes.sh TAG SPEC [--no-suite]
set -u
TAG=$1; SPEC=$2; SUITE=${3:-}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ "$SUITE" != "--no-suite" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 \
    || { tail -n 30 $OUT/pytest.log; exit 1; }
  tail -n 2 $OUT/pytest.log
fi
while read -r name args; do
  [ -z "$name" ] && continue
  case "$name" in \#*) continue;; esac
  timeout -k 10 240 python -u tools/ab_variants.py $args > $OUT/ab_$name.txt 2>&1 || { tail -n 20 $OUT/ab_$name.txt; exit 1; }
  echo "== $name"; grep image $OUT/ab_$name.txt
done < "$SPEC"
