#!/bin/bash
# GPU box: in-process A/B of the given libraries (tools/ab_variants.py) on the given scenes
# (comma-separated), stopping at the first failing step.
#   bash tools/gpu/ab_only.sh TAG ROUNDS SCENES [ab_variants args --] lib1.so lib2.so ...
set -u
TAG=$1; ROUNDS=$2; SCENES=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p $OUT
for sc in ${SCENES//,/ }; do
  timeout -k 10 300 python -u tools/ab_variants.py --rounds $ROUNDS --scene $sc "$@" > $OUT/ab_$sc.txt 2>&1 || { tail -n 20 $OUT/ab_$sc.txt; exit 1; }
  echo "== $sc"; grep image $OUT/ab_$sc.txt
done
