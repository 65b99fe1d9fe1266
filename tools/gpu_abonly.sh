#!/bin/bash
# GPU box: in-process A/B of library variants only (tools/ab_variants.py), optional
# extra ab_variants arguments via AB_ARGS (e.g. "--scene refl --samples 4").
#   bash tools/gpu_abonly.sh TAG lib.so ...
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 500 python tools/ab_variants.py --rounds ${AB_ROUNDS:-5} ${AB_ARGS:-} "$@" > $OUT/ab.txt 2>&1
rc=$?
grep -v '^{' $OUT/ab.txt | grep -v amdgpu.ids
exit $rc
