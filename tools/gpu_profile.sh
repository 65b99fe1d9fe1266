#!/bin/bash
# Round profile on the GPU box: kernel-trace stats of the bench, then the two PMC
# passes (FETCH_SIZE, WRITE_SIZE) in separate runs, summarised into traffic json.
#   bash tools/gpu_profile.sh TAG [bench args...]
set -euo pipefail
TAG=$1; shift
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
B="bench.py --steps 3 --warmup 1 --cpu-seconds 0 $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ks -o ks -- python3 $B > $OUT/ks.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/p3 -o p3 -- python3 $B > $OUT/p3.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/p4 -o p4 -- python3 $B > $OUT/p4.log 2>&1
find $OUT -name '*.csv' | sort
