#!/bin/bash
# Counter passes (one rocprofv3 run per group, kernel trace only -- never combined with
# sys/runtime traces) over a short bench run.
#   bash tools/gpu_pmc.sh TAG "CTR1 CTR2 ..." ["CTR ..." ...] -- [bench args]
set -euo pipefail
TAG=$1; shift
groups=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do groups+=("$1"); shift; done
[ "${1:-}" = "--" ] && shift
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
i=0
for g in "${groups[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $g --output-format csv -d $OUT/g$i -o g$i -- \
    python3 bench.py --steps 1 --warmup 0 --cpu-seconds 0 "$@" > $OUT/g$i.log 2>&1
done
find $OUT -name '*counter_collection.csv' | sort
