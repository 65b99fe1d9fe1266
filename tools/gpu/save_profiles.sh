#!/bin/bash
# Copy one tools/gpu/evidence.sh run's evidence from gpurun_out/TAG into
# profiles/ROUND/TAG: bench lines, logs, counter CSVs, kernel stats and summaries (the
# run's raw rocprofv3 output directories stay in gpurun_out/).
#   bash tools/gpu/save_profiles.sh TAG [ROUND]     (ROUND: r6 by default)
set -eu
TAG=$1; ROUND=${2:-r6}
S=gpurun_out/$TAG; D=profiles/$ROUND/$TAG
mkdir -p $D
for f in $S/*.json $S/pytest*.log $S/smoke.log; do [ -e "$f" ] && cp "$f" $D/; done
for p in $S/pmc_*/; do
  n=$(basename $p); mkdir -p $D/$n
  cp $p/p*/p*_counter_collection.csv $p/ks/ks_kernel_stats.csv $p/summary.json $D/$n/
done
[ -e $S/issue_counters.json ] && cp $S/issue_counters.json $S/pmc_traffic.json profiles/
ls $D
