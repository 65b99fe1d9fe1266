#!/bin/bash
# SQ instruction counters of the shadow kernel for several builds (one rocprofv3 pass each)
set -u
export TMPDIR=/tmp
for lib in "$@"; do
  n=$(basename $lib .so)
  YRT_LIB=$lib timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_SMEM SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_ab/$n -o p -- python3 bench.py --steps 1 --warmup 0 --cpu-seconds 0 > gpurun_out/pmc_ab/$n.log 2>&1 || exit 1
  python3 - gpurun_out/pmc_ab/$n <<'PY'
import csv,glob,sys,collections
f=glob.glob(sys.argv[1]+'/**/*counter_collection.csv',recursive=True)[0]
acc=collections.defaultdict(float); cnt=collections.Counter()
for r in csv.DictReader(open(f)):
    k=r['Kernel_Name'][:40]
    acc[(k,r['Counter_Name'])]+=float(r['Counter_Value'])
    cnt[k]+=1
for (k,c),v in sorted(acc.items()):
    if 'shadow' in k or 'primary' in k: print(sys.argv[1].split('/')[-1],k,c,'%.4g'%v)
PY
done
