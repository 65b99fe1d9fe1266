set -u
V=yocto_raytracing_amd/variants
for lib in "" $V/libyrt_v8s.so $V/libyrt_call5.so "" $V/libyrt_v8s.so; do
  if [ -n "$lib" ]; then export YRT_LIB=$lib; else unset YRT_LIB; fi
  YRT_BENCH_DEVICES=1 YRT_BENCH_BACKEND=gloo YRT_BENCH_OVERLAP=1 timeout -k 10 300 python bench.py --gpus 2 --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/n2.tmp 2>/dev/null || exit 1
  python3 -c "
import json,sys
for l in open('gpurun_out/n2.tmp'):
    if l.startswith('{'):
        d=json.loads(l); c=d['config']; print('${lib:-current}', round(d['value']), round(d['ms_per_step'],2), {k:round(v,2) for k,v in c['phase_ms_per_frame'].items()}, round(c['gpu_ms_per_frame'],2))" >> gpurun_out/n2_ab.txt
done
