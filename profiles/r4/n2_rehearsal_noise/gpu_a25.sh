set -u
OUT=gpurun_out/a25
mkdir -p $OUT
V=yocto_raytracing_amd/variants
for lib in $V/libyrt_fin.so yocto_raytracing_amd/libyrt.so $V/libyrt_fin.so yocto_raytracing_amd/libyrt.so; do
YRT_LIB=$lib YRT_BENCH_DEVICES=1 YRT_BENCH_BACKEND=gloo YRT_BENCH_OVERLAP=1 timeout -k 10 300 python bench.py --gpus 2 --steps 3 --warmup 1 --cpu-seconds 0 > $OUT/n2.json 2> $OUT/n2.err
rc=$?; echo "$lib rc=$rc $(grep -h '^{' $OUT/n2.json | python -c 'import json,sys; j=json.loads(sys.stdin.read()); print(round(j["ms_per_step"],1), {k: round(v,1) for k,v in j["config"]["phase_ms_per_frame"].items()})')"; if [ $rc -ne 0 ]; then exit $rc; fi
done
