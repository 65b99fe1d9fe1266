set -u
OUT=gpurun_out/a19
mkdir -p $OUT
V=yocto_raytracing_amd/variants
for sh in 0/1 0/8; do
timeout -k 10 120 python tools/tail_stats.py $V/libyrt_tail.so --share $sh > $OUT/tail_${sh/\//of}.txt 2>&1
rc=$?; grep -v amdgpu.ids $OUT/tail_${sh/\//of}.txt; if [ $rc -ne 0 ]; then exit $rc; fi
done
