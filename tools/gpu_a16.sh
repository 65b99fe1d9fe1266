set -u
OUT=gpurun_out/a16
mkdir -p $OUT
V=yocto_raytracing_amd/variants
for sh in 0/8 0/4 0/2; do
n=${sh#0/}
timeout -k 10 200 python tools/ab_variants.py --rounds 5 --share $sh $V/libyrt_cur.so@auto $V/libyrt_cur.so@off $V/libyrt_pall.so@auto $V/libyrt_pall.so@off > $OUT/ab_r0of$n.txt 2>&1
rc=$?; grep -v '^{' $OUT/ab_r0of$n.txt | grep -v amdgpu.ids; if [ $rc -ne 0 ]; then exit $rc; fi
done
