set -u
OUT=gpurun_out/a22
mkdir -p $OUT
V=yocto_raytracing_amd/variants
run() { tag=$1; shift; timeout -k 10 240 python tools/ab_variants.py --rounds 7 "$@" $V/libyrt_st0.so $V/libyrt_st32.so $V/libyrt_st16.so $V/libyrt_st8.so > $OUT/ab_$tag.txt 2>&1; rc=$?; grep -v '^{' $OUT/ab_$tag.txt | grep -v amdgpu.ids | sed "s/^/$tag /"; return $rc; }
run c4_r0of8 --share 0/8 && run c4 && run c4_r0of4 --share 0/4 && run c3 --scene refl --samples 4 && run i100k --scene instance100k
