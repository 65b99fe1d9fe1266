set -u
OUT=gpurun_out/a26
mkdir -p $OUT
V=yocto_raytracing_amd/variants
run() { tag=$1; shift; timeout -k 10 240 python tools/ab_variants.py --rounds 7 "$@" $V/libyrt_head.so $V/libyrt_ref0.so $V/libyrt_sup.so > $OUT/ab_$tag.txt 2>&1; rc=$?; grep -v '^{' $OUT/ab_$tag.txt | grep -v amdgpu.ids | sed "s/^/$tag /"; return $rc; }
run c4 && run i1k --scene instance1k && run c4_r0of8 --share 0/8 && run c5_r0of8 --resolution 4096 --width 4096 --samples 16 --share 0/8 --rounds 3
