set -u
OUT=gpurun_out/a27
mkdir -p $OUT
V=yocto_raytracing_amd/variants
run() { tag=$1; shift; timeout -k 10 240 python tools/ab_variants.py --rounds 7 "$@" $V/libyrt_main.so@off $V/libyrt_main.so@on $V/libyrt_nocam.so@on > $OUT/ab_$tag.txt 2>&1; rc=$?; grep -v '^{' $OUT/ab_$tag.txt | grep -v amdgpu.ids | sed "s/^/$tag /"; return $rc; }
run i100k --scene instance100k && run c4 && run i1k --scene instance1k
