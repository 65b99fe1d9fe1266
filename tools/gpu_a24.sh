set -u
OUT=gpurun_out/a24
mkdir -p $OUT
V=yocto_raytracing_amd/variants
run() { tag=$1; shift; timeout -k 10 240 python tools/ab_variants.py --rounds 7 "$@" $V/libyrt_fin.so $V/libyrt_sort.so $V/libyrt_sortd.so $V/libyrt_sortc.so > $OUT/ab_$tag.txt 2>&1; rc=$?; grep -v '^{' $OUT/ab_$tag.txt | grep -v amdgpu.ids | sed "s/^/$tag /"; return $rc; }
run c4 && run i1k --scene instance1k && run i100k --scene instance100k
