#!/bin/bash
set -u
OUT=gpurun_out/s3; mkdir -p $OUT
V=yocto_raytracing_amd/variants
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -n 40 $OUT/pytest.log; exit 1; }
tail -n 2 $OUT/pytest.log
ab() { local tag=$1 sc=$2; shift 2; timeout -k 10 300 python -u tools/ab_variants.py --rounds 7 --scene $sc "$@" > $OUT/ab_$tag.txt 2>&1 || { tail -n 20 $OUT/ab_$tag.txt; exit 1; }; echo "== $tag"; grep image $OUT/ab_$tag.txt; }
ab tree100k instance100k $V/libyrt_r4.so $V/libyrt_s1.so $V/libyrt_lane0.so $V/libyrt_uorig0.so $V/libyrt_surf0.so $V/libyrt_vconst0.so $V/libyrt_idx0.so $V/libyrt_f32.so
ab on100k instance100k $V/libyrt_r4.so $V/libyrt_r4.so@on $V/libyrt_f32.so@on $V/libyrt_f16.so@on $V/libyrt_f8.so@on $V/libyrt_f4.so@on
ab c4 instance10000 $V/libyrt_r4.so $V/libyrt_f32.so $V/libyrt_f16.so $V/libyrt_f8.so $V/libyrt_f4.so $V/libyrt_f32.so@off
ab on1k instance1k $V/libyrt_r4.so $V/libyrt_f32.so@on $V/libyrt_f16.so@on $V/libyrt_f8.so@on $V/libyrt_f4.so@on
