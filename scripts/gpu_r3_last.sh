#!/bin/bash
# Last round-3 GPU call: the driver's steps (gpu_final.sh), the fused bench lines, and a same-box
# A/B of the fused-with-volume pass on band_h2 (bin/ab/lib_h2fuse.so) vs band_h2db.
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r3_final5}; OUT=gpurun_out/$TAG
bash scripts/gpu_final.sh "$TAG" || exit 2
timeout -k 10 300 python bench.py --pipeline fused > "$OUT/bench_fused.json" 2> "$OUT/bench_fused.err" || exit 3
timeout -k 10 300 python bench.py --pipeline fused-novolume > "$OUT/bench_fused_nv.json" 2> "$OUT/bench_fused_nv.err" || exit 4
tail -c 200 "$OUT/bench_fused.json"
bash scripts/gpu_ab_ops.sh "$TAG/ab_fused" cfg2_fused bin/ab/lib_h2fuse.so realtime_stereo_matcher_amd/libstereocv.so || exit 5
