#!/bin/bash
# Diagnostic builds of band_h2ws (SMCV_WS_ABL bits, see ip_h2ws.hip) linked with the library's
# other objects: bin/ab/lib_ws<N>.so.   bash scripts/build_ab_ws.sh 0 1 2 ...
set -e
cd "$(dirname "$0")/.."
python -m realtime_stereo_matcher_amd.build_lib > /dev/null
mkdir -p bin/ab /tmp/ab_ws
OBJS=$(ls build/stereocv/*.o | grep -v ip_h2ws.o)
for n in "$@"; do
  /opt/rocm/bin/hipcc -O3 -std=c++20 -fPIC --offload-arch=gfx950 -I include -Wall -Wno-unused-function \
    -DSMCV_WS_ABL=$n -c realtime_stereo_matcher_amd/csrc/ip_h2ws.hip -o /tmp/ab_ws/ws$n.o
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $OBJS /tmp/ab_ws/ws$n.o -o bin/ab/lib_ws$n.so
  echo "bin/ab/lib_ws$n.so"
done
