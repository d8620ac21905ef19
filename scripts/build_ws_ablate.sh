#!/bin/bash
# Build ws ablation binaries in this container (parallel); they run on the GPU box from bin/.
#   bash scripts/build_ws_ablate.sh "NAME:FLAGS ..."   e.g. "a0:-DSMCV_ABLATE=0 nb7:-DSMCV_WS_NB=7"
cd "$(dirname "$0")/.." || exit 1
mkdir -p bin
for spec in $1; do
  name=${spec%%:*}; flags=${spec#*:}; flags=${flags//,/ }
  /opt/rocm/bin/hipcc -O3 -std=c++20 --offload-arch=gfx950 $flags -Iinclude scripts/ws_ablate.hip -o bin/wsa_$name > bin/wsa_$name.log 2>&1 &
done
wait
ls -la bin/ | grep wsa_ | grep -v log
