#!/bin/bash
# Diagnostic builds of scripts/ip_stamps.hip (here, on the CPU): the phase-stamp binary and one
# binary per SMCV_ABLATE value given (default 0 1 2 4 8 16), into bin/stamps/.
cd "$(dirname "$0")/.." || exit 1
mkdir -p bin/stamps
hipcc -O3 -std=c++20 --offload-arch=gfx950 -DSMCV_STAMPS -Iinclude scripts/ip_stamps.hip -o bin/stamps/ip_stamps &
for ab in ${@:-0 1 2 4 8 16}; do
  hipcc -O3 -std=c++20 --offload-arch=gfx950 -DSMCV_ABLATE=$ab -Iinclude scripts/ip_stamps.hip -o bin/stamps/ip_ab$ab &
done
wait
ls -la bin/stamps
