#!/bin/bash
# Build the stand-alone gather micro-benchmarks from their sources.
set -e
cd "$(dirname "$0")"
for t in gather_bench gather_model; do
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -o $t $t.hip
done
