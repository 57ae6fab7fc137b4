#!/bin/bash
# round-5 A/B probe library (tools/r05_probe.hip: the product's kernels + host shim + probe kernels)
cd "$(dirname "$0")/../../pb-af-xdp_amd" || exit 1
mkdir -p lib
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -shared \
  -o lib/libpbprobe.so tools/r05_probe.hip "$@"
