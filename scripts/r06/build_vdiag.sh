#!/bin/bash
# round-6 pb_vline_kernel decomposition probe (probes/r06_vdiag.hip: the gate probe + a cut copy of the kernel)
cd "$(dirname "$0")/../.." || exit 1
mkdir -p pb-af-xdp_amd/lib
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -shared \
  -Iinclude -o pb-af-xdp_amd/lib/libpbprobe6v.so probes/r06_vdiag.hip "$@"
