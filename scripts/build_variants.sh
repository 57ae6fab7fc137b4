#!/bin/bash
# compile-time variants of libpbgpu.so for scripts/ab_lib.py: name=FLAGS ...
cd "$(dirname "$0")/../pb-af-xdp_amd" || exit 1
mkdir -p lib/variants
for v in "$@"; do
  name=${v%%=*}; flags=${v#*=}
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $flags -shared \
    -o lib/variants/libpbgpu_$name.so csrc/pbgpu_kernels.hip csrc/pbgpu.cpp || exit 1
done
