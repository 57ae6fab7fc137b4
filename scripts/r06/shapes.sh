#!/bin/bash
# round-6 page store shapes (workgroup sizes, XCD maps), chunk-mapped then hipMalloc'ed buffers
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r06
timeout -k 10 300 python3 -u scripts/r06/probe.py shapes ${REPS:-3} ${NBUF:-3} > gpurun_out/r06/shapes_vmm.jsonl 2> gpurun_out/r06/shapes_vmm.err || { tail -5 gpurun_out/r06/shapes_vmm.err; exit 1; }
PBGPU_ALLOC=malloc timeout -k 10 300 python3 -u scripts/r06/probe.py shapes ${REPS:-3} ${NBUF:-3} > gpurun_out/r06/shapes_malloc.jsonl 2> gpurun_out/r06/shapes_malloc.err || { tail -5 gpurun_out/r06/shapes_malloc.err; exit 1; }
