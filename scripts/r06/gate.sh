#!/bin/bash
# round-6 gate probe: default (chunk-mapped) buffers, then hipMalloc'ed ones
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r06
timeout -k 10 300 python3 -u scripts/r06/probe.py gate ${REPS:-5} ${NBUF:-3} > gpurun_out/r06/gate_vmm.jsonl 2> gpurun_out/r06/gate_vmm.err || { tail -5 gpurun_out/r06/gate_vmm.err; exit 1; }
PBGPU_ALLOC=malloc timeout -k 10 300 python3 -u scripts/r06/probe.py gate ${REPS:-5} ${NBUF:-3} > gpurun_out/r06/gate_malloc.jsonl 2> gpurun_out/r06/gate_malloc.err || { tail -5 gpurun_out/r06/gate_malloc.err; exit 1; }
