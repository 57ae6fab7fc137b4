#!/bin/bash
# Allocation-time placement check, fresh processes (tool only): scripts/r05/probe.py remap REPS times
# per allocator, alternating; NBUF buffers each.  -> gpurun_out/r05/remap_runs.jsonl
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out/r05
O=gpurun_out/r05/${OUT:-remap_runs}.jsonl
for r in $(seq 1 "${REPS:-3}"); do
  for a in ${ALLOCS:-malloc vmm}; do
    if [ $a = malloc ]; then export PBGPU_ALLOC=malloc; else unset PBGPU_ALLOC; fi
    echo "{\"run\": $r, \"alloc\": \"$a\"}" >> $O
    timeout -k 10 180 python3 scripts/r05/probe.py remap >> $O 2>gpurun_out/r05/remap_err.log || { echo "FAIL rc=$? run $r $a"; tail -5 gpurun_out/r05/remap_err.log; exit 1; }
    echo "run $r $a done"
  done
done
