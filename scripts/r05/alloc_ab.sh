#!/bin/bash
# Fresh-process A/B of the frame-buffer allocation (tool only): the default bench line (64-B
# metric + 1500-B leg) and configs[2], alternating PBGPU_ALLOC=malloc and the chunk-mapped
# default (vmm: 64-MiB chunks; vmm2: 2-MiB), REPS times (MODES); one JSON summary line per run into gpurun_out/r05/alloc_ab.jsonl.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
REPS=${REPS:-3}
out=gpurun_out/r05/alloc_ab.jsonl
mkdir -p gpurun_out/r05
: > $out
for r in $(seq 1 $REPS); do
  for mode in ${MODES:-malloc vmm}; do
    for cfg in c2_udp_64 c3_udp_var; do
      unset PBGPU_ALLOC PBGPU_ALLOC_CHUNK_MB
      [ $mode = malloc ] && export PBGPU_ALLOC=malloc
      [ $mode = vmm2 ] && export PBGPU_ALLOC_CHUNK_MB=2
      V=--no-variants; [ $cfg = c2_udp_64 ] && V=
      timeout -k 10 240 python3 bench.py --steps 50 --warmup 5 --cpu-seconds 0 --config $cfg $V > gpurun_out/r05/alloc_ab_last.log 2>&1 || { echo "FAIL $mode $cfg"; tail -5 gpurun_out/r05/alloc_ab_last.log; exit 1; }
      python3 - "$mode" "$cfg" "$r" >> $out <<'PY'
import json, sys
mode, cfg, r = sys.argv[1:]
d = [json.loads(l) for l in open("gpurun_out/r05/alloc_ab_last.log") if l.startswith('{"metric"')][0]
row = {"rep": int(r), "alloc": mode, "config": cfg, "ms": d["roofline"]["kernel_ms_avg"], "frac": d["roofline"]["frac"]}
if "udp_1500" in d:
    row["udp_1500_ms"] = d["udp_1500"]["kernel_ms_avg"]
    row["udp_1500_frac"] = d["udp_1500"]["roofline_frac"]
print(json.dumps(row))
PY
      tail -1 $out
    done
  done
done
