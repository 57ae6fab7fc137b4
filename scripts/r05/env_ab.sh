#!/bin/bash
# Fresh-process A/B of load-time options on one config (tool only):
#   CFG=c3_udp_var VAR=PBGPU_VL_WGF VALUES="0 200 168" REPS=2 scripts/r05/env_ab.sh
# ("unset" leaves the variable unset); one JSON summary line per run into gpurun_out/r05/env_ab.jsonl.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
out=gpurun_out/r05/env_ab.jsonl
mkdir -p gpurun_out/r05
: > $out
for r in $(seq 1 ${REPS:-2}); do
  for v in $VALUES; do
    unset $VAR
    [ "$v" != unset ] && export $VAR=$v
    timeout -k 10 240 python3 bench.py --steps 50 --warmup 5 --cpu-seconds 0 --no-variants --config $CFG > gpurun_out/r05/env_ab_last.log 2>&1 || { echo "FAIL $VAR=$v"; tail -5 gpurun_out/r05/env_ab_last.log; exit 1; }
    python3 - "$VAR" "$v" "$r" >> $out <<'PY'
import json, sys
var, v, r = sys.argv[1:]
d = [json.loads(l) for l in open("gpurun_out/r05/env_ab_last.log") if l.startswith('{"metric"')][0]
print(json.dumps({"rep": int(r), var: v, "config": d["config"]["workload"][:12], "ms": d["roofline"]["kernel_ms_avg"],
                  "frac": d["roofline"]["frac"], "per_launch_med": d["roofline"]["per_launch_ms"]["median"]}))
PY
    tail -1 $out
  done
done
