#!/bin/bash
# generic env sweep of the frame-length probe: SWEEP="tag1:VAR=a,VAR2=b tag2:..."; LENS as in align_probe
set -e
mkdir -p gpurun_out/sweep
for item in $SWEEP; do
  tag=${item%%:*}; envs=${item#*:}
  env $(echo $envs | tr ',' ' ') LENS=${LENS:-1500,1536,1024,512} timeout -k 10 200 python3 scripts/align_probe.py $tag > gpurun_out/sweep/$tag.json
done
python3 - <<'PY'
import json, glob, os
for tag in os.environ["SWEEP"].split():
    d = json.load(open(f"gpurun_out/sweep/{tag.split(':')[0]}.json"))
    print(d["tag"], "fill", d["fill_gbps"], " ".join(f"{k}={v['gbps']}" for k, v in d.items() if isinstance(v, dict)), d["udp1500"]["kernel"])
PY
