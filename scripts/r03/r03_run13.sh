#!/bin/bash
# Round 3: landing granularity by frame size (1500-B and configs[2] frames, one TX thread, the
# reference's 4,096-slot UMEM): chunk x landings in flight.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${OUT:-gpurun_out/r03s2m}
mkdir -p $O
for c in udp1500 var; do
  REPS=2 timeout -k 10 400 python -u scripts/e2e_ab.py $c 1 'c2048_i2:' 'c1024_i3:PB_LAND_CHUNK=1024,PB_LAND_INFLIGHT=3' \
      'c1024_i4:PB_LAND_CHUNK=1024,PB_LAND_INFLIGHT=4' 'c512_i8:PB_LAND_CHUNK=512,PB_LAND_INFLIGHT=8' \
      > $O/e2e_${c}_land.jsonl 2>&1 || exit 1
done
