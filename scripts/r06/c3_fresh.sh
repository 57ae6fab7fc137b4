#!/bin/bash
# configs[2] in fresh processes (verdict r05 item 1's done criterion): bench.py --config c3_udp_var,
# N processes with chunk-mapped frame buffers and N with PBGPU_ALLOC=malloc, alternating; one bench
# JSON line per process in $out/c3_fresh.jsonl (tagged with the allocator).
cd "$(dirname "$0")/../.." || exit 1
out=${1:-gpurun_out/r06/c3fresh}
n=${N:-5}
mkdir -p "$out"
for i in $(seq 1 "$n"); do
  for alloc in chunks malloc; do
    if [ $alloc = malloc ]; then export PBGPU_ALLOC=malloc; else unset PBGPU_ALLOC; fi
    line=$(timeout -k 10 120 python3 bench.py --config c3_udp_var --steps 30 --warmup 5 --no-variants \
      --cpu-seconds 0 2> "$out/err_${i}_${alloc}.log") || { echo "bench failed ($alloc $i)"; exit 1; }
    echo "{\"alloc\": \"$alloc\", \"proc\": $i, \"line\": $line}" >> "$out/c3_fresh.jsonl"
    echo "$alloc $i done"
  done
done
