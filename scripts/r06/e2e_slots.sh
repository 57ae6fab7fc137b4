#!/bin/bash
# End-to-end host pipeline (build -> land -> TX ring) with 4-KiB and smaller UMEM slots
# (--umemslot), 1 and 2 TX threads, N scaled x4 (scripts/e2e_probe.py); one JSON line per case.
cd "$(dirname "$0")/../.." || exit 1
out=${1:-gpurun_out/r06/slot}
mkdir -p "$out"
for args in "" "--umemslot 64"; do
  E2E_CASES=udp64 E2E_THREADS=1,2 E2E_BATCHES=262144,1048576 E2E_SCALE=4 E2E_ARGS="$args" \
    timeout -k 10 300 python3 -u scripts/e2e_probe.py >> "$out/e2e.jsonl" || exit 1
done
for args in "" "--umemslot 2048"; do
  E2E_CASES=udp1500 E2E_THREADS=1,2 E2E_BATCHES=262144 E2E_SCALE=4 E2E_ARGS="$args" \
    timeout -k 10 300 python3 -u scripts/e2e_probe.py >> "$out/e2e.jsonl" || exit 1
done
