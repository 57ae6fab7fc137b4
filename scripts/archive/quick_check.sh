#!/bin/bash
# parity (default + kernel shapes), staged-kernel phase timing, frame-length probe
set -e
mkdir -p gpurun_out
timeout -k 10 600 python3 -m pytest tests/test_gpu_parity.py tests/test_gpu_kernels.py -x -q -m gpu > gpurun_out/qc_tests.txt 2>&1 || { tail -30 gpurun_out/qc_tests.txt; exit 1; }
tail -n 1 gpurun_out/qc_tests.txt
LENS=${LENS:-1500,1536,1024,512,9000} timeout -k 10 200 python3 scripts/align_probe.py ${TAG:-qc} > gpurun_out/qc_probe.json
cat gpurun_out/qc_probe.json
[ -n "$NO_TIMING" ] || KBS="24" bash scripts/timing_probe.sh
