#!/bin/bash
# pb_xpage_kernel at any byte phase: small-frame parity (every length, forced shapes), then length A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -k "small" --timeout 120 \
  --timeout-method thread > gpurun_out/xpl_par.txt 2>&1 || { tail -40 gpurun_out/xpl_par.txt; exit 1; }
tail -n 1 gpurun_out/xpl_par.txt
timeout -k 10 400 python3 -u scripts/xp_len_ab.py | tee gpurun_out/xpl_ab.txt
