#!/bin/bash
# pb_fstage_kernel: parity (kernel-shape tests + the 1500-B parity tests), then an
# in-process A/B of its shapes against pb_stage_kernel on configs[1] 1500-B frames
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -k "fstage" --timeout 120 \
  --timeout-method thread > gpurun_out/fst_par.txt 2>&1 || { tail -40 gpurun_out/fst_par.txt; exit 1; }
tail -n 2 gpurun_out/fst_par.txt
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "1500" --timeout 120 \
  --timeout-method thread > gpurun_out/fst_par2.txt 2>&1 || { tail -40 gpurun_out/fst_par2.txt; exit 1; }
tail -n 2 gpurun_out/fst_par2.txt
[ -n "$PARITY_ONLY" ] && exit 0
REPS=${REPS:-5} timeout -k 10 300 python3 -u scripts/ab_env.py c2_udp_1500 ${NPK:-8388608} \
  stage:PBGPU_KERNEL=stage \
  fst16:PBGPU_FST_G=16 \
  fst16nb1:PBGPU_FST_G=16,PBGPU_FST_NBUF=1 \
  fst16w128:PBGPU_FST_G=16,PBGPU_FST_WGF=128 \
  fst32:PBGPU_FST_G=32 \
  fst32nb1:PBGPU_FST_G=32,PBGPU_FST_NBUF=1 \
  fst32w128:PBGPU_FST_G=32,PBGPU_FST_WGF=128 \
  fst64:PBGPU_FST_G=64 \
  | tee gpurun_out/fst_ab.txt
