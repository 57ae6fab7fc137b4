#!/bin/bash
# PMC passes of c2_udp_1500 under the staged kernel and the group-per-frame kernel
set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
CFG=c2_udp_1500 PKTS=2097152 bash scripts/pmc_pass.sh
mv gpurun_out/pmc_c2_udp_1500 gpurun_out/pmc_stage_1500
PBGPU_KERNEL=gpf CFG=c2_udp_1500 PKTS=2097152 bash scripts/pmc_pass.sh
mv gpurun_out/pmc_c2_udp_1500 gpurun_out/pmc_gpf_1500
python3 scripts/pmc_summary.py gpurun_out/pmc_stage_1500 pb_stage
python3 scripts/pmc_summary.py gpurun_out/pmc_gpf_1500 pb_gpf
