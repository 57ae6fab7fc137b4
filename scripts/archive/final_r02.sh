#!/bin/bash
# Round-2 closing run: the whole GPU suite, smoke(), then the profile refresh (trace, PMC, per-config lines)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/final
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final/pytest.log 2>&1 || { tail -30 gpurun_out/final/pytest.log; exit 1; }
tail -2 gpurun_out/final/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.log 2>&1 || { tail -20 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
bash scripts/profile_round_r02.sh
