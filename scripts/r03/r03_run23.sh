#!/bin/bash
# runs r03_run2.sh then r03_run3.sh in one box session
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash scripts/r03/r03_run2.sh && bash scripts/r03/r03_run3.sh
