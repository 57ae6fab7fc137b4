#!/bin/bash
# Run named GPU steps in order, each under its own time limit, output to gpurun_out/r06/<name>.log.
# Any non-zero status (a failed test, a crash, an abort, a GPU fault, a time limit) ends the
# script there: nothing more runs on the GPU after a step that failed.
#   scripts/r05/gpu_steps.sh "name|seconds|command" ...
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
for step in "$@"; do
  name=${step%%|*}; rest=${step#*|}; secs=${rest%%|*}; cmd=${rest#*|}
  echo "== $name ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/r06/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc"; tail -3 "gpurun_out/r06/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
done
