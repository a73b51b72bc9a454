#!/bin/bash
# Run named GPU steps in order on the gpurun box, each under its own time limit; stop at the first failure.
#   bash tools/gpu_steps.sh TAG 'name|seconds|command' ['name|seconds|command' ...]
# Each step's output goes to gpurun_out/TAG_name.log; a one-line status per step goes to stdout.  A step whose name
# starts with "t-" (a pytest run) may fail its tests (exit 1) without stopping the later steps; any other non-zero
# exit (a time limit, a crash, an abort) ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=$1; shift
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; t=${rest%%|*}; cmd=${rest#*|}
  timeout -k 10 "$t" bash -c "$cmd" > gpurun_out/${T}_$name.log 2>&1
  rc=$?
  echo "$name rc=$rc: $(grep -v '^W20\|^E20\|amdgpu.ids' gpurun_out/${T}_$name.log | tail -1 | cut -c1-300)"
  if [ $rc -ne 0 ] && ! { [ $rc -eq 1 ] && [ "${name#t-}" != "$name" ]; }; then exit $rc; fi
done
echo done
