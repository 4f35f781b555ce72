#!/bin/bash
# GPU suite + optional extra commands (each GPU step time-limited; stop on fault).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-tests}
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/steps.log
  tail -3 "$OUT/$name.log" | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread ${PYTEST_ARGS:-}
if [ -n "${EXTRA:-}" ]; then step extra 300 bash -c "$EXTRA"; fi
