#!/bin/bash
# GPU session helper (sourced by the scripts that gpurun runs).
#   run  <name> <timeout_s> <cmd...>   bench/profile step: rc 0 or 1 continue, anything else stops
#   check <name> <timeout_s> <cmd...>   test step: any non-zero rc (pytest: 1 = failures) stops
# Every step runs under its own timeout; after a fault / abort / timeout nothing else touches the GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
_step() {
  local strict=$1 name=$2 t=$3; shift 3
  echo "== $name: $*" >&2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >&2
  tail -n 15 "gpurun_out/$name.log" >&2
  if [ $rc -ne 0 ]; then
    if [ "$strict" = 1 ] || [ $rc -ne 1 ]; then echo "FAIL: STOP after $name (rc=$rc)" >&2; exit $rc; fi
  fi
  return 0
}
run() { _step 0 "$@"; }
check() { _step 1 "$@"; }
