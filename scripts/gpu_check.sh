#!/bin/bash
# One GPU session: kernel numerics, then short benches. Stops at the first crash/timeout.
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "abort after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step "${@}"
