#!/usr/bin/env bash
# Runs a sequence of GPU steps on the gpurun box, each under its own time
# limit.  A step that fails ordinarily (exit 1, e.g. a failing test) does not
# stop the session; a fault-like status (timeout 124/137, abort 134,
# segfault 139, anything >= 124) ends it immediately.
# usage: tools/gpu_session.sh STEPFILE   (lines: "<timeout_s> <name> <command...>")
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
status=0
while read -r tmo name cmd; do
  [[ -z "${tmo:-}" || "${tmo:0:1}" == "#" ]] && continue
  echo "=== step $name (timeout ${tmo}s): $cmd" | tee -a gpurun_out/session.log
  start=$(date +%s)
  timeout -k 10 "$tmo" bash -c "$cmd" > "gpurun_out/$name.out" 2>&1
  rc=$?
  echo "=== step $name rc=$rc $(( $(date +%s) - start ))s" | tee -a gpurun_out/session.log
  tail -5 "gpurun_out/$name.out"
  if (( rc >= 124 )); then
    echo "fault-like exit $rc: stopping session" | tee -a gpurun_out/session.log
    exit "$rc"
  fi
  # a child process that aborted / segfaulted / faulted the GPU under a
  # launcher that itself exits 1 (torchrun, pytest-xdist, ...) is fatal too
  if grep -qE "SIGABRT|SIGSEGV|Signal 6|Signal 11|exitcode *: *-|Segmentation fault|Memory access fault|illegal memory access|core dumped" "gpurun_out/$name.out"; then
    echo "child fault detected in $name: stopping session" | tee -a gpurun_out/session.log
    exit 134
  fi
  (( rc != 0 )) && status=1
done < "$1"
exit $status
