#!/bin/bash
# Run one gpurun call; on exit 3 (no box/slot free, nothing charged) wait and
# try again, up to 6 times. Any other exit code is returned as is.
# Usage: scripts/gpurun_retry.sh TIMEOUT 'command'
T=$1; shift
for i in 1 2 3 4 5 6; do
  rm -f gpurun_out/.last_call.json
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  echo "[retry] no box (attempt $i), waiting 60 s" >&2
  sleep 60
done
exit 3
