#!/bin/bash
# Submit one gpurun call; re-submit ONLY when nothing ran (no box / slot free, or the box was taken
# away before the command started: gpurun exit 3 or status=transient with run 0.0s).  Never
# re-submits a command that ran, failed or timed out.
#   tools/gpu/submit.sh <log> <timeout-s> '<command>'
LOG=$1; T=$2; CMD=$3
for attempt in 1 2 3 4 5 6 7 8 9 10; do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || { grep -q "status=transient" "$LOG" && grep -q "run 0.0s" "$LOG"; }; then
    echo "[submit] attempt $attempt: nothing ran (rc $rc); retrying in 150 s" >> "$LOG.tries"
    sleep 150
    continue
  fi
  exit $rc
done
exit 3
