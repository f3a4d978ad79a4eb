#!/bin/bash
# Acquisition retry around ONE gpurun call: re-submits only when gpurun
# reports that no command ran (no free box / box lost while being prepared /
# backing off: status "transient", nothing charged). A command that ran —
# whatever its exit status — is never re-run.
#   tools/gpurun_retry.sh LOG TIMEOUT 'COMMAND' [TRIES]
LOG=$1; TO=$2; CMD=$3; TRIES=${4:-8}
for i in $(seq 1 $TRIES); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  if grep -q "status=transient" "$LOG" && grep -q "run 0.0s\|run Nones" "$LOG"; then
    w=$(grep -o "retry in [0-9]*s" "$LOG" | grep -o "[0-9]*" | tail -1)
    sleep $(( ${w:-150} + 15 ))
    continue
  fi
  break
done
tail -40 "$LOG"
