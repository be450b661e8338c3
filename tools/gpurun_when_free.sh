#!/bin/bash
# Submit one gpurun call, resubmitting it only while gpurun answers "no box / slot free right now"
# (exit 3: nothing ran, nothing charged), at most 8 times, 3 minutes apart.  Any other outcome --
# success, a failed command, a refusal -- ends it.  usage: tools/gpurun_when_free.sh <log> <timeout> <command>
log=${1:?log}; t=${2:?timeout}; cmd=${3:?command}
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$cmd" > "$log" 2>&1
  rc=$?
  echo "exit $rc (try $i)" >> "$log"
  [ $rc -ne 3 ] && exit $rc
  sleep 180
done
exit 3
