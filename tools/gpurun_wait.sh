#!/bin/bash
# Submit one gpurun call; when the pool answers "no slot / no box free right now" (exit 3:
# nothing ran, nothing charged) wait and submit it again, up to 60 times.  Any other outcome
# (success, a failing command, a refusal) ends the script: GPU failures are never retried.
# Usage: tools/gpurun_wait.sh OUTFILE TIMEOUT 'command'
out=$1; to=$2; cmd=$3
for i in $(seq 1 60); do
    /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$out" 2>&1
    rc=$?
    if [ $rc -ne 3 ]; then echo "gpurun rc=$rc (attempt $i)" >> "$out"; exit $rc; fi
    sleep 90
done
echo "gpurun: gave up after 60 busy answers" >> "$out"
exit 3
