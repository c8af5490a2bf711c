#!/bin/bash
# Run one gpurun call, retrying ONLY while the pool has no box for it (exit 3: nothing ran, nothing
# charged), at most 12 tries 2 minutes apart. Any other outcome (success, failure, refusal) ends it.
# usage: tools/gpurun_retry.sh <timeout_s> <log> '<command>'
t=$1; log=$2; cmd=$3
for i in $(seq 1 12); do
    /usr/local/graft/bin/gpurun --timeout "$t" -- "$cmd" > "$log" 2>&1
    rc=$?
    if [ $rc -ne 3 ] && ! grep -q "status=transient" "$log"; then exit $rc; fi
    sleep 120
done
exit $rc
