#!/bin/bash
# Runs one gpurun call, waiting and calling again ONLY while the pool reports that no box was free or
# the box failed before the command started (nothing ran, nothing was charged). Any other outcome —
# the command's own success or failure — ends the loop. usage: tools/gpurun_when_free.sh <out> <timeout> <cmd>
out=$1; lim=$2; cmd=$3
for attempt in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$lim" -- "$cmd" > "$out" 2>&1
  rc=$?
  if grep -q "no free box right now\|stopped responding while being prepared\|are busy" "$out" && grep -q "run 0.0s of limit" "$out"; then
    echo "attempt $attempt: no box; waiting" >> "$out.retries"
    sleep 180
    continue
  fi
  exit $rc
done
exit 3
