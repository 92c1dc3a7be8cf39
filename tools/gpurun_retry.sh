#!/bin/bash
# gpurun with retries while no box is free (status "transient": nothing ran, nothing charged).
# Never retries a command that ran. usage: tools/gpurun_retry.sh TIMEOUT 'command' OUTFILE
to=$1; cmd=$2; out=$3
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$out" 2>&1
  st=$(python3 -c "import json;print(json.load(open('/root/repo/gpurun_out/.last_call.json'))['status'])" 2>/dev/null)
  [ "$st" != "transient" ] && break
  sleep 150
done
tail -3 "$out"
