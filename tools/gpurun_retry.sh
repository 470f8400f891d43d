#!/bin/bash
# Re-submit a gpurun call only when the box could not be prepared (status "transient": nothing
# ran, nothing charged).  Usage: tools/gpurun_retry.sh TIMEOUT 'command'
T=$1; shift
for i in $(seq 1 ${RETRY_N:-8}); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" > /tmp/gpurun_retry.out 2>&1
  rc=$?
  st=$(python3 -c "import json;print(json.load(open('/root/repo/gpurun_out/.last_call.json')).get('status'))" 2>/dev/null)
  if [ "$st" != "transient" ] && [ $rc -ne 3 ]; then tail -3 /tmp/gpurun_retry.out; exit $rc; fi
  echo "[retry] status=$st rc=$rc; waiting" ; sleep 120
done
tail -3 /tmp/gpurun_retry.out
exit $rc
