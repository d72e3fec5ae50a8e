#!/bin/bash
# Run one gpurun call, re-submitting it only while the pool reports no free box or slot ("transient":
# nothing ran, nothing was charged), at most $TRIES times, $WAIT seconds apart.  Any other outcome
# (success, failure, timeout, fault) ends the loop: a GPU step that ran is never repeated here.
#   tools/gpurun_wait.sh TIMEOUT 'command'
T=$1
shift
for i in $(seq 1 ${TRIES:-8}); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
  rc=$?
  st=$(python3 -c "import json; print(json.load(open('gpurun_out/.last_call.json')).get('status'))" 2>/dev/null)
  [ "$st" = "transient" ] || [ $rc -eq 3 ] || exit $rc
  sleep ${WAIT:-150}
done
exit $rc
