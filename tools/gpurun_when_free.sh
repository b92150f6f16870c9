#!/bin/bash
# gpurun, re-submitted while the pool reports no free slot or box
# (status=transient: nothing ran, nothing charged).  A call that ran -- pass
# or fail -- is never repeated.  Usage: tools/gpurun_when_free.sh LOG TIMEOUT 'CMD'
log=$1; to=$2; cmd=$3
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$log" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || { grep -q "status=transient" "$log" && ! grep -q "charged=[1-9]" "$log"; }; then sleep 90; continue; fi
  exit $rc
done
exit 3
