#!/bin/bash
# dev: submit one gpurun command, resubmitting ONLY while the pool reports no free
# box / slot (gpurun exit code 3: nothing ran, nothing charged); any other outcome
# (success, failure, refusal) ends it.  usage: tools/gpurun_wait.sh LOG TIMEOUT 'cmd'
log=$1; to=$2; cmd=$3
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$log" 2>&1
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 180
done
exit 3
