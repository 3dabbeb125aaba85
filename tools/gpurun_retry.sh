#!/bin/bash
# Submit one gpurun call, resubmitting only while the pool reports no free box (exit 3: nothing
# ran, nothing charged).  Any other outcome -- success, a failed or killed GPU step -- is final.
#   tools/gpurun_retry.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; CMD=$3
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$CMD" > $LOG 2>&1
  rc=$?
  [ $rc -ne 3 ] && ! grep -q "no free box right now\|backing off" $LOG && break
  echo "no box (attempt $i), waiting" >> $LOG.wait
  sleep 90
done
echo "rc=$rc" >> $LOG
