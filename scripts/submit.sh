#!/bin/bash
# Submit one gpurun call; when the pool has no box (a transient refusal: nothing ran, nothing
# charged), wait and submit the same call again -- at most N times.  A call that actually ran
# (any exit status) is never resubmitted.
# usage: scripts/r04/submit.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; CMD=$3
for i in $(seq 1 ${SUBMIT_TRIES:-20}); do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$CMD" > $LOG 2>&1
  rc=$?
  if grep -q "status=transient" $LOG; then
    echo "[submit] attempt $i: no box ($(grep -o 'retry in [0-9]*s' $LOG | head -1)); waiting" >> $LOG.attempts
    sleep 150
    continue
  fi
  exit $rc
done
exit 3
