#!/bin/bash
# gpurun with a bounded wait for a free slot: when gpurun reports that no
# slot or box was free (nothing ran, nothing charged), wait and call again,
# at most 12 times. Every attempt's output is appended to the log.
#   tools/gpurun_retry.sh <log> <gpurun args...>
LOG=$1; shift
: > $LOG
for i in 1 2 3 4 5 6 7 8 9 10 11 12; do
  echo "=== attempt $i $(date -u +%H:%M:%S)" >> $LOG
  /usr/local/graft/bin/gpurun "$@" > $LOG.part 2>&1
  rc=$?
  cat $LOG.part >> $LOG
  if ! grep -q "status=transient" $LOG.part; then
    rm -f $LOG.part
    echo "rc=$rc" >> $LOG
    exit $rc
  fi
  sleep 150
done
rm -f $LOG.part
echo "gave up: no slot" >> $LOG
