#!/usr/bin/env bash
# retry a gpurun call only while no box is free (exit 3 / transient); log to $1
LOG=$1; shift
for i in $(seq 1 8); do
  /usr/local/graft/bin/gpurun "$@" > $LOG 2>&1; rc=$?
  if grep -q "status=transient" $LOG && ! grep -q "status=ok" $LOG; then sleep 200; continue; fi
  break
done
echo "done rc=$rc tries=$i" >> $LOG
