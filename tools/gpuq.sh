#!/bin/bash
# gpurun with a wait for a free slot: re-submits ONLY when gpurun reports rc 3 (no slot; nothing ran, nothing charged)
OUT=$1; shift
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun "$@" > $OUT 2>&1
  rc=$?
  if [ $rc -ne 3 ]; then echo "rc=$rc" >> $OUT; exit $rc; fi
  sleep 90
done
