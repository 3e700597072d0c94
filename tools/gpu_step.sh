#!/bin/bash
# Run one GPU step under a time limit; exit non-zero (ending the caller's && chain) only when the step crashed, was
# killed or timed out (status > 1): pytest's status 1 (test failures) lets the next step run.
#   bash tools/gpu_step.sh <seconds> <log> <command...>
T=$1; LOG=$2; shift 2
timeout -k 10 $T "$@" > $LOG 2>&1
rc=$?
echo "[gpu_step] rc=$rc: $*" >> $LOG
[ $rc -le 1 ]
