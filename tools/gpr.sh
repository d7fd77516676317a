#!/bin/bash
# (tools/gpr.sh) gpurun with a resubmit only when no GPU box was free (exit 3: nothing ran, nothing charged)
# usage: gpr.sh <out> <timeout> <script>  — resubmit only while no box is free (rc 3: nothing ran)
out=$1; to=$2; shift 2
for i in $(seq 1 30); do
  timeout $((to + 900)) /usr/local/graft/bin/gpurun --timeout $to -- "$@" > $out 2>&1
  rc=$?
  echo "[gpr] attempt $i rc=$rc" >> $out
  [ $rc -ne 3 ] && exit $rc
  sleep 150
done
