#!/bin/bash
# gpurun_retry.sh OUTFILE TIMEOUT CMD: one gpurun call, re-submitted only while the pool has no
# free slot or box (status=transient: nothing ran, nothing charged).  A call that ran is never
# repeated, whatever its outcome.
out=$1; lim=$2; shift 2
for i in $(seq 1 12); do
  timeout $((lim + 1500)) /usr/local/graft/bin/gpurun --timeout "$lim" -- "$@" > "$out" 2>&1
  rc=$?
  grep -q "status=transient" "$out" || exit $rc
  sleep 120
done
exit $rc
