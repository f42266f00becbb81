#!/bin/bash
# Local helper (build container only): run ONE gpurun call, re-submitting it only when gpurun reports
# an infrastructure "status=transient" outcome (nothing ran, nothing charged); any real result,
# failure or refusal is returned as is.  usage: tools/gpurun_retry.sh <timeout-s> <command>
T=$1; shift
for i in $(seq 1 20); do
    out=$(timeout $((T + 900)) /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1)
    rc=$?
    echo "$out" | grep -v "every call sends" | tail -3
    if echo "$out" | grep -q "status=transient"; then sleep 60; continue; fi
    exit $rc
done
exit 3
