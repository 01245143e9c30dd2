#!/bin/bash
# Runs named GPU steps in order, each under its own time limit.  A step that
# exits 0 or 1 (test failures, Python exceptions) lets the next one run; any
# other status (fault, abort, segfault, timeout) ends the script there.
# usage: tools/gpu_run.sh name:seconds:'command' ...
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
    name="${spec%%:*}"; rest="${spec#*:}"
    secs="${rest%%:*}"; cmd="${rest#*:}"
    echo "== $name (limit ${secs}s): $cmd"
    start=$(date +%s)
    timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
    rc=$?
    echo "== $name rc=$rc ($(( $(date +%s) - start ))s)"
    tail -5 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "== stopping: $name exited with $rc"
        exit $rc
    fi
done
