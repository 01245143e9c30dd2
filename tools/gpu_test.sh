#!/bin/bash
# The -m gpu suite (optionally a -k filter in $1).
K="${1:-}"
if [ -n "$K" ]; then
  exec tools/gpu_run.sh "gputest:400:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k '$K'"
fi
exec tools/gpu_run.sh "gputest:400:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread"
