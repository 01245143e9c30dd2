#!/bin/bash
# Round-end rehearsal of the driver's GPU steps: the -m gpu suite, smoke(), the default bench line.
exec tools/gpu_run.sh \
 "gputest:400:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "smoke:200:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench:400:python bench.py"
