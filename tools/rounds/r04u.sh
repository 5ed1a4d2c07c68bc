#!/bin/bash
# r04u: the whole GPU suite, smoke() and the default bench line at HEAD.
export TMPDIR=/tmp
T=tools/gpu_step.sh
$T r04u_tests 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider && \
$T r04u_smoke 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" && \
$T r04u_bench 400 python bench.py && \
echo ALLDONE_R
