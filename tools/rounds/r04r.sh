#!/bin/bash
# r04r: the whole GPU suite, smoke() and the default bench line at HEAD.
export TMPDIR=/tmp
T=tools/gpu_step.sh
$T r04r_tests 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider && \
$T r04r_smoke 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" && \
$T r04r_bench 400 python bench.py && \
echo ALLDONE_R
