#!/bin/bash
# evidence.sh TAG — the round-end set on one box: every -m gpu test, smoke(), the default bench line,
# and a kernel trace of the default bench (profiles/r03/...).
export TMPDIR=/tmp
T=tools/gpu_step.sh
TAG=${1:-evidence}
$T ${TAG}_tests 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider && \
$T ${TAG}_smoke 200 python -c "import __graft_entry__ as g; g.smoke()" && \
$T ${TAG}_bench 500 python bench.py && \
echo ALLDONE
