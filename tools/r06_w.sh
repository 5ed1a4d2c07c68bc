#!/bin/bash
# r06_w.sh TAG — final round-6 state on one box: every -m gpu test, smoke(), the default bench line.
export TMPDIR=/tmp
T=tools/gpu_step.sh
TAG=${1:-r06w}
$T ${TAG}_tests 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider && \
$T ${TAG}_smoke 200 python -c "import __graft_entry__ as g; g.smoke()" && \
$T ${TAG}_bench 600 python bench.py && \
echo ALLDONE
