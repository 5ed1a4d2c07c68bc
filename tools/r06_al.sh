#!/bin/bash
# r06_al.sh TAG -- HEAD check after the r06aj / r06ak reverts: exact GPU tests (incl. the
# admission-forms subprocess check), smoke.
export TMPDIR=/tmp
TAG=${1:-r06al}
T=tools/gpu_step.sh
mkdir -p gpurun_out
$T ${TAG}_exact 400 python -u -m pytest tests/test_exact_gpu.py tests/test_search_gpu.py -m gpu -x -q --timeout 280 --timeout-method thread -p no:cacheprovider && \
$T ${TAG}_smoke 200 python -c "import __graft_entry__ as g; g.smoke()" && \
echo ALLDONE
