#!/bin/bash
# r06_an.sh TAG -- HEAD at the end of round 6: smoke and the default bench line.
export TMPDIR=/tmp
T=tools/gpu_step.sh
TAG=${1:-r06an}
mkdir -p gpurun_out
$T ${TAG}_smoke 200 python -c "import __graft_entry__ as g; g.smoke()" && \
$T ${TAG}_bench 600 python bench.py && \
echo ALLDONE
