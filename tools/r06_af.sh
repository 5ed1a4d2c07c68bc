#!/bin/bash
# r06_af.sh TAG — state after the r06 flag / deep-k changes: every -m gpu test, smoke(), the
# default bench line, and the kernel-trace stats of the default bench command.
export TMPDIR=/tmp
T=tools/gpu_step.sh
TAG=${1:-r06af}
mkdir -p gpurun_out
$T ${TAG}_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider && \
$T ${TAG}_smoke 200 python -c "import __graft_entry__ as g; g.smoke()" && \
$T ${TAG}_bench 600 python bench.py && \
$T ${TAG}_kt_bench 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt_bench -o run -- python bench.py && \
echo ALLDONE
