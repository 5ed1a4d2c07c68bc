#!/bin/bash
# r06_ai.sh TAG — final round-6 state: every -m gpu test, smoke(), the default bench line, the
# rocprofv3 kernel-trace stats of the default bench command, deep k timings.
export TMPDIR=/tmp
T=tools/gpu_step.sh
TAG=${1:-r06ai}
mkdir -p gpurun_out
$T ${TAG}_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider && \
$T ${TAG}_smoke 200 python -c "import __graft_entry__ as g; g.smoke()" && \
$T ${TAG}_bench 600 python bench.py && \
$T ${TAG}_kt_bench 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt_bench -o run -- python bench.py && \
$T ${TAG}_deep 120 python -u tools/deep_prof.py && \
$T ${TAG}_deep1k 120 python -u tools/deep_prof.py --k 1000 && \
echo ALLDONE
