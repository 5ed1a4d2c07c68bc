#!/bin/bash
# r06_z.sh TAG -- K6m admitted keys staged per block in LDS: exact GPU tests, deep-k timing + trace.
export TMPDIR=/tmp
TAG=${1:-r06z}
S=tools/gpu_step.sh
mkdir -p gpurun_out
T() { "$S" "$@"; r=$?; [ $r -eq 99 ] && exit 99; return $r; }
T ${TAG}_exact 400 python -u -m pytest tests/test_exact_gpu.py tests/test_search_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider && \
T ${TAG}_deep 200 python -u tools/deep_prof.py && \
T ${TAG}_deep1k 200 python -u tools/deep_prof.py --k 1000 && \
T ${TAG}_kt_deep 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt_deep -o run -- python -u tools/deep_prof.py --steps 3 && \
echo ALLDONE
