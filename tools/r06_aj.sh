#!/bin/bash
# r06_aj.sh TAG -- K6c writes per-query pair lists and K6r holds the query in registers: exact GPU
# tests, deep k timings (compare r06ai: k = 5000 0.628 ms, k = 1000 0.50), kernel trace.
export TMPDIR=/tmp
TAG=${1:-r06aj}
S=tools/gpu_step.sh
mkdir -p gpurun_out
T() { "$S" "$@"; r=$?; [ $r -eq 99 ] && exit 99; return $r; }
T ${TAG}_exact 400 python -u -m pytest tests/test_exact_gpu.py -m gpu -x -q --timeout 280 --timeout-method thread -p no:cacheprovider && \
T ${TAG}_d1 120 python -u tools/deep_prof.py && \
T ${TAG}_d2 120 python -u tools/deep_prof.py && \
T ${TAG}_d1k 120 python -u tools/deep_prof.py --k 1000 && \
T ${TAG}_d768 180 python -u tools/deep_prof.py --dim 768 && \
T ${TAG}_kt_deep 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt_deep -o run -- python -u tools/deep_prof.py --steps 3 && \
T ${TAG}_search 400 python -u -m pytest tests/test_search_gpu.py -m gpu -x -q --timeout 280 --timeout-method thread -p no:cacheprovider && \
echo ALLDONE
