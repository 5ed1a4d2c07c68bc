#!/bin/bash
# r06_ak.sh TAG -- K6c with both query groups of a pair per wave (QB = 4, ld = 384) against one
# group (HCRAG_K6_QB2): exact GPU tests, deep k A/B (alternating processes), kernel trace.
export TMPDIR=/tmp
TAG=${1:-r06ak}
S=tools/gpu_step.sh
mkdir -p gpurun_out
T() { "$S" "$@"; r=$?; [ $r -eq 99 ] && exit 99; return $r; }
T ${TAG}_exact 400 python -u -m pytest tests/test_exact_gpu.py -m gpu -x -q --timeout 280 --timeout-method thread -p no:cacheprovider || exit 1
for rep in 1 2; do
  T ${TAG}_d_qb4_$rep 120 python -u tools/deep_prof.py || exit 1
  T ${TAG}_d_qb2_$rep 120 env HCRAG_K6_QB2=1 python -u tools/deep_prof.py || exit 1
done
T ${TAG}_d1k_qb4 120 python -u tools/deep_prof.py --k 1000 || exit 1
T ${TAG}_d1k_qb2 120 env HCRAG_K6_QB2=1 python -u tools/deep_prof.py --k 1000 || exit 1
T ${TAG}_kt_deep 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt_deep -o run -- python -u tools/deep_prof.py --steps 3 && \
echo ALLDONE
