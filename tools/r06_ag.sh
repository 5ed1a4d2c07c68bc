#!/bin/bash
# r06_ag.sh TAG -- K6c with only its pair queues in LDS (4 blocks per CU), the deep sort's chunk
# chosen to fill the chip (HCRAG_SORT_CHUNK=8192: one block per query, the previous form): exact
# GPU tests, deep k A/B (alternating processes), kernel trace.
export TMPDIR=/tmp
TAG=${1:-r06ag}
S=tools/gpu_step.sh
mkdir -p gpurun_out
T() { "$S" "$@"; r=$?; [ $r -eq 99 ] && exit 99; return $r; }
T ${TAG}_exact 400 python -u -m pytest tests/test_exact_gpu.py -m gpu -x -q --timeout 280 --timeout-method thread -p no:cacheprovider || exit 1
for rep in 1 2; do
  T ${TAG}_d_def_$rep 120 python -u tools/deep_prof.py || exit 1
  T ${TAG}_d_s8192_$rep 120 env HCRAG_SORT_CHUNK=8192 python -u tools/deep_prof.py || exit 1
  T ${TAG}_d_s4096_$rep 120 env HCRAG_SORT_CHUNK=4096 python -u tools/deep_prof.py || exit 1
done
T ${TAG}_d1k 120 python -u tools/deep_prof.py --k 1000 || exit 1
T ${TAG}_d20k 120 python -u tools/deep_prof.py --k 20000 || exit 1
T ${TAG}_kt_deep 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt_deep -o run -- python -u tools/deep_prof.py --steps 3 && \
echo ALLDONE
