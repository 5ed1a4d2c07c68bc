#!/bin/bash
# r06_ah.sh TAG -- K6h's sampling rule (HCRAG_K6H_RATIO: sampled rows per k the next stride must
# leave; 100 the previous default): deep k A/B at 1M x 384 and 10M x 768 (alternating processes),
# exact GPU tests under the candidate default.
export TMPDIR=/tmp
TAG=${1:-r06ah}
S=tools/gpu_step.sh
mkdir -p gpurun_out
T() { "$S" "$@"; r=$?; [ $r -eq 99 ] && exit 99; return $r; }
for rep in 1 2; do
  for r in 100 25 12; do
    T ${TAG}_d_r${r}_$rep 120 env HCRAG_K6H_RATIO=$r python -u tools/deep_prof.py || exit 1
  done
done
for r in 100 25; do
  T ${TAG}_big_r${r}_k1000 240 env HCRAG_K6H_RATIO=$r python -u tools/deep_prof.py --rows 10000000 --dim 768 --k 1000 || exit 1
  T ${TAG}_big_r${r}_k5000 240 env HCRAG_K6H_RATIO=$r python -u tools/deep_prof.py --rows 10000000 --dim 768 --k 5000 || exit 1
done
T ${TAG}_exact25 400 env HCRAG_K6H_RATIO=25 python -u -m pytest tests/test_exact_gpu.py -m gpu -x -q --timeout 280 --timeout-method thread -p no:cacheprovider && \
echo ALLDONE
