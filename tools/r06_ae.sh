#!/bin/bash
# r06_ae.sh TAG -- K6r with vector query loads, side-by-side wave sums and a 960-key stage; the
# deep sort enqueued before the round read-back: exact + search GPU tests, deep k timings, K6r
# grid A/B, kernel trace.
export TMPDIR=/tmp
TAG=${1:-r06ae}
S=tools/gpu_step.sh
mkdir -p gpurun_out
T() { "$S" "$@"; r=$?; [ $r -eq 99 ] && exit 99; return $r; }
T ${TAG}_exact 400 python -u -m pytest tests/test_exact_gpu.py -m gpu -x -q --timeout 280 --timeout-method thread -p no:cacheprovider || exit 1
for rep in 1 2; do
  T ${TAG}_d_def_$rep 120 python -u tools/deep_prof.py || exit 1
  T ${TAG}_d_r256_$rep 120 env HCRAG_K6R_BLOCKS=256 python -u tools/deep_prof.py || exit 1
  T ${TAG}_d_r1024_$rep 120 env HCRAG_K6R_BLOCKS=1024 python -u tools/deep_prof.py || exit 1
done
T ${TAG}_d1k 120 python -u tools/deep_prof.py --k 1000 || exit 1
T ${TAG}_d768 180 python -u tools/deep_prof.py --dim 768 || exit 1
T ${TAG}_kt_deep 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt_deep -o run -- python -u tools/deep_prof.py --steps 3 && \
T ${TAG}_search 400 python -u -m pytest tests/test_search_gpu.py tests/test_global_seed_gpu.py tests/test_qw_gpu.py -m gpu -x -q --timeout 280 --timeout-method thread -p no:cacheprovider && \
echo ALLDONE
