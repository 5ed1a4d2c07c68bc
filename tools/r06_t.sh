#!/bin/bash
# r06_t.sh TAG -- round-0 thresholds on the device (hist_seed_kernel): exact / deep GPU tests,
# deep-k timing + trace; then configs[1] with and without the sampling pre-pass.
export TMPDIR=/tmp
TAG=${1:-r06t}
S=tools/gpu_step.sh
mkdir -p gpurun_out
T() { "$S" "$@"; r=$?; [ $r -eq 99 ] && exit 99; return $r; }
T ${TAG}_exact 400 python -u -m pytest tests/test_exact_gpu.py tests/test_search_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider && \
T ${TAG}_deep 200 python -u tools/deep_prof.py && \
T ${TAG}_deep1k 200 python -u tools/deep_prof.py --k 1000 && \
T ${TAG}_kt_deep 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt_deep -o run -- python -u tools/deep_prof.py --steps 3 || exit 99
for r in 1 2 3; do
  timeout -k 10 150 python tools/opt_ab.py 1000000 384 256 10 2 default >> gpurun_out/${TAG}_c1_ab.txt 2>&1 || exit 99
  timeout -k 10 150 env HCRAG_NO_PREPASS=1 python tools/opt_ab.py 1000000 384 256 10 2 default >> gpurun_out/${TAG}_c1_noprepass.txt 2>&1 || exit 99
done
echo ALLDONE
