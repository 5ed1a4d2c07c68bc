#!/bin/bash
# r06_i.sh TAG -- batched K6m admissions (4 pairs per rescore) + 1024-thread bitonic sort +
# high-priority encoder sub-batch streams: exact / deep GPU tests, encoder tests, deep-k timing
# and trace, large-k bench points, the bench's encoder leg alone, enc_prof.
export TMPDIR=/tmp
TAG=${1:-r06i}
S=tools/gpu_step.sh
mkdir -p gpurun_out
T() { "$S" "$@"; r=$?; [ $r -eq 99 ] && exit 99; return $r; }
T ${TAG}_exact 400 python -u -m pytest tests/test_exact_gpu.py tests/test_search_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider && \
T ${TAG}_enc_tests 300 python -u -m pytest tests/test_encoder_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider && \
T ${TAG}_deep 200 python -u tools/deep_prof.py && \
T ${TAG}_deep1k 200 python -u tools/deep_prof.py --k 1000 && \
T ${TAG}_kt_deep 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt_deep -o run -- python -u tools/deep_prof.py --steps 3 && \
T ${TAG}_enc_prof 120 python tools/enc_prof.py --steps 10 && \
T ${TAG}_be 300 python -u bench.py --power-seconds 0 --no-cpu-baseline --no-configs0 --no-configs1 --no-configs4 --pipe-modes f32 --sweep '' --no-vendor-gemm --enc-modes f32,f16 --steps 5 --warmup 2 && \
echo ALLDONE
