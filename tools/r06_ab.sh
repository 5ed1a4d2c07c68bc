#!/bin/bash
# r06_ab.sh TAG -- two-launch K6 (K6c compaction + K6r rescoring) and the flag store folded into
# the finish launch: exact/search GPU tests; deep k A/B against the inline K6m (alternating
# processes); configs[1] flag-read arms; kernel traces.
export TMPDIR=/tmp
TAG=${1:-r06ab}
S=tools/gpu_step.sh
mkdir -p gpurun_out
T() { "$S" "$@"; r=$?; [ $r -eq 99 ] && exit 99; return $r; }
T ${TAG}_exact 400 python -u -m pytest tests/test_exact_gpu.py -m gpu -x -q --timeout 280 --timeout-method thread -p no:cacheprovider && \
T ${TAG}_deepA1 120 python -u tools/deep_prof.py && \
T ${TAG}_deepB1 120 env HCRAG_K6_INLINE=1 python -u tools/deep_prof.py && \
T ${TAG}_deepA2 120 python -u tools/deep_prof.py && \
T ${TAG}_deepB2 120 env HCRAG_K6_INLINE=1 python -u tools/deep_prof.py && \
T ${TAG}_deep1kA 120 python -u tools/deep_prof.py --k 1000 && \
T ${TAG}_deep1kB 120 env HCRAG_K6_INLINE=1 python -u tools/deep_prof.py --k 1000 && \
T ${TAG}_ab 300 python -u tools/opt_ab.py 1000000 384 256 10 6 FLAG_READ=1 FLAG_READ=3 default && \
T ${TAG}_kt_deep 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt_deep -o run -- python -u tools/deep_prof.py --steps 3 && \
T ${TAG}_search 400 python -u -m pytest tests/test_search_gpu.py tests/test_global_seed_gpu.py -m gpu -x -q --timeout 280 --timeout-method thread -p no:cacheprovider && \
echo ALLDONE
