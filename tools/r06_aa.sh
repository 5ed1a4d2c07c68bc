#!/bin/bash
# r06_aa.sh TAG -- HCR_OPT_FLAG_READ: exact/search GPU tests, configs[1] interleaved A/B of the
# pass's flag read-back (1 pageable copy, 2 pinned copy, 3 kernel store + poll + sync, 4 no sync),
# configs[1] kernel trace at the new default.
export TMPDIR=/tmp
TAG=${1:-r06aa}
S=tools/gpu_step.sh
mkdir -p gpurun_out
T() { "$S" "$@"; r=$?; [ $r -eq 99 ] && exit 99; return $r; }
T ${TAG}_tests 300 python -u -m pytest tests/test_exact_gpu.py -k "flag_read or out_of_range" -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider && \
T ${TAG}_ab 300 python -u tools/opt_ab.py 1000000 384 256 10 6 FLAG_READ=1 FLAG_READ=2 FLAG_READ=3 FLAG_READ=4 && \
T ${TAG}_ab768 300 python -u tools/opt_ab.py 1250000 768 1024 32 3 FLAG_READ=1 FLAG_READ=4 && \
T ${TAG}_kt_c1 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt_c1 -o run -- \
    python bench.py --rows 1000000 --dim 384 --global-batch 256 --k 10 --steps 20 --warmup 3 --encoder none \
    --no-cpu-baseline --no-configs0 --no-configs1 --no-configs4 --sweep "" && \
echo ALLDONE
