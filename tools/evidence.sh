#!/bin/bash
# evidence.sh TAG — the round-end set on one box, every GPU step under its own limit and chained
# with && (gpu_step.sh): every -m gpu test, smoke(), the default bench line, a kernel trace of the
# headline search (configs[2]), and configs[1]'s kernel trace + FETCH_SIZE / WRITE_SIZE passes
# (HBM traffic per search: tools/pmc_summary.py).  Output: gpurun_out/TAG_*
export TMPDIR=/tmp
T=tools/gpu_step.sh
TAG=${1:-evidence}
H="python bench.py --no-cpu-baseline --encoder none --no-configs0 --no-configs1 --no-configs4 --no-vendor-gemm --sweep ,"
C1="python bench.py --rows 1000000 --dim 384 --global-batch 256 --k 10 --encoder none --no-cpu-baseline --no-configs0 --no-configs1 --no-configs4 --no-vendor-gemm --sweep ,"
$T ${TAG}_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider && \
$T ${TAG}_smoke 200 python -c "import __graft_entry__ as g; g.smoke()" && \
$T ${TAG}_bench 600 python bench.py && \
$T ${TAG}_kt 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt -o run -- $H --steps 10 --warmup 2 && \
$T ${TAG}_c1_kt 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_c1_kt -o run -- $C1 --steps 20 --warmup 3 && \
$T ${TAG}_c1_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_c1_fetch -o run -- $C1 --steps 4 --warmup 1 && \
$T ${TAG}_c1_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_c1_write -o run -- $C1 --steps 4 --warmup 1 && \
echo ALLDONE
