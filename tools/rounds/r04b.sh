#!/bin/bash
# r04b: configs[1] -- QS issue-priority A/B (HCRAG_QS_PRIO), a kernel trace with timestamps
# (what the per-search fill is), the stamps build's per-tile split -- and the 48-row QW route's
# parity (HCRAG_QW_SR=48) on the QW tests.
export TMPDIR=/tmp
T=tools/gpu_step.sh
C1="python bench.py --rows 1000000 --dim 384 --global-batch 256 --k 10 --encoder none --no-cpu-baseline --no-configs0 --no-configs1 --no-configs4 --no-vendor-gemm --sweep , --large-k , --power-seconds 0"
$T r04b_prio 300 tools/ab_env.sh r04b_prio 2 X=0 HCRAG_QS_PRIO=1 --rows 1000000 --dim 384 --global-batch 256 --k 10 --encoder none --no-cpu-baseline --no-configs0 --no-configs1 --no-configs4 --no-vendor-gemm --sweep , --large-k , --power-seconds 0 --steps 50 --warmup 5 && \
$T r04b_c1kt 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04b_c1kt -o run -- $C1 --steps 20 --warmup 3 && \
$T r04b_stamps 120 env HCRAG_LIB=hc-rag_amd/lib/stamps/libhcrag_hip.so python tools/qs_stamps.py 1000000 384 256 && \
$T r04b_ab 300 tools/ab_env.sh r04b_ab 3 HCRAG_QW_SR=32 HCRAG_QW_SR=48 && \
$T r04b_qw48 200 env HCRAG_QW_SR=48 python -u -m pytest tests/test_qw_gpu.py tests/test_search_gpu.py -k "qw or rank or multiblock" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider && \
echo ALLDONE
