#!/bin/bash
# r05d: QW by default from 129 queries at D = 384 with spread DMA for one query block; the
# pipelined MFMA prefilter scan (large k); the MFMA-shape microbenchmark;
# QW stamps at configs[1].
export TMPDIR=/tmp
T=tools/gpu_step.sh
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
S="env HCRAG_LIB=hc-rag_amd/lib/stamps_qw/libhcrag_hip.so"
$T r05d_tests 900 $P tests/test_qw_gpu.py tests/test_qs_forms_gpu.py tests/test_exact_gpu.py tests/test_search_gpu.py && \
$T r05d_c1full 300 $P tests/test_full_size_gpu.py -k configs1 && \
$T r05d_lk 300 python bench.py --no-cpu-baseline --encoder none --no-configs0 --no-configs1 --no-configs4 --no-vendor-gemm --sweep , --power-seconds 0 --steps 3 --warmup 1 && \
$T r05d_shape 300 tools/bin/mfma_shape_ab 40000 3 && \
$T r05d_st_c1_3 200 $S python tools/qw_stamps.py 1000000 384 256 10 && \
$T r05d_st_c1_0 200 $S python tools/qw_stamps.py 1000000 384 256 10 QW_DM=0 && \
$T r05d_c1 600 python tools/opt_ab.py 1000000 384 256 10 3 default QW_MIN=100000 && \
echo ALLDONE_D
