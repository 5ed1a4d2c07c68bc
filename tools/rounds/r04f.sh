#!/bin/bash
# r04f: where the split GEMM's stream-K time goes -- f32 encoder kernel traces (bge-base,
# 1024 x S = 32) with whole tiles (HCRAG_SPLIT_NOSK), stream-K, stream-K without the halves'
# meeting (HCRAG_SK_DIAG, timing only) and stream-K on 192-wide tiles; then the QS register-count
# appends: the configs[1] leg, its stamps and the QS / search tests.
export TMPDIR=/tmp
T=tools/gpu_step.sh
E="python bench.py --rows 200000 --no-cpu-baseline --no-configs0 --no-configs1 --no-configs4 --no-vendor-gemm --sweep , --large-k , --power-seconds 0 --pipe-modes , --steps 3 --warmup 1 --enc-steps 5 --enc-modes f32"
$T r04f_k_nosk 200 env HCRAG_SPLIT_NOSK=1 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04f_k_nosk -o run -- $E && \
$T r04f_k_sk 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04f_k_sk -o run -- $E && \
$T r04f_k_diag 200 env HCRAG_SK_DIAG=1 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04f_k_diag -o run -- $E && \
$T r04f_k_192 200 env HCRAG_GEMM_FT=192 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04f_k_192 -o run -- $E && \
$T r04f_qstests 400 python -u -m pytest tests/test_qs_forms_gpu.py tests/test_search_gpu.py tests/test_finish_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider && \
$T r04f_stamps 120 env HCRAG_LIB=hc-rag_amd/lib/stamps/libhcrag_hip.so python tools/qs_stamps.py 1000000 384 256 && \
$T r04f_c1 200 python bench.py --rows 200000 --encoder none --no-cpu-baseline --no-configs0 --no-configs4 --no-vendor-gemm --sweep 32,64,128,256 --large-k , --power-seconds 0 && \
echo ALLDONE_F
