#!/bin/bash
# r04g: QS appends staged in rolling LDS slots -- its tests, the configs[1] leg, stamps (a no-store
# diagnostic build was dropped: its garbage candidate ids reached the rescore's row gather); the
# split GEMM's tile-width rule under stream-K (A/B against whole-tile rounds).
export TMPDIR=/tmp
T=tools/gpu_step.sh
$T r04g_qstests 400 python -u -m pytest tests/test_qs_forms_gpu.py tests/test_search_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider && \
$T r04g_stamps 120 env HCRAG_LIB=hc-rag_amd/lib/stamps/libhcrag_hip.so python tools/qs_stamps.py 1000000 384 256 && \
$T r04g_c1 200 python bench.py --rows 200000 --encoder none --no-cpu-baseline --no-configs0 --no-configs4 --no-vendor-gemm --sweep 32,256 --large-k , --power-seconds 0 && \
$T r04g_ab 500 tools/ab_enc.sh r04g_ab 2 HCRAG_SPLIT_NOSK=1 X=0 && \
echo ALLDONE_G
