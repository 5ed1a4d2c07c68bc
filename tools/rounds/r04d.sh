#!/bin/bash
# r04d: the suite after the compact QS epilogue and the 48-row QW default, the QS stamps, the
# configs[1] leg, then the r04c evidence set (headline traced in-process, its HBM traffic,
# encoder kernel trace).
export TMPDIR=/tmp
T=tools/gpu_step.sh
$T r04d_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider && \
$T r04d_stamps 120 env HCRAG_LIB=hc-rag_amd/lib/stamps/libhcrag_hip.so python tools/qs_stamps.py 1000000 384 256 && \
$T r04d_c1 200 python bench.py --rows 200000 --encoder none --no-cpu-baseline --no-configs0 --no-configs4 --no-vendor-gemm --sweep 32,64,128,256 --large-k , --power-seconds 0 && \
bash tools/rounds/r04c.sh && echo ALLDONE_D
