#!/bin/bash
# r05g: QW stamps with the in-kernel clock at configs[1], B = 256 and the headline; configs[1]
# kernel trace (the whole search step's kernels).
export TMPDIR=/tmp
T=tools/gpu_step.sh
S="env HCRAG_LIB=hc-rag_amd/lib/stamps_qw/libhcrag_hip.so"
$T r05g_st_c1 200 $S python tools/qw_stamps.py 1000000 384 256 10 && \
$T r05g_st_b256 200 $S python tools/qw_stamps.py 10000000 768 256 32 && \
$T r05g_st_c2 200 $S python tools/qw_stamps.py 10000000 768 1024 32 && \
$T r05g_kt_c1 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05g_kt_c1 -o run -- python tools/opt_ab.py 1000000 384 256 10 1 default && \
echo ALLDONE_G
