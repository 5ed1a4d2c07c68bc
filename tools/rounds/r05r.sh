#!/bin/bash
# r05r: QW / QW1 / QS / search tests after the final-lists stride change; the merge + rescore
# kernel's phase stamps at configs[1] and B = 512; configs[1] kernel trace.
export TMPDIR=/tmp
T=tools/gpu_step.sh
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
F="env HCRAG_LIB=hc-rag_amd/lib/stamps_fin/libhcrag_hip.so"
$T r05r_tests 400 $P tests/test_qw_gpu.py tests/test_qw1_gpu.py tests/test_qs_forms_gpu.py tests/test_search_gpu.py && \
$T r05r_fs_c1 200 $F python tools/finish_stamps.py 1000000 384 256 10 && \
$T r05r_fs_512 200 $F python tools/finish_stamps.py 1000000 768 512 32 && \
$T r05r_kt_c1 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05r_kt_c1 -o run -- python tools/opt_ab.py 1000000 384 256 10 1 default && \
echo ALLDONE_R
