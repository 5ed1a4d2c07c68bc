#!/bin/bash
# r03_qsdiag.sh — what the QS epilogue's appends cost at configs[1] (1M x 384, B = 256, the
# default 128-deep stages, stride 16): stamps of the product kernel, of a build without the
# appends' global stores, and of one without the appends (diagnostic builds: wrong lists,
# timing only; make -C hc-rag_amd/csrc stamps stamps_qs_diag).
export TMPDIR=/tmp
T=tools/gpu_step.sh
$T qsd_base 120 env HCRAG_LIB=hc-rag_amd/lib/stamps/libhcrag_hip.so python tools/qs_stamps.py 1000000 384 256 0 16 && \
$T qsd_nostore 120 env HCRAG_LIB=hc-rag_amd/lib/stamps_nostore/libhcrag_hip.so python tools/qs_stamps.py 1000000 384 256 0 16 && \
$T qsd_noappend 200 env HCRAG_LIB=hc-rag_amd/lib/stamps_noappend/libhcrag_hip.so python tools/qs_stamps.py 1000000 384 256 0 16 && \
echo ALLDONE
