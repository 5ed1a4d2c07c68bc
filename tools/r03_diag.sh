#!/bin/bash
# r03_diag.sh — power / clocks of the headline dense pass (QW vs QW1), QW1 and QS stamps at
# configs[1], kernel traces of configs[1] and of the W = 8 rank shape (finish kernel in).
export TMPDIR=/tmp
T=tools/gpu_step.sh
$T r03e_power 240 python -u tools/power_watch.py --shape c2 --variants 0,1 --seconds 6 && \
HCRAG_LIB=hc-rag_amd/lib/stamps_qw1/libhcrag_hip.so $T r03e_st_c1 200 python -u tools/qw1_stamps.py 1000000 384 256 1 0 && \
HCRAG_LIB=hc-rag_amd/lib/stamps/libhcrag_hip.so $T r03e_qs_c1 200 python -u tools/qs_stamps.py 1000000 384 256 && \
$T r03e_cfg1 300 tools/prof_cfg1.sh r03 256 && \
$T r03e_rs8 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rs_w8_kt_r03 -o run -- python bench.py --encoder none --no-cpu-baseline --no-configs0 --no-configs1 --no-configs4 --sweep , --steps 30 --warmup 3 --rows 1250000 && \
echo ALLDONE
