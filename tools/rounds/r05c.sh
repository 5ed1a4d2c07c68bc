#!/bin/bash
# r05c: (1) the exact fallback with 4 query groups per scan + the sampled round-0 histogram
# (tests + the bench's large-k leg); (2) QW DM 4 (spread DMA issue + partition sync) vs 0 / 3:
# parity, stamps, interleaved timing, FETCH_SIZE, SQ counters (MFMA busy, clock).
export TMPDIR=/tmp
T=tools/gpu_step.sh
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
S="env HCRAG_LIB=hc-rag_amd/lib/stamps_qw/libhcrag_hip.so"
B="python bench.py --no-cpu-baseline --encoder none --no-configs0 --no-configs1 --no-configs4 --no-vendor-gemm --sweep , --large-k , --power-seconds 0 --steps 3 --warmup 1"
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
$T r05c_exact 600 $P tests/test_exact_gpu.py && \
$T r05c_lk 300 python bench.py --no-cpu-baseline --encoder none --no-configs0 --no-configs1 --no-configs4 --no-vendor-gemm --sweep , --power-seconds 0 --steps 3 --warmup 1 && \
$T r05c_par4 300 env HCRAG_QW_DM=4 $P tests/test_qw_gpu.py && \
$T r05c_st4 200 $S HCRAG_QW_DM=4 python tools/qw_stamps.py 10000000 768 1024 && \
$T r05c_ab 900 tools/ab_arms.sh r05c 3 X=0 HCRAG_QW_DM=3 HCRAG_QW_DM=4 && \
$T r05c_f4 120 env HCRAG_QW_DM=4 timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r05c_f4 -o run -- $B && \
$T r05c_sq0 120 timeout -s KILL 110 rocprofv3 --pmc $SQ --output-format csv -d gpurun_out/r05c_sq0 -o run -- $B && \
$T r05c_sq4 120 env HCRAG_QW_DM=4 timeout -s KILL 110 rocprofv3 --pmc $SQ --output-format csv -d gpurun_out/r05c_sq4 -o run -- $B && \
$T r05c_sq3 120 env HCRAG_QW_DM=3 timeout -s KILL 110 rocprofv3 --pmc $SQ --output-format csv -d gpurun_out/r05c_sq3 -o run -- $B && \
echo ALLDONE_C &&
# configs[1] (1M x 384, B = 256, k = 10) and B = 256 at 10M x 768: QS vs QW, pre-pass forms, DMA modes
$T r05c_c1 600 python tools/opt_ab.py 1000000 384 256 10 3 default PREPASS=2 QW_MIN=129 QW_MIN=129,QW_DM=3 QW_MIN=129,QW_DM=1 && \
$T r05c_b256 600 python tools/opt_ab.py 10000000 768 256 32 3 default QW_DM=3 QW_DM=1 && \
echo ALLDONE_C2
