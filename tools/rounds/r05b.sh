#!/bin/bash
# r05b: QW stage DMA-issue modes (HCRAG_QW_DM 0 / 1 / 2 / 3: every wave at the barrier / waves 0-3
# at the barrier / waves 0-3 spread over their MFMA groups / every wave spread): parity,
# stamps, interleaved timing, FETCH_SIZE of the dense launch; and the r05 correctness tests
# (deep k, planted key).
export TMPDIR=/tmp
T=tools/gpu_step.sh
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
S="env HCRAG_LIB=hc-rag_amd/lib/stamps_qw/libhcrag_hip.so"
B="python bench.py --no-cpu-baseline --encoder none --no-configs0 --no-configs1 --no-configs4 --no-vendor-gemm --sweep , --large-k , --power-seconds 0 --steps 3 --warmup 1"
$T r05b_deep 400 $P tests/test_exact_gpu.py tests/test_llama_gpu.py -k "deep or out_of_range or vector_store" && \
$T r05b_par 600 bash -c "for m in 1 2 3; do HCRAG_QW_DM=\$m $P tests/test_qw_gpu.py || exit 1; done" && \
$T r05b_st1 200 $S HCRAG_QW_DM=1 python tools/qw_stamps.py 10000000 768 1024 && \
$T r05b_st2 200 $S HCRAG_QW_DM=2 python tools/qw_stamps.py 10000000 768 1024 && \
$T r05b_st3 200 $S HCRAG_QW_DM=3 python tools/qw_stamps.py 10000000 768 1024 && \
$T r05b_ab 1000 tools/ab_arms.sh r05b 2 X=0 HCRAG_QW_DM=1 HCRAG_QW_DM=2 HCRAG_QW_DM=3 && \
$T r05b_f0 120 timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r05b_f0 -o run -- $B && \
$T r05b_f3 120 env HCRAG_QW_DM=3 timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r05b_f3 -o run -- $B && \
echo ALLDONE_B
