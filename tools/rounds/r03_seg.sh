#!/bin/bash
# r03_seg.sh — QS with lane-private segmented candidate buffers: the full -m gpu suite, the QS
# stamps at configs[1], the configs[1] A/B of the QS stage depth, and a kernel trace of
# configs[1] (per-kernel times vs profiles/r03/evidence_b).
export TMPDIR=/tmp
T=tools/gpu_step.sh
C1="python bench.py --rows 1000000 --dim 384 --global-batch 256 --k 10 --encoder none --no-cpu-baseline --no-configs0 --no-configs1 --no-configs4 --no-vendor-gemm --sweep ,"
$T seg_tests 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider && \
$T seg_stamps 120 env HCRAG_LIB=hc-rag_amd/lib/stamps/libhcrag_hip.so python tools/qs_stamps.py 1000000 384 256 0 16 && \
$T seg_ab_c1 300 python tools/qw1_ab.py --shapes c1 --rounds 4 --reps 7 --variants=-1:0:0:0,-1:0:0:1,-1:0:0:4 && \
$T seg_c1_kt 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/seg_c1_kt -o run -- $C1 --steps 20 --warmup 3 && \
echo ALLDONE
