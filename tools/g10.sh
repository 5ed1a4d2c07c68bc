export TMPDIR=/tmp
T=tools/gpu_step.sh
B="python bench.py --no-cpu-baseline --encoder none --steps 10"
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES"
$T tests 300 python -u -m pytest tests/test_search_gpu.py -x -q --timeout 120 --timeout-method thread && \
$T abo 200 tests/debug/abl_orig x x && $T ab5 200 tests/debug/abl_v5 && \
$T b5 200 $B && HCRAG_V4=1 $T b4 200 $B && HCRAG_SAMPLE_STRIDE=64 $T b5s64 200 $B && \
$T p5 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/p5 -o run -- tests/debug/abl_v5
