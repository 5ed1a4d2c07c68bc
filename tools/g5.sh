T=tools/gpu_step.sh
B="python bench.py --no-cpu-baseline --encoder none --steps 10"
$T tests 300 python -u -m pytest tests/test_search_gpu.py -x -q --timeout 120 --timeout-method thread && \
$T abo 200 tests/debug/abl_orig x x && $T ab5 200 tests/debug/abl_v5 && \
$T b5 200 $B && HCRAG_V4=1 $T b4 200 $B && HCRAG_NO_UNIT=1 $T b5inv 200 $B && HCRAG_DEBUG_KEEP_TAUG=1 $T b5warm 200 $B
