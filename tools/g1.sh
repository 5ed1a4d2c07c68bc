T=tools/gpu_step.sh
$T tests 300 python -u -m pytest tests/test_search_gpu.py -x -q --timeout 120 --timeout-method thread && \
$T bench 200 python bench.py --no-cpu-baseline --encoder none --steps 10 && \
HCRAG_NO_PREPASS=1 $T bench_nopre 200 python bench.py --no-cpu-baseline --encoder none --steps 10 && \
$T abl 200 tests/debug/abl_full && $T ablst 200 tests/debug/abl_stamps
