T=tools/gpu_step.sh
B="python bench.py --no-cpu-baseline --encoder none --steps 20"
$T t 600 python -u -m pytest tests/test_search_gpu.py -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread && $T ao 200 tests/debug/abl_v4old v4 x && $T an 200 tests/debug/abl_v4 v4 x && $T ao2 200 tests/debug/abl_v4old v4 x && $T an2 200 tests/debug/abl_v4 v4 x && $T b1 300 $B && $T b2 300 $B
