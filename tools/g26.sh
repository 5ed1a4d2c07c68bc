T=tools/gpu_step.sh
B="python bench.py --no-cpu-baseline --encoder none --steps 20"
$T t 600 python -u -m pytest tests/test_search_gpu.py -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread && $T unit1 300 $B && HCRAG_NO_UNIT=1 $T nounit1 300 $B && $T unit2 300 $B && HCRAG_NO_UNIT=1 $T nounit2 300 $B
