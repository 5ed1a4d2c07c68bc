T=tools/gpu_step.sh
$T t 600 python -u -m pytest tests/test_search_gpu.py -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -k "prepass or v5"
