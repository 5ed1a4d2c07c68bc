T=tools/gpu_step.sh
$T tests 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread && $T bench 300 python bench.py
