T=tools/gpu_step.sh
$T tests 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread && $T smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" && $T bench 400 python bench.py
