T=tools/gpu_step.sh
$T tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread && \
$T smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
