T=tools/gpu_step.sh
$T gr 300 python -u -m pytest tests/test_graph_relevance.py tests/test_relevance.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread
