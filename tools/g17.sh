T=tools/gpu_step.sh
$T tests 500 python -u -m pytest tests/test_relevance.py tests/test_ingest.py -x -q -m gpu --timeout 300 --timeout-method thread
