T=tools/gpu_step.sh
$T t 600 python -u -m pytest tests/test_search_gpu.py tests/test_relevance.py tests/test_graph_relevance.py tests/test_ingest.py -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread && $T sw 400 python bench.py --no-cpu-baseline --encoder none --steps 10 --sweep 1,16,64,128,256,512,1024
