T=tools/gpu_step.sh
B="python bench.py --no-cpu-baseline --encoder none --steps 20"
$T t 600 python -u -m pytest tests/test_search_gpu.py -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread && $T mx1 300 $B && HCRAG_PREPASS_TOPK=1 $T tk1 300 $B && HCRAG_SAMPLE_STRIDE=32 $T m32 300 $B && HCRAG_SAMPLE_STRIDE=128 $T m128 300 $B && $T mx2 300 $B && HCRAG_PREPASS_TOPK=1 $T tk2 300 $B
