T=tools/gpu_step.sh
B="python bench.py --no-cpu-baseline --encoder none --steps 20"
$T t 600 python -u -m pytest tests/test_search_gpu.py -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread && $T est1 300 $B && HCRAG_RIGOROUS_SEED=1 $T rig1 300 $B && HCRAG_SAMPLE_STRIDE=128 $T s128 300 $B && $T est2 300 $B && HCRAG_RIGOROUS_SEED=1 $T rig2 300 $B && HCRAG_SAMPLE_STRIDE=32 $T s32 300 $B
