T=tools/gpu_step.sh
K="tests/test_encoder_gpu.py -q -m gpu -p no:cacheprovider"
$T n1 300 python -m pytest $K && $T n2 300 python -m pytest $K && $T n3 300 python -m pytest $K
