T=tools/gpu_step.sh
K="tests/test_encoder_gpu.py -q -m gpu -p no:cacheprovider"
HCRAG_LIB=$PWD/build_var/lib_old.so $T old1 300 python -m pytest $K && HCRAG_LIB=$PWD/build_var/lib_old.so $T old2 300 python -m pytest $K && \
$T new1 300 python -m pytest $K && $T new2 300 python -m pytest $K
