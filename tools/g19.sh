T=tools/gpu_step.sh
K="tests/test_encoder_gpu.py -q -m gpu -k minilm_shape -p no:cacheprovider"
for i in 1 2 3; do HCRAG_LIB=$PWD/build_var/lib_old.so $T old$i 200 python -m pytest $K || exit 1; done
for i in 1 2 3; do HCRAG_GEMM_FT=256 $T new$i 200 python -m pytest $K || exit 1; done
