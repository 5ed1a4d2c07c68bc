T=tools/gpu_step.sh
K="-k minilm_shape"
HCRAG_GEMM_FT=256 $T t256 300 python -m pytest tests/test_encoder_gpu.py -q -m gpu $K && \
HCRAG_GEMM_FT=256 HCRAG_LN_SCALAR=1 $T t256ln 300 python -m pytest tests/test_encoder_gpu.py -q -m gpu $K && \
HCRAG_GEMM_FT=256 HCRAG_SCALAR_ATTENTION=1 $T t256at 300 python -m pytest tests/test_encoder_gpu.py -q -m gpu $K && \
HCRAG_GEMM_FT=192 $T t192 300 python -m pytest tests/test_encoder_gpu.py -q -m gpu $K
