T=tools/gpu_step.sh
$T te1 400 python -m pytest tests/test_encoder_gpu.py -q -m gpu -x && \
HCRAG_GEMM_FT=256 $T te2 300 python -m pytest tests/test_encoder_gpu.py -q -m gpu -k "tiny_ragged or minilm_shape or cls_pooling" && \
HCRAG_GEMM_FT=256 $T te3 300 python -m pytest tests/test_encoder_gpu.py -q -m gpu -k "tiny_ragged or minilm_shape or cls_pooling"
