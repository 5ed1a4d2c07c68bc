export TMPDIR=/tmp
T=tools/gpu_step.sh
B="python bench.py --no-cpu-baseline --steps 3 --enc-steps 10"
$T tests 500 python -u -m pytest tests/test_encoder_gpu.py -x -q --timeout 600 --timeout-method thread && \
$T be 200 $B && HCRAG_GEMM_NOP=1 $T benop 200 $B && \
$T kte 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kte -o run -- $B
