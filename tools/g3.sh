T=tools/gpu_step.sh
B="python bench.py --no-cpu-baseline --encoder none --steps 10"
$T abo 200 tests/debug/abl_orig && $T abls 200 tests/debug/abl_split && \
$T b16 200 $B && HCRAG_SAMPLE_STRIDE=32 $T b32 200 $B && HCRAG_SAMPLE_STRIDE=64 $T b64 200 $B && \
HCRAG_SAMPLE_STRIDE=128 $T b128 200 $B && HCRAG_SAMPLE_STRIDE=256 $T b256 200 $B && HCRAG_NO_PREPASS=1 $T bno 200 $B
