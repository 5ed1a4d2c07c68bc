export TMPDIR=/tmp
T=tools/gpu_step.sh
B="python bench.py --no-cpu-baseline --encoder none --steps 10"
HCRAG_DEBUG_KEEP_TAUG=1 $T bwarm 200 $B && HCRAG_SAMPLE_STRIDE=64 $T b64 200 $B && \
HCRAG_SAMPLE_STRIDE=64 $T kt64 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt64 -o run -- $B && \
$T kt16 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt16 -o run -- $B
