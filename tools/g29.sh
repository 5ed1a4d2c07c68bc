T=tools/gpu_step.sh
HCRAG_DEBUG_UNIT=1 $T b 300 python bench.py --no-cpu-baseline --encoder none --steps 2 --warmup 1
