T=tools/gpu_step.sh
B="python bench.py --no-cpu-baseline --encoder none --steps 20"
$T base 300 $B && HCRAG_DEBUG_KEEP_TAUG=1 $T keep 300 $B && HCRAG_DEBUG_KEEP_TAUG=1 HCRAG_DEBUG_ORACLE_TAU=64 $T orc64 300 $B && HCRAG_DEBUG_KEEP_TAUG=1 HCRAG_DEBUG_ORACLE_TAU=16 $T orc16 300 $B && $T base2 300 $B
