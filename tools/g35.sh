T=tools/gpu_step.sh
B="python bench.py --no-cpu-baseline --encoder none --steps 20"
for r in 1 2; do for st in 128 256 512 1024; do HCRAG_SAMPLE_STRIDE=$st $T s${st}_$r 300 $B || exit 1; done; done
