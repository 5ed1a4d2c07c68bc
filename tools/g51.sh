T=tools/gpu_step.sh
B="python bench.py --no-cpu-baseline --encoder none --steps 20"
for r in 1 2; do $T base$r 300 $B || exit 1; HCRAG_LIB=build_var/lib_fc.so $T fc$r 300 $B || exit 1; done
