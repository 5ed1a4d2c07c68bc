T=tools/gpu_step.sh
B="python bench.py --no-cpu-baseline --encoder none --steps 20"
for r in 1 2; do HCRAG_LIB=build_var/lib_prev.so $T prev$r 300 $B || exit 1; $T new$r 300 $B || exit 1; done
