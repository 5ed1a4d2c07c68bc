T=tools/gpu_step.sh
S="python bench.py --no-cpu-baseline --encoder none --steps 3 --warmup 1 --sweep 1,16,64,128"
for r in 1 2; do $T b$r 300 $S || exit 1; HCRAG_LIB=build_var/lib_nt.so $T nt$r 300 $S || exit 1; done
