T=tools/gpu_step.sh
HCRAG_LIB=build_var/lib_cnt.so $T bc 300 python bench.py --no-cpu-baseline --encoder none --steps 2 --warmup 1
