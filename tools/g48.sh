export TMPDIR=/tmp
T=tools/gpu_step.sh
$T kn 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/g48_norm -o run -- python bench.py --no-cpu-baseline --encoder none --steps 3 --warmup 1 && HCRAG_LIB=build_var/lib_noepi.so $T ke 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/g48_noepi -o run -- python bench.py --no-cpu-baseline --encoder none --steps 3 --warmup 1
