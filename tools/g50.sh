T=tools/gpu_step.sh
$T sw 400 python bench.py --no-cpu-baseline --encoder none --steps 5 --sweep 1,8,16,32,64,128,256,512,1024,2048,4096
