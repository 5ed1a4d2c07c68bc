#!/bin/bash
# ab_c1.sh TAG ROUNDS "ENV_A" "ENV_B" — interleaved A/B of the configs[1] leg (1M x 384 f16,
# B = 256, k = 10) under two environment settings, one bench process per arm and round; prints
# the step and score-kernel ms and the kernel id of each.
TAG=$1; R=$2; A=$3; B=$4
ARGS="--rows 200000 --encoder none --no-cpu-baseline --no-configs0 --no-configs4 --no-vendor-gemm --sweep , --large-k , --power-seconds 0 --steps 3 --warmup 1"
mkdir -p gpurun_out
for r in $(seq 1 $R); do
  for arm in A B; do
    if [ $arm = A ]; then E=$A; else E=$B; fi
    env $E timeout -k 10 300 python bench.py $ARGS > gpurun_out/${TAG}_${arm}_${r}.json 2> gpurun_out/${TAG}_${arm}_${r}.log
    rc=$?
    if [ $rc -ne 0 ]; then echo "STOP $TAG $arm $r rc=$rc"; exit 99; fi
    python -c "import json,sys; d=json.load(open(sys.argv[1]))['configs1']; print(sys.argv[2], sys.argv[3], d['ms_per_step'], d['score_kernel_ms'], d['score_kernel'], d['uncertified_queries'])" gpurun_out/${TAG}_${arm}_${r}.json $arm "$E"
  done
done
