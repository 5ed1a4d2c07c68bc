#!/bin/bash
# ab_enc.sh TAG ROUNDS "ENV_A" "ENV_B" — interleaved A/B of the encoder legs (bge-base shape,
# S = 32, 1024 ragged queries, f32 and f16) under two environment settings, one bench process
# per arm and round (the hooks are read once per process); lines in gpurun_out/TAG_<arm>_<r>.json
TAG=$1; R=$2; A=$3; B=$4
ARGS="--rows 200000 --no-cpu-baseline --no-configs0 --no-configs1 --no-configs4 --no-vendor-gemm --sweep , --large-k , --power-seconds 0 --pipe-modes , --steps 3 --warmup 1"
mkdir -p gpurun_out
for r in $(seq 1 $R); do
  for arm in A B; do
    if [ $arm = A ]; then E=$A; else E=$B; fi
    env $E timeout -k 10 300 python bench.py $ARGS > gpurun_out/${TAG}_${arm}_${r}.json 2> gpurun_out/${TAG}_${arm}_${r}.log
    rc=$?
    if [ $rc -ne 0 ]; then echo "STOP $TAG $arm $r rc=$rc"; exit 99; fi
    python -c "import json,sys; d=json.load(open(sys.argv[1])); e=d['encoder']; print(sys.argv[2], sys.argv[3], *[(m, e[m]['query_embeddings_per_s'], e[m]['gpu_ms_per_batch']) for m in e])" gpurun_out/${TAG}_${arm}_${r}.json $arm "$E"
  done
done
