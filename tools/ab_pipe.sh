#!/bin/bash
# ab_pipe.sh TAG ROUNDS "ENV_A" "ENV_B" — interleaved A/B of the f32 encoder leg and the f32
# query pipeline (bge-base S = 32 -> certified top-k on the 10M x 768 corpus), one bench process
# per arm and round; prints encoder emb/s, pipeline q/s and the pipeline's encoder-only ms.
TAG=$1; R=$2; A=$3; B=$4
ARGS="--no-cpu-baseline --no-configs0 --no-configs1 --no-configs4 --no-vendor-gemm --sweep , --large-k , --power-seconds 0 --enc-modes f32 --pipe-modes f32 --steps 3 --warmup 1"
mkdir -p gpurun_out
for r in $(seq 1 $R); do
  for arm in A B; do
    if [ $arm = A ]; then E=$A; else E=$B; fi
    env $E timeout -k 10 300 python bench.py $ARGS > gpurun_out/${TAG}_${arm}_${r}.json 2> gpurun_out/${TAG}_${arm}_${r}.log
    rc=$?
    if [ $rc -ne 0 ]; then echo "STOP $TAG $arm $r rc=$rc"; exit 99; fi
    python -c "import json,sys; d=json.load(open(sys.argv[1])); e=d['encoder']['f32']; p=d['query_pipeline']['f32']; print(sys.argv[2], sys.argv[3], e['query_embeddings_per_s'], e['ms_per_batch'], p['query_pipeline_qps'], p['ms_per_step'], p['encoder_ms'], p['search_ms'])" gpurun_out/${TAG}_${arm}_${r}.json $arm "$E"
  done
done
