#!/bin/bash
# ab_arms.sh TAG ROUNDS "ENV_1" "ENV_2" ... — interleaved A/B/C... of the headline search under
# several environment settings (hooks read once per process: one bench process per arm and
# round; "X=0" = the default build), each arm's bench line into gpurun_out/TAG_<i>_<round>.json.
# Bench arguments from $BENCH_ARGS (default: the headline search only, 20 timed steps).
TAG=$1; R=$2; shift 2
ARGS=${BENCH_ARGS:-"--no-cpu-baseline --encoder none --no-configs0 --no-configs1 --no-configs4 --no-vendor-gemm --sweep , --large-k , --power-seconds 0 --steps 20 --warmup 3"}
mkdir -p gpurun_out
for r in $(seq 1 $R); do
  i=0
  for E in "$@"; do
    i=$((i + 1))
    env $E timeout -k 10 300 python bench.py $ARGS > gpurun_out/${TAG}_${i}_${r}.json 2> gpurun_out/${TAG}_${i}_${r}.log
    rc=$?
    if [ $rc -ne 0 ]; then echo "STOP $TAG $i $r rc=$rc"; exit 99; fi
    python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], sys.argv[3], d['ms_per_step'], r['kernel_ms_avg'], r['frac'])" gpurun_out/${TAG}_${i}_${r}.json "$r" "$E" | tee -a gpurun_out/${TAG}_summary.txt
  done
done
