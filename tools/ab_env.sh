#!/bin/bash
# ab_env.sh TAG ROUNDS "ENV_A" "ENV_B" [bench args...] — interleaved A/B of the headline search
# under two environment settings (test hooks read once per process: one bench process per arm
# and round), each arm's bench line into gpurun_out/TAG_<arm>_<round>.json.  GPU steps under
# their own limits, chained so that a failed step ends the script.
TAG=$1; R=$2; A=$3; B=$4; shift 4
ARGS=${*:-"--no-cpu-baseline --encoder none --no-configs0 --no-configs1 --no-configs4 --no-vendor-gemm --sweep , --large-k , --power-seconds 0 --steps 20 --warmup 3"}
mkdir -p gpurun_out
for r in $(seq 1 $R); do
  for arm in A B; do
    if [ $arm = A ]; then E=$A; else E=$B; fi
    env $E timeout -k 10 300 python bench.py $ARGS > gpurun_out/${TAG}_${arm}_${r}.json 2> gpurun_out/${TAG}_${arm}_${r}.log
    rc=$?
    if [ $rc -ne 0 ]; then echo "STOP $TAG $arm $r rc=$rc"; exit 99; fi
    python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], sys.argv[3], d['ms_per_step'], r['kernel_ms_avg'], r['frac'])" gpurun_out/${TAG}_${arm}_${r}.json $arm "$E"
  done
done
