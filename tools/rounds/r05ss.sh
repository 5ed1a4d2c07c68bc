#!/bin/bash
# r05ss: seed select from the valid keys' common prefix, two bits a step -- configs[1] bench leg,
# new vs lib/ab_old (HEAD) in alternating processes, then the GPU suite.
export TMPDIR=/tmp
T=tools/gpu_step.sh
O="env HCRAG_LIB=$PWD/hc-rag_amd/lib/ab_old/libhcrag_hip.so"
ARGS="--rows 200000 --encoder none --no-cpu-baseline --no-configs0 --no-configs4 --no-vendor-gemm --sweep , --large-k , --power-seconds 0 --steps 3 --warmup 1"
show() { python -c "import json,sys; d=json.load(open(sys.argv[1]))['configs1']; print(sys.argv[2], d['ms_per_step'], d['score_kernel_ms'], d['uncertified_queries'])" gpurun_out/$1.json $2; }
for r in 1 2 3; do
  $T r05ss_new_$r 200 sh -c "python bench.py $ARGS > gpurun_out/r05ss_new_$r.json" && show r05ss_new_$r new && \
  $T r05ss_old_$r 200 sh -c "$O python bench.py $ARGS > gpurun_out/r05ss_old_$r.json" && show r05ss_old_$r old || exit 1
done && \
$T r05ss_tests 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu && \
echo ALLDONE_TF
