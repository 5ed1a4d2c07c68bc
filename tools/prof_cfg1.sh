#!/bin/bash
# prof_cfg1.sh TAG [BATCHES] — kernel trace of the configs[1] search (1M x 384, k = 10) at B = 256
# (and 128): the per-kernel split of a batch (prep, pre-pass, seed, score, merge / finish).
tag=${1:-r02}
export TMPDIR=/tmp
mkdir -p gpurun_out
for b in ${2:-256 128}; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_cfg1_b$b -o run -- \
    python bench.py --rows 1000000 --dim 384 --global-batch $b --k 10 --steps 20 --warmup 3 --encoder none \
    --no-cpu-baseline --no-configs0 --no-configs1 --no-configs4 --sweep "" > gpurun_out/prof_${tag}_cfg1_b$b.json 2> gpurun_out/prof_${tag}_cfg1_b$b.err || exit 1
done
echo done
