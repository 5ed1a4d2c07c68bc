#!/bin/bash
# prof_cfg1_pmc.sh TAG — configs[1] (1M x 384, B = 256, k = 10): kernel trace + stats, then the
# FETCH_SIZE and WRITE_SIZE passes (separate runs, each under its own limit).
export TMPDIR=/tmp
tag=${1:-r02}
mkdir -p gpurun_out
B="python bench.py --rows 1000000 --dim 384 --global-batch 256 --k 10 --encoder none --no-cpu-baseline --no-configs0 --sweep ,"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_cfg1_kt -o run -- $B --steps 20 --warmup 3 > gpurun_out/${tag}_cfg1_kt.json 2>/dev/null && \
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${tag}_cfg1_fetch -o run -- $B --steps 4 --warmup 1 > /dev/null 2>&1 && \
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${tag}_cfg1_write -o run -- $B --steps 4 --warmup 1 > /dev/null 2>&1 && echo done
