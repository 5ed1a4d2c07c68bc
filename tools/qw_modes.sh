#!/bin/bash
# qw_modes.sh — issue-schedule A/B of the QW kernel: per variant the headline's score ms and the
# FETCH_SIZE of the dense launch (L2 sharing between the 4 query blocks of a row partition).
export TMPDIR=/tmp
B="python bench.py --encoder none --no-cpu-baseline --no-configs0 --sweep ,"
for v in 0 3 4 5; do
  HCRAG_QW_VARIANT=$v timeout -k 10 200 $B --steps 10 --warmup 2 > gpurun_out/mode_$v.log 2>&1 || exit 1
  HCRAG_QW_VARIANT=$v timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/mode_${v}_fetch -o run -- $B --steps 3 --warmup 1 > /dev/null 2>&1 || exit 1
  echo "variant $v done"
done
echo ALLDONE
