#!/bin/bash
# round_r02.sh — the round's GPU evidence: full GPU test suite, smoke, default bench line,
# kernel trace + stats and the FETCH_SIZE / WRITE_SIZE passes of the headline score phase.
# Every step under its own limit (tools/gpu_step.sh), chained with && (nothing runs after a
# failed or faulted step).  Output: gpurun_out/r02_*.
export TMPDIR=/tmp
T=tools/gpu_step.sh
$T r02_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider && \
$T r02_smoke 300 python -c "import __graft_entry__ as g; g.smoke()" && \
$T r02_bench 600 python bench.py && \
$T r02_kt 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02_prof_kt -o run -- python bench.py --steps 5 --warmup 2 --encoder none --no-cpu-baseline --no-configs0 --sweep "" && \
$T r02_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r02_prof_fetch -o run -- python bench.py --steps 3 --warmup 1 --encoder none --no-cpu-baseline --no-configs0 --sweep "" && \
$T r02_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r02_prof_write -o run -- python bench.py --steps 3 --warmup 1 --encoder none --no-cpu-baseline --no-configs0 --sweep "" && \
echo ALLDONE
