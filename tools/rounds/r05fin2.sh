#!/bin/bash
# r05fin2: smoke() and the default bench line at the final code (after r05tf).
export TMPDIR=/tmp
T=tools/gpu_step.sh
$T r05fin2_smoke 200 python -c "import __graft_entry__ as g; g.smoke()" && \
$T r05fin2_bench 600 python bench.py && \
echo ALLDONE_FIN2
