#!/bin/bash
# r05fin: the GPU suite and smoke() at HEAD after the A/B hooks were removed.
export TMPDIR=/tmp
T=tools/gpu_step.sh
$T r05fin_tests 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu && \
$T r05fin_smoke 200 python -c "import __graft_entry__ as g; g.smoke()" && \
echo ALLDONE_FIN
