#!/bin/bash
# r04j: the whole GPU suite at HEAD, then smoke().
export TMPDIR=/tmp
T=tools/gpu_step.sh
$T r04j_tests 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider && \
$T r04j_smoke 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" && \
echo ALLDONE_J
