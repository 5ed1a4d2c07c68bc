#!/bin/bash
# Full GPU validation of HEAD: parity suite, smoke, default bench line
T=tools/gpu_step.sh
$T gpu_tests 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread && \
$T smoke 200 python -c "import __graft_entry__ as g; g.smoke()" && \
$T bench 400 python bench.py
