#!/bin/bash
# r05l: the GPU suite with the staggered epilogue on by default at D = 384, then QW stagger
# variants A/B (0 off / 1 two accumulator sets / 2 one set) at configs[1] and 1M x 384 B = 1024.
export TMPDIR=/tmp
T=tools/gpu_step.sh
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
$T r05l_tests 600 $P tests -m gpu && \
$T r05l_c1 300 python tools/opt_ab.py 1000000 384 256 10 4 default QW_STAGGER=2 QW_STAGGER=0 && \
$T r05l_c1b 300 python tools/opt_ab.py 1000000 384 1024 32 3 default QW_STAGGER=2 QW_STAGGER=0 && \
echo ALLDONE_L
