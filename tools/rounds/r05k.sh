#!/bin/bash
# r05k: QW stagger (waves 4-7's epilogue one stage late) at D = 384: parity, interleaved A/B at
# configs[1] (1M x 384, B = 256) and at 1M x 384 with 1024 queries.
export TMPDIR=/tmp
T=tools/gpu_step.sh
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
$T r05k_par 300 $P tests/test_qw_gpu.py -k "stagger" && \
$T r05k_c1 300 python tools/opt_ab.py 1000000 384 256 10 4 default QW_STAGGER=1 && \
$T r05k_c1b 300 python tools/opt_ab.py 1000000 384 1024 32 3 default QW_STAGGER=1 && \
echo ALLDONE_K
