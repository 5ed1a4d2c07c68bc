#!/bin/bash
# r04p: encoder parity with stream-K opt-in (whole tiles by default), then the default bench line.
export TMPDIR=/tmp
T=tools/gpu_step.sh
$T r04p_enctests 500 python -u -m pytest tests/test_encoder_gpu.py tests/test_configs0_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider && \
$T r04p_bench 600 python bench.py && \
echo ALLDONE_P
