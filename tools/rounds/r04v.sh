#!/bin/bash
# r04v: the headline with and without the sampling pre-pass (A/B)
export TMPDIR=/tmp
T=tools/gpu_step.sh
$T r04v_prepass 500 tools/ab_env.sh r04v_prepass 2 HCRAG_NO_PREPASS=1 X=0 && echo ALLDONE_V
