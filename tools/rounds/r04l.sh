#!/bin/bash
# r04l: the f32 query pipeline's encoder time with and without the split GEMM's stream-K
export TMPDIR=/tmp
T=tools/gpu_step.sh
$T r04l_pipe 700 tools/ab_pipe.sh r04l_pipe 2 HCRAG_SPLIT_NOSK=1 X=0 && echo ALLDONE_L
