#!/bin/bash
# r04a: the suite after the r04 changes, the default bench line, and the A/Bs of the QW stage
# shape (HCRAG_QW_SR) and stage test (HCRAG_QW_OLDTEST) and of the split GEMM's stage issue
# (HCRAG_SPLIT_EARLY).  Every GPU step under its own limit, chained with && (gpu_step.sh).
export TMPDIR=/tmp
python tools/sysfs_probe.py > gpurun_out/r04a_sysfs.log 2>&1
T=tools/gpu_step.sh
$T r04a_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider && \
$T r04a_smoke 200 python -c "import __graft_entry__ as g; g.smoke()" && \
$T r04a_bench 400 python bench.py && \
$T r04a_qwt 200 tools/ab_env.sh r04a_qwt 1 HCRAG_QW_OLDTEST=1 X=0 && \
$T r04a_ab 200 tools/ab_env.sh r04a_ab 1 HCRAG_QW_SR=32 HCRAG_QW_SR=48 && \
$T r04a_enc 200 tools/ab_enc.sh r04a_enc 1 X=0 HCRAG_SPLIT_EARLY=1 && \
$T r04a_enc2 200 tools/ab_enc.sh r04a_enc2 1 "HCRAG_ENC_PADDED=1 HCRAG_ENC_STREAMS=1" HCRAG_ENC_STREAMS=1 && \
echo ALLDONE
