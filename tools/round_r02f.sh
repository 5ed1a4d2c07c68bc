#!/bin/bash
# round_r02b.sh — GPU evidence with the QW kernel as the headline's dense pass: full GPU test
# suite, smoke, default bench line, kernel trace + stats, FETCH_SIZE / WRITE_SIZE passes and an
# SQ pass (wave-cycle buckets, MFMA busy, clock) of the headline.  Every step under its own
# limit (tools/gpu_step.sh), chained with && (nothing runs after a failed or faulted step).
export TMPDIR=/tmp
T=tools/gpu_step.sh
Q="python bench.py --encoder none --no-cpu-baseline --no-configs0 --sweep ,"
$T r02f_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider && \
$T r02f_smoke 300 python -c "import __graft_entry__ as g; g.smoke()" && \
$T r02f_bench 600 python bench.py && \
$T r02f_kt 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02f_prof_kt -o run -- $Q --steps 10 --warmup 2 && \
$T r02f_fetch 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r02f_prof_fetch -o run -- $Q --steps 3 --warmup 1 && \
$T r02f_write 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r02f_prof_write -o run -- $Q --steps 3 --warmup 1 && \
$T r02f_sq 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/r02f_prof_sq -o run -- $Q --steps 3 --warmup 1 && \
echo ALLDONE
