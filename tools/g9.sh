export TMPDIR=/tmp
T=tools/gpu_step.sh
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES"
$T p4 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/p4 -o run -- tests/debug/abl_orig x x && \
$T p5 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/p5 -o run -- tests/debug/abl_v5 && \
$T p5n 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/p5n -o run -- tests/debug/abl_v5noepi
