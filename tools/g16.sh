export TMPDIR=/tmp
T=tools/gpu_step.sh
B="python bench.py --no-cpu-baseline --steps 1 --warmup 1 --enc-steps 3 --rows 1000000"
S="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
$T pf 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pf -o run -- $B && \
$T pt 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pt -o run -- $B && \
$T ps 200 rocprofv3 --pmc $S --output-format csv -d gpurun_out/ps -o run -- $B && \
HCRAG_GEMM_P=1 $T pt2 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pt2 -o run -- $B
