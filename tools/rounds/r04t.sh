#!/bin/bash
# r04t: the split reduction reading two slabs at a time -- parity, trace, encoder leg.
export TMPDIR=/tmp
T=tools/gpu_step.sh
E="python bench.py --rows 200000 --no-cpu-baseline --no-configs0 --no-configs1 --no-configs4 --no-vendor-gemm --sweep , --large-k , --power-seconds 0 --pipe-modes , --enc-modes f32 --steps 3 --warmup 1 --enc-steps 10"
$T r04t_enctests 400 python -u -m pytest tests/test_encoder_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "split or two_stream or packed or full_depth or variants" && \
$T r04t_77 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04t_77 -o run -- $E --enc-seed 77 && \
$T r04t_enc 300 $E && \
echo ALLDONE_T
