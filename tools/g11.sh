export TMPDIR=/tmp
T=tools/gpu_step.sh
$T tests 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread && \
$T smoke 120 python -c "import __graft_entry__ as g; g.smoke()" && \
$T bench 400 python bench.py && \
$T kt 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt -o run -- python bench.py --no-cpu-baseline --steps 10
