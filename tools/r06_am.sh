#!/bin/bash
# r06_am.sh TAG -- HBM traffic of the deep k = 5000 path's kernels (1M x 384, 64 queries):
# FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes (MI355X_MICROARCH.md HBM section).
export TMPDIR=/tmp
TAG=${1:-r06am}
mkdir -p gpurun_out
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_fetch -o run -- python -u tools/deep_prof.py --steps 2 > gpurun_out/${TAG}_fetch.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_write -o run -- python -u tools/deep_prof.py --steps 2 > gpurun_out/${TAG}_write.log 2>&1 && \
echo ALLDONE
