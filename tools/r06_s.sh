#!/bin/bash
# r06_s.sh TAG -- configs[1] (1M x 384, B = 256, k = 10) with and without the sampling pre-pass
# (HCRAG_NO_PREPASS=1: the dense pass starts from no seed), alternating processes on one box.
export TMPDIR=/tmp
TAG=${1:-r06s}
mkdir -p gpurun_out
for r in 1 2 3; do
  timeout -k 10 150 python tools/opt_ab.py 1000000 384 256 10 2 default >> gpurun_out/${TAG}_ab.txt 2>&1 || exit 99
  timeout -k 10 150 env HCRAG_NO_PREPASS=1 python tools/opt_ab.py 1000000 384 256 10 2 default >> gpurun_out/${TAG}_ab_noprepass.txt 2>&1 || exit 99
done
grep -i 'median\|summary' gpurun_out/${TAG}_ab.txt gpurun_out/${TAG}_ab_noprepass.txt
