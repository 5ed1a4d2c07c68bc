#!/bin/bash
# r06_ac.sh TAG -- fallback init kernels (no per-group copies / per-round memsets); K6 scan and
# K6r grid sizes A/B at deep k (alternating processes); exact GPU tests.
export TMPDIR=/tmp
TAG=${1:-r06ac}
S=tools/gpu_step.sh
mkdir -p gpurun_out
T() { "$S" "$@"; r=$?; [ $r -eq 99 ] && exit 99; return $r; }
T ${TAG}_exact 400 python -u -m pytest tests/test_exact_gpu.py -m gpu -x -q --timeout 280 --timeout-method thread -p no:cacheprovider || exit 1
for rep in 1 2; do
  T ${TAG}_d_def_$rep 120 python -u tools/deep_prof.py || exit 1
  T ${TAG}_d_c256_$rep 120 env HCRAG_K6_CHUNKS=256 HCRAG_K6R_BLOCKS=256 python -u tools/deep_prof.py || exit 1
  T ${TAG}_d_c512_$rep 120 env HCRAG_K6_CHUNKS=512 HCRAG_K6R_BLOCKS=512 python -u tools/deep_prof.py || exit 1
  T ${TAG}_d_c1024_$rep 120 env HCRAG_K6_CHUNKS=1024 HCRAG_K6R_BLOCKS=256 python -u tools/deep_prof.py || exit 1
  T ${TAG}_d_c256i_$rep 120 env HCRAG_K6_CHUNKS=256 HCRAG_K6_INLINE=1 python -u tools/deep_prof.py || exit 1
  T ${TAG}_d_inl_$rep 120 env HCRAG_K6_INLINE=1 python -u tools/deep_prof.py || exit 1
done
T ${TAG}_kt_c256 200 env HCRAG_K6_CHUNKS=256 HCRAG_K6R_BLOCKS=256 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt_c256 -o run -- python -u tools/deep_prof.py --steps 3 && \
T ${TAG}_kt_def 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt_def -o run -- python -u tools/deep_prof.py --steps 3 && \
echo ALLDONE
