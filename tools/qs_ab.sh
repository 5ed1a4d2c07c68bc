# A/B of the query-stationary kernel (HCRAG_QS_MAX=256, default) against the v3/v4 tiles
# (HCRAG_QS_MAX=0) on configs[1] (1M x 384, B = 256) and the headline corpus (10M x 768),
# after the search parity tests.  Run under gpurun from the repo root.
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r02j}
timeout -k 10 400 python -u -m pytest tests/test_search_gpu.py tests/test_exact_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${tag}_tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
for q in 0 256; do
  HCRAG_QS_MAX=$q timeout -k 10 200 python bench.py --rows 1000000 --dim 384 --global-batch 256 --k 10 --steps 20 --encoder none --no-cpu-baseline --no-configs0 --sweep 32,64,128,256 > gpurun_out/${tag}_cfg1_$q.json 2> gpurun_out/${tag}_cfg1_$q.err || exit 1
  HCRAG_QS_MAX=$q timeout -k 10 300 python bench.py --steps 3 --encoder none --no-cpu-baseline --no-configs0 --sweep 32,64,128,256 > gpurun_out/${tag}_cfg2_$q.json 2> gpurun_out/${tag}_cfg2_$q.err || exit 1
done
echo done
