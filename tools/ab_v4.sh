# ab_v4.sh TAG — headline bench, product library vs hc-rag_amd/lib/ab_old (the previous
# commit's build), alternated twice in one call; then the search parity tests.
set -o pipefail
tag=${1:-r02}
mkdir -p gpurun_out
B="python bench.py --steps 10 --warmup 2 --encoder none --no-cpu-baseline --no-configs0 --sweep 256,512"
for r in 1 2; do
  HCRAG_LIB=hc-rag_amd/lib/ab_old/libhcrag_hip.so timeout -k 10 300 $B > gpurun_out/${tag}_old_$r.json 2>/dev/null || exit 1
  timeout -k 10 300 $B > gpurun_out/${tag}_new_$r.json 2>/dev/null || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_search_gpu.py tests/test_exact_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${tag}_tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
