# enc_check.sh TAG — encoder GPU tests (incl. configs[0]) + the bench's encoder block.
set -o pipefail
tag=${1:-r02}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_encoder_gpu.py tests/test_configs0_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${tag}_enc_tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/${tag}_enc_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_enc_tests.log
timeout -k 10 300 python bench.py --rows 100000 --steps 2 --warmup 1 --encoder bge-base --enc-modes f32,f16 --no-cpu-baseline --no-configs0 --sweep "" > gpurun_out/${tag}_enc.json 2>/dev/null || exit 1
python - <<'PY' gpurun_out/${tag}_enc.json
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for m, e in d["encoder"].items():
    print(m, e["query_embeddings_per_s"], e["ms_per_batch"], e["TFLOPs"], e["mfma_frac"], e.get("mfma_frac_executed"))
PY
