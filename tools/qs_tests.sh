# qs_tests.sh TAG — search parity tests (incl. the QS kernel matrix), then qs_check.sh TAG.
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r02}
timeout -k 10 600 python -u -m pytest tests/test_search_gpu.py tests/test_exact_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${tag}_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
bash tools/qs_check.sh $tag
