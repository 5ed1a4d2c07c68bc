# qs_check.sh TAG — stamps of the QS kernel (diagnostic build) + batch sweeps at 1M x 384 and
# 10M x 768 with the product library.  Run under gpurun from the repo root.
set -o pipefail
tag=${1:-r02}
mkdir -p gpurun_out
HCRAG_LIB=hc-rag_amd/lib/stamps/libhcrag_hip.so timeout -k 10 120 python tools/qs_stamps.py 1000000 384 128 > gpurun_out/${tag}_stamps_1M_384.txt 2>&1 || exit 1
HCRAG_LIB=hc-rag_amd/lib/stamps/libhcrag_hip.so timeout -k 10 120 python tools/qs_stamps.py 1000000 768 128 > gpurun_out/${tag}_stamps_1M_768.txt 2>&1 || exit 1
timeout -k 10 200 python bench.py --rows 1000000 --dim 384 --global-batch 256 --k 10 --steps 20 --encoder none --no-cpu-baseline --no-configs0 --sweep 32,64,128,256 > gpurun_out/${tag}_cfg1.json 2> gpurun_out/${tag}_cfg1.err || exit 1
timeout -k 10 300 python bench.py --steps 3 --encoder none --no-cpu-baseline --no-configs0 --sweep 1,32,64,128 > gpurun_out/${tag}_cfg2.json 2> gpurun_out/${tag}_cfg2.err || exit 1
echo done
