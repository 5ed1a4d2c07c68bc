set -o pipefail
mkdir -p gpurun_out
for q in 128 256; do
HCRAG_QS_MAX=$q timeout -k 10 200 python bench.py --rows 1000000 --dim 384 --global-batch 256 --k 10 --steps 20 --encoder none --no-cpu-baseline --no-configs0 --sweep 160,200,256 > gpurun_out/ab256_cfg1_$q.json 2>/dev/null || exit 1
HCRAG_QS_MAX=$q timeout -k 10 300 python bench.py --steps 2 --encoder none --no-cpu-baseline --no-configs0 --sweep 160,256 > gpurun_out/ab256_cfg2_$q.json 2>/dev/null || exit 1
done
echo done
