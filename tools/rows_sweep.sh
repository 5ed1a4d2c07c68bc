# rows_sweep.sh TAG — score-kernel time vs corpus size at D = 384 (B = 128: QS; B = 256: v4):
# the fixed cost per launch is the intercept.  Run under gpurun from the repo root.
set -o pipefail
tag=${1:-r02}
mkdir -p gpurun_out
for b in 128 256; do for r in 1000000 2000000 4000000 8000000; do
  timeout -k 10 200 python bench.py --rows $r --dim 384 --global-batch $b --k 10 --steps 10 --warmup 2 --encoder none \
    --no-cpu-baseline --no-configs0 --sweep "" > gpurun_out/${tag}_rows_${b}_${r}.json 2> gpurun_out/${tag}_rows_${b}_${r}.err || exit 1
done; done
echo done
