#!/bin/bash
# r06_h.sh TAG -- why the bench's f32 encoder leg runs 15.8 ms against enc_prof's 13.3: the
# power / clock sampler thread on and off (enc_prof and bench's encoder leg), one and two
# streams; then the deep top-k (k = 5000, 64 queries, 1M x 384) kernel trace.
export TMPDIR=/tmp
TAG=${1:-r06h}
S=tools/gpu_step.sh
mkdir -p gpurun_out
T() { "$S" "$@"; r=$?; [ $r -eq 99 ] && exit 99; return 0; }
AB() { timeout -k 10 120 env "$@" python tools/enc_prof.py --steps 10 ${POW:+--power} | sed "s|\"split_dm\"|\"env\": \"$* pow=${POW:-0}\", \"split_dm\"|" >> gpurun_out/${TAG}_ab.jsonl 2>> gpurun_out/${TAG}_ab.err || exit 99; }
for r in 1 2; do
  POW= AB HCRAG_ENC_STREAMS=2 && POW=1 AB HCRAG_ENC_STREAMS=2 && POW= AB HCRAG_ENC_STREAMS=1 && POW=1 AB HCRAG_ENC_STREAMS=1 || exit 99
done
BE() { tag=$1; ev=$2; shift 2; timeout -k 10 240 env $ev python -u bench.py --rows 200000 --power-seconds 0 --no-cpu-baseline --no-configs0 --no-configs1 --no-configs4 --pipe-modes f32 --sweep '' --large-k '' --no-vendor-gemm --enc-modes f32 --steps 5 --warmup 2 "$@" > gpurun_out/${TAG}_be_${tag}.log 2>&1 || exit 99; }
BE pow_s2 HCRAG_ENC_STREAMS=2 && BE nopow_s2 HCRAG_ENC_STREAMS=2 --no-leg-power && BE pow_s1 HCRAG_ENC_STREAMS=1 && BE nopow_s1 HCRAG_ENC_STREAMS=1 --no-leg-power && \
T ${TAG}_kt_bench_enc 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt_bench_enc -o run -- python -u bench.py --rows 200000 --power-seconds 0 --no-cpu-baseline --no-configs0 --no-configs1 --no-configs4 --pipe-modes '' --sweep '' --large-k '' --no-vendor-gemm --enc-modes f32 --steps 5 --warmup 2 && \
T ${TAG}_deep 200 python -u tools/deep_prof.py && \
T ${TAG}_kt_deep 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt_deep -o run -- python -u tools/deep_prof.py --steps 3 && \
echo ALLDONE
