T=tools/gpu_step.sh
for r in 1 2; do for v in v4 prio incr both; do $T ${v}$r 200 tests/debug/abl_$v v4 x || exit 1; done; done
