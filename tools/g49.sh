T=tools/gpu_step.sh
$T ne 200 tests/debug/abl_noepi ne x && $T nq 200 tests/debug/abl_noqdma nq x
