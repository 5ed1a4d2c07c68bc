T=tools/gpu_step.sh
$T v6ne 120 tests/debug/abl_v6ne v6 x && $T v6 120 tests/debug/abl_v6 v6 x
