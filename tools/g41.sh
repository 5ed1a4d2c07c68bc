T=tools/gpu_step.sh
$T v6 120 tests/debug/abl_v6 v6 x
