T=tools/gpu_step.sh
$T cnt 200 tests/debug/abl_v4cnt c x
