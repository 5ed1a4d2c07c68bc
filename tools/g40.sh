T=tools/gpu_step.sh
$T st 200 tests/debug/abl_stamps st x
