T=tools/gpu_step.sh
$T ao 200 tests/debug/abl_v4old v4 x && $T an 200 tests/debug/abl_v4 v4 x && $T ao2 200 tests/debug/abl_v4old v4 x && $T an2 200 tests/debug/abl_v4 v4 x
