T=tools/gpu_step.sh
$T a4 200 tests/debug/abl_v4 v4 x && $T ans 200 tests/debug/abl_noslow ns x && $T ane 200 tests/debug/abl_noepi ne x
