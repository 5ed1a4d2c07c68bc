T=tools/gpu_step.sh
$T a4 200 tests/debug/abl_v4 v4 x && $T a4ro 200 tests/debug/abl_v4ro ro x && $T ane 200 tests/debug/abl_noepi ne x && $T b 300 python bench.py --no-cpu-baseline --encoder none --steps 20
