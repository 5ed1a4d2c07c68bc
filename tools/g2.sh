T=tools/gpu_step.sh
$T abo 200 tests/debug/abl_orig && $T abl 200 tests/debug/abl_full && $T abls 200 tests/debug/abl_split && $T abo2 200 tests/debug/abl_orig && $T abl2 200 tests/debug/abl_full && $T abls2 200 tests/debug/abl_split
