T=tools/gpu_step.sh
$T abo 200 tests/debug/abl_orig x x && $T ab5 200 tests/debug/abl_v5 && $T ab5z 200 tests/debug/abl_v5z && \
$T abst 200 tests/debug/abl_stamps x x && $T ab5st 200 tests/debug/abl_v5st && $T ab5zst 200 tests/debug/abl_v5zst
