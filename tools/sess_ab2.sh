set -o pipefail
export TMPDIR=/tmp
export RT_AMD_GRID_RESERVE=0
STEPS=20 bash tools/ab_session.sh ab2 "cornell:1 readme:1 cornell:8" || exit 1
bash tools/sweep_env.sh tune2 pawn_fog f32 "base RT_AMD_LEAF_EXIT_PCT=70 RT_AMD_LEAF_EXIT_PCT=85" 3 || exit 1
bash tools/sweep_env.sh tune2 pawn_fog f64 "RT_AMD_LEAF_EXIT_PCT=85" 3 || exit 1
