set -o pipefail
export TMPDIR=/tmp
bash tools/sess_flat.sh || exit 1
bash tools/sweep_env.sh tune bunny_cornell f32 "base RT_AMD_TRAV_PCT=35 RT_AMD_TRAV_PCT=65 RT_AMD_LEAF_EXIT_PCT=15 RT_AMD_LEAF_EXIT_PCT=40" || exit 1
bash tools/sweep_env.sh tune bunny_cornell f64 "base RT_AMD_TRAV_PCT=35 RT_AMD_TRAV_PCT=65 RT_AMD_LEAF_EXIT_PCT=15 RT_AMD_LEAF_EXIT_PCT=40" || exit 1
bash tools/sweep_env.sh tune pawn_fog f64 "base RT_AMD_TRAV_PCT=60 RT_AMD_TRAV_PCT=90 RT_AMD_LEAF_EXIT_PCT=40 RT_AMD_LEAF_EXIT_PCT=70" 3 || exit 1
