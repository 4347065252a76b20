set -o pipefail
export TMPDIR=/tmp
export RT_AMD_GRID_RESERVE=0
STEPS=20 bash tools/ab_session.sh ab3 "cornell:1 readme:1 cornell:8 bunny_cornell:1" || exit 1
