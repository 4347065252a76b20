set -o pipefail
export TMPDIR=/tmp
bash tools/ab_libs.sh g7/ab "readme:1 demo1:1 bunny_cornell:1 pawn_fog:1 cornell:1" 3
echo exit $?
