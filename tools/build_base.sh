# Builds the library as of a git revision (default HEAD) into shuffle-coding_amd/lib_<name>/,
# for same-box A/B runs with tools/inproc_ab.py or tools/gpu_ab.sh.  usage: bash tools/build_base.sh [rev] [name]
set -e
REV=${1:-HEAD}; NAME=${2:-base}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
git -C "$ROOT" archive "$REV" shuffle-coding_amd include | tar -x -C "$TMP"
make -s -j8 -C "$TMP/shuffle-coding_amd"
mkdir -p "$ROOT/shuffle-coding_amd/lib_$NAME"
cp "$TMP/shuffle-coding_amd/lib/libshufflecoding_amd.so" "$ROOT/shuffle-coding_amd/lib_$NAME/"
rm -rf "$TMP"
echo "built $REV -> shuffle-coding_amd/lib_$NAME"
