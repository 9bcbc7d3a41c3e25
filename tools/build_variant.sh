# Builds the working tree's library with extra compiler flags into shuffle-coding_amd/lib_<name>/,
# for same-process A/B runs (tools/inproc_ab.py).  usage: bash tools/build_variant.sh <name> "<flags>"
set -e
NAME=$1; FLAGS=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
cp -r "$ROOT/shuffle-coding_amd" "$ROOT/include" "$TMP/"
rm -rf "$TMP/shuffle-coding_amd/build" "$TMP/shuffle-coding_amd/lib"
make -s -j8 -C "$TMP/shuffle-coding_amd" CXXFLAGS="-O3 -std=c++17 -fPIC -Wall -Wextra -Wno-unused-parameter $FLAGS"
mkdir -p "$ROOT/shuffle-coding_amd/lib_$NAME"
cp "$TMP/shuffle-coding_amd/lib/libshufflecoding_amd.so" "$ROOT/shuffle-coding_amd/lib_$NAME/"
rm -rf "$TMP"
echo "built working tree ($FLAGS) -> shuffle-coding_amd/lib_$NAME"
