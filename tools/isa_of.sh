# Disassembles one kernel of the built library's gfx950 code object (from build/<obj>.o's
# .hip_fatbin) into a file, and prints its per-block instruction counts (tools/asm_blocks.py).
# usage: bash tools/isa_of.sh <kernel-name-substring> [obj=ans_kernels] [out=/tmp/kernel.s]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
B=/opt/rocm/lib/llvm/bin
OBJ=${2:-ans_kernels}
OUT=${3:-/tmp/kernel.s}
T=$(mktemp -d)
$B/llvm-objcopy --dump-section=.hip_fatbin=$T/fat.bin "$ROOT/shuffle-coding_amd/build/$OBJ.o"
$B/clang-offload-bundler --unbundle --type=o --input=$T/fat.bin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/k.co
$B/llvm-objdump -d --no-show-raw-insn $T/k.co > $T/k.s
python3 "$ROOT/tools/asm_blocks.py" $T/k.s "$1" "$OUT"
rm -rf $T
