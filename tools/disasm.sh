# Disassembles one built unit's gfx950 code object: bash tools/disasm.sh ans_launch_enc_u8 > /tmp/x.s
B=/opt/rocm/lib/llvm/bin
T=$(mktemp -d)
$B/llvm-objcopy --dump-section=.hip_fatbin=$T/f.bin "$(dirname "$0")/../shuffle-coding_amd/build/$1.o"
$B/clang-offload-bundler --unbundle --type=o --input=$T/f.bin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/k.co
$B/llvm-objdump -d --no-show-raw-insn $T/k.co
rm -rf $T
