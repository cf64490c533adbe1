# Per-kernel resource usage (VGPRs, SGPRs, scratch, LDS) of the gfx950 code objects inside a built
# library: tools/kernel_resources.sh [lib] [name-regex].  Offline (build container), no GPU.  The
# fatbin holds one offload bundle per translation unit, compressed (CCOB, --offload-compress) or not.
LIB=${1:-minigrid_dynamicprogramming_amd/libmgdp.so}
PAT=${2:-.}
T=$(mktemp -d)
objcopy --dump-section .hip_fatbin=$T/fat.bin "$LIB" &&
python3 - "$T" <<'PY'
import struct, sys
d = sys.argv[1]
b = open(d + "/fat.bin", "rb").read()
starts = []
i = 0
while True:  # bundles start at a magic: compressed "CCOB" or plain "__CLANG_OFFLOAD_BUNDLE__"
    j = min([x for x in (b.find(b"CCOB", i), b.find(b"__CLANG_OFFLOAD_BUNDLE__", i)) if x >= 0], default=-1)
    if j < 0:
        break
    starts.append(j)
    i = j + 4
for n, s in enumerate(starts):
    if b[s:s + 4] == b"CCOB":
        ver = struct.unpack("<H", b[s + 4:s + 6])[0]
        size = struct.unpack("<Q", b[s + 8:s + 16])[0] if ver >= 3 else struct.unpack("<I", b[s + 8:s + 12])[0]
    else:
        size = (starts[n + 1] if n + 1 < len(starts) else len(b)) - s
    open(f"{d}/b{n}.bin", "wb").write(b[s:s + size])
PY
for f in $T/b*.bin; do
  /opt/rocm/lib/llvm/bin/clang-offload-bundler --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 \
    --input=$f --output=$f.co --unbundle --allow-missing-bundles 2>/dev/null || continue
  [ -s $f.co ] || continue
  /opt/rocm/lib/llvm/bin/llvm-readelf --notes $f.co
done | python3 -c "
import re, sys
txt = sys.stdin.read()
pat = re.compile(sys.argv[1])
for blk in txt.split('\n  - .agpr_count')[1:]:
    def f(k):
        m = re.search(r'\.' + k + r':\s+(\S+)', blk)
        return m.group(1) if m else '?'
    name = f('name')
    if pat.search(name):
        print(f'vgpr {f(\"vgpr_count\"):>4} sgpr {f(\"sgpr_count\"):>4} scratch {f(\"private_segment_fixed_size\"):>5} lds {f(\"group_segment_fixed_size\"):>6}  {name[:160]}')
" "$PAT"
rm -rf $T
