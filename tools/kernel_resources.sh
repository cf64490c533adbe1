# Per-kernel resource usage (VGPRs, SGPRs, scratch, LDS) of the gfx950 code object inside a built
# library: tools/kernel_resources.sh [lib] [name-regex].  Offline (build container), no GPU.
LIB=${1:-minigrid_dynamicprogramming_amd/libmgdp.so}
PAT=${2:-.}
T=$(mktemp -d)
objcopy --dump-section .hip_fatbin=$T/fat.bin "$LIB" &&
/opt/rocm/lib/llvm/bin/clang-offload-bundler --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 \
  --input=$T/fat.bin --output=$T/x.co --unbundle --allow-missing-bundles &&
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $T/x.co | python3 -c "
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
