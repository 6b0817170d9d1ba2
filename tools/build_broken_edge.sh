#!/bin/bash
# A deliberately broken library for the parity bars' sensitivity check: HEAD's sources
# with the round-5 dot2 operand fix of the per-edge logit (commit bc3298b, snd_gather.hpp
# dot8_bf16) reverted, i.e. the per-edge logits hipcc miscompiled for one session.  Output:
# ab/edge_broken.so (git-ignored, travels to the GPU box); load it with
# SND_LIB_PATH=ab/edge_broken.so.  tests/test_gpu_c2_bench.py::...[bf16] must FAIL on it.
set -e
cd "$(dirname "$0")/.."
tmp=$(mktemp -d)
git archive HEAD include snd_vae_amd/csrc | tar -x -C "$tmp"
# only the per-edge logit (dot8_bf16) goes back to the miscompiled form; the gather sums
# (acc8v) keep their fix, so the library is wrong exactly where round 5's was
python3 - "$tmp/snd_vae_amd/csrc/snd_gather.hpp" <<'PY'
import sys
p = sys.argv[1]; s = open(p).read()
old = "acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(gbf16x2, wa[p]), __builtin_bit_cast(gbf16x2, wb[p]),"
new = "acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(gbf16x2, a[p]), __builtin_bit_cast(gbf16x2, b[p]),"
assert s.count(old) == 1
open(p, "w").write(s.replace(old, new))
PY
grep -q "__builtin_bit_cast(gbf16x2, a\[p\])" "$tmp/snd_vae_amd/csrc/snd_gather.hpp"
mkdir -p ab
objs=()
for src in "$tmp"/snd_vae_amd/csrc/*.hip; do
  o=$tmp/$(basename $src).o
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I "$tmp/include" -I "$tmp/snd_vae_amd/csrc" -c "$src" -o "$o" &
  objs+=("$o")
done
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ab/edge_broken.so "${objs[@]}"
rm -rf "$tmp"
echo ab/edge_broken.so
