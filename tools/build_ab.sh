#!/bin/bash
# A/B builds: libsndvae.so from the sources of git revision REV (default HEAD) into
# ab/<name>.so, loaded by the A/B tools through SND_LIB_PATH.  ab/ is git-ignored
# but travels to the GPU box.  usage: build_ab.sh NAME [REV] [-DFLAG...]
set -e
cd "$(dirname "$0")/.."
name=$1; shift
rev=${1:-HEAD}; [ $# -gt 0 ] && shift
tmp=$(mktemp -d)
git archive "$rev" include snd_vae_amd/csrc | tar -x -C "$tmp"
mkdir -p ab
objs=()
for src in "$tmp"/snd_vae_amd/csrc/*.hip; do
  o=$tmp/$(basename $src).o
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I "$tmp/include" -I "$tmp/snd_vae_amd/csrc" "$@" -c "$src" -o "$o" &
  objs+=("$o")
done
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ab/$name.so "${objs[@]}"
rm -rf "$tmp"
echo ab/$name.so
