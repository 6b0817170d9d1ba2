#!/bin/bash
# A/B experiment builds of libsndvae.so with extra -D flags into tools/_exp/<name>.so
# (loaded through SND_LIB_PATH by the profiling tools).  usage: build_exp.sh NAME -DFLAG...
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p tools/_exp/$name.objs
objs=()
for src in snd_vae_amd/csrc/*.hip; do
  o=tools/_exp/$name.objs/$(basename $src).o
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I include -I snd_vae_amd/csrc "$@" -c $src -o $o &
  objs+=($o)
done
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o tools/_exp/$name.so "${objs[@]}"
rm -rf tools/_exp/$name.objs
echo tools/_exp/$name.so
