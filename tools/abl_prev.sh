#!/bin/bash
# A/B baseline build: abl/libprev.so = the in-tree library with csrc/<name>.hip of each named source taken from
# git revision ${REV:-HEAD} (the other objects as built now).  Diagnostic only; the product loads the in-tree
# library.   tools/abl_prev.sh conv3x3 [head ...]
set -e
cd "$(dirname "$0")/.."
make -s -C enhanced-unet_amd -j8 >/dev/null
mkdir -p abl
objs=$(ls enhanced-unet_amd/build/*.o)
prev=""
for src in "$@"; do
  git show ${REV:-HEAD}:enhanced-unet_amd/csrc/$src.hip > abl/${src}_prev.hip
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function -Wno-unused-variable -Wno-inline-asm \
    -Ienhanced-unet_amd/csrc -c abl/${src}_prev.hip -o abl/${src}_prev.o
  objs=$(echo "$objs" | grep -v "/$src.o")
  prev="$prev abl/${src}_prev.o"
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o abl/libprev.so $objs $prev
for src in "$@"; do rm -f abl/${src}_prev.hip abl/${src}_prev.o; done
echo abl/libprev.so
