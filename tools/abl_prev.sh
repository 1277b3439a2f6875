#!/bin/bash
# A/B baseline build: abl/libprev.so = the in-tree library with csrc/$1.hip taken from git revision ${REV:-HEAD}
# (the other objects as built now).  Diagnostic only; the product loads the in-tree library.
set -e
cd "$(dirname "$0")/.."
make -s -C enhanced-unet_amd -j8 >/dev/null
mkdir -p abl
src=$1
git show ${REV:-HEAD}:enhanced-unet_amd/csrc/$src.hip > abl/${src}_prev.hip
objs=$(ls enhanced-unet_amd/build/*.o | grep -v "/$src.o")
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function -Wno-unused-variable \
  -Ienhanced-unet_amd/csrc -c abl/${src}_prev.hip -o abl/${src}_prev.o
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o abl/libprev.so $objs abl/${src}_prev.o
rm -f abl/${src}_prev.hip abl/${src}_prev.o
echo abl/libprev.so
