#!/bin/bash
# Diagnostic variant builds of libeunet_hip: [SRC=head] tools/abl_build.sh NAME "-DMACRO=V ..." -> abl/libNAME.so
# (run conv_bench against one with EUNET_LIB=abl/libNAME.so).  Never used by the product path.
set -e
cd "$(dirname "$0")/../enhanced-unet_amd"
make -s -j8 >/dev/null
mkdir -p ../abl
name=$1; shift
src=${SRC:-conv3x3}  # the one source file rebuilt with the variant flags
objs=$(ls build/*.o | grep -v "/$src.o")
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function -Wno-unused-variable -Wno-inline-asm $@ -c csrc/$src.hip -o ../abl/${src}_$name.o
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../abl/lib$name.so $objs ../abl/${src}_$name.o
echo ../abl/lib$name.so
