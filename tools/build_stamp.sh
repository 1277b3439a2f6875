#!/bin/bash
# Diagnostic build: conv3x3.hip with -DCONV_STAMP=1 and head.hip with -DHEAD_STAMP=1, linked with the in-tree
# objects -> abl/libstamp.so (tools/conv_stamps.py, tools/head_stamps.py).  Never used by the product path.
set -e
cd "$(dirname "$0")/../enhanced-unet_amd"
make -s -j8 >/dev/null
mkdir -p ../abl
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function -Wno-unused-variable"
/opt/rocm/bin/hipcc $F -DCONV_STAMP=1 -c csrc/conv3x3.hip -o /tmp/conv3x3_stamp.o
/opt/rocm/bin/hipcc $F -DHEAD_STAMP=1 -c csrc/head.hip -o /tmp/head_stamp.o
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../abl/libstamp.so \
  $(ls build/*.o | grep -v "/conv3x3.o\|/head.o") /tmp/conv3x3_stamp.o /tmp/head_stamp.o
echo ../abl/libstamp.so
