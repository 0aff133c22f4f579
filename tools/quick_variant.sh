#!/bin/bash
# Build lib/libcai_<name>.so from the default build's objects with ONE source recompiled under extra flags
# (A/B and diagnostic variants of a single kernel file).  usage: tools/quick_variant.sh <name> <file.hip> "<flags>"
set -e
name=$1; src=$2; flags=$3
CSRC=$(cd $(dirname $0)/../165-learning-based-multi-modality-image-and-video-compression_amd/csrc && pwd)
make -C $CSRC -j8 > /dev/null
tmp=$CSRC/build_$name; mkdir -p $tmp
base=${src%.hip}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -I$CSRC/../../include \
    $flags -c $CSRC/$src -o $tmp/$base.o
objs=$(ls $CSRC/build/*.o | grep -v "/$base.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs $tmp/$base.o -o $CSRC/../lib/libcai_$name.so
echo "built libcai_$name.so ($src: $flags)"
