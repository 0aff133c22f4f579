#!/bin/bash
# Build libcai variants for A/B sweeps: tools/build_variants.sh name1 "-DX=1" name2 "-DY=2" ...
# -> 165-.../lib/libcai_<name>.so (objects under csrc/build_<name>; both git-ignored)
set -e
CSRC=$(dirname $0)/../165-learning-based-multi-modality-image-and-video-compression_amd/csrc
while [ $# -ge 2 ]; do
  make -C $CSRC -j8 BUILD=build_$1 OUT=../lib/libcai_$1.so EXTRA="$2" ../lib/libcai_$1.so > /dev/null
  echo "built libcai_$1.so ($2)"
  shift 2
done
