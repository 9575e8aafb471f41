#!/bin/bash
# Build the libraries of another git revision in-tree for A/B timing against the working tree:
# tools/ab_build.sh REV NAME  ->  convolutional-codes_amd/build_ab/NAME/lib/*.so (git-ignored, travels
# to the GPU box). Load it with CCV_LIB_DIR=$PWD/convolutional-codes_amd/build_ab/NAME/lib.
set -eu
cd "$(dirname "$0")/.."
REV=$1 NAME=$2
SRC=/tmp/ab_src_$NAME
rm -rf $SRC && mkdir -p $SRC
git archive "$REV" include convolutional-codes_amd | tar -x -C $SRC
make -C $SRC/convolutional-codes_amd -j8 > /tmp/ab_build_$NAME.log 2>&1
mkdir -p convolutional-codes_amd/build_ab/$NAME
rm -rf convolutional-codes_amd/build_ab/$NAME/lib
cp -r $SRC/convolutional-codes_amd/lib convolutional-codes_amd/build_ab/$NAME/lib
echo "built $REV into convolutional-codes_amd/build_ab/$NAME/lib"
