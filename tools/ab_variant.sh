#!/bin/bash
# Build the WORKING TREE's libraries with extra compiler flags for A/B timing (kernel variants behind
# macros): tools/ab_variant.sh NAME OBJ "flags" -> convolutional-codes_amd/build_ab/NAME/lib. Only
# build/OBJ.o is recompiled (the other objects are copied from the tree's current build/); load the
# result with CCV_LIB_DIR=$PWD/convolutional-codes_amd/build_ab/NAME/lib.
set -eu
cd "$(dirname "$0")/.."
NAME=$1 OBJ=$2 FLAGS=$3
SRC=/tmp/abv_src_$NAME
rm -rf $SRC && mkdir -p $SRC
cp -r include $SRC/
mkdir -p $SRC/convolutional-codes_amd
cp -rp convolutional-codes_amd/csrc convolutional-codes_amd/Makefile convolutional-codes_amd/build $SRC/convolutional-codes_amd/
rm -f $SRC/convolutional-codes_amd/build/$OBJ.o
make -C $SRC/convolutional-codes_amd -j8 HIPFLAGS="-O3 -std=c++20 -fPIC --offload-arch=gfx950 -fno-slp-vectorize -Wall -Wno-unused-function $FLAGS" > /tmp/abv_$NAME.log 2>&1
mkdir -p convolutional-codes_amd/build_ab/$NAME
rm -rf convolutional-codes_amd/build_ab/$NAME/lib
cp -r $SRC/convolutional-codes_amd/lib convolutional-codes_amd/build_ab/$NAME/lib
echo "built $NAME ($OBJ.o with $FLAGS) into convolutional-codes_amd/build_ab/$NAME/lib"
