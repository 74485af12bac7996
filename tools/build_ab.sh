#!/bin/bash
# Build A/B variants of libgpfit.so that differ only in predict.hip: _ab/lib_<tag>.so
# usage: tools/build_ab.sh tag [extra hipcc flags...]   (PREDICT_SRC overrides the source)
set -e
R=/root/repo; tag=$1; shift
src=${PREDICT_SRC:-$R/gladsgp_amd/csrc/predict.hip}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function -I$R/gladsgp_amd/csrc "$@" -c $src -o /tmp/predict_$tag.o
objs=$(ls $R/gladsgp_amd/_obj/*.o | grep -v predict.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/_ab/lib_$tag.so $objs /tmp/predict_$tag.o -ldl
echo built _ab/lib_$tag.so
