#!/bin/bash
# Builds an A/B variant of the engine with extra compile-time definitions, e.g.
#   bash tools/build_variant.sh ku4 -DKECCAK_UNROLL=4
# -> janus_amd/variants/libjanus_prio3_ku4.so (select with JANUS_PRIO3_LIB=...).
#   ONLY="prio3_prep_pair" bash tools/build_variant.sh ...: only that source recompiled.
set -e
TAG=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/janus_amd/variants/$TAG
mkdir -p $OUT
SRCS=$(cd $R/janus_amd/csrc && ls *.hip | sed "s/\.hip$//")
# ONLY="a b": recompile only those sources with the definitions, the rest from the in-tree build
for f in $SRCS; do
  if [ -n "$ONLY" ] && ! [[ " $ONLY " == *" $f "* ]]; then
    cp $R/janus_amd/build/$f.o $OUT/$f.o
    continue
  fi
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function "$@" \
    -c -o $OUT/$f.o $R/janus_amd/csrc/$f.hip &
done
wait
/opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared -o $R/janus_amd/variants/libjanus_prio3_$TAG.so $(for f in $SRCS; do echo $OUT/$f.o; done)
rm -rf $OUT
echo built janus_amd/variants/libjanus_prio3_$TAG.so
