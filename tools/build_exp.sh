#!/bin/bash
# Experiment builds of libatgpu.so (exp/libatgpu_<name>.so, NOT byte-exact):
# the product objects with one source recompiled under extra -D flags.
#   tools/build_exp.sh <name> "<source.hip> [more.hip ...]" <flags...>
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; src=$2; shift 2
C=$R/python-audio-tools_amd/csrc
make -s -C "$C" -j8 ../audiotools/libatgpu.so
mkdir -p "$C/obj_$name" "$R/exp"
cp -p "$C"/obj/*.o "$C/obj_$name/"
for f in $src; do rm -f "$C/obj_$name/${f%.hip}.o"; done
make -s -C "$C" OBJDIR="obj_$name" OUT="$R/exp/libatgpu_$name.so" EXTRA="-DATG_EXPERIMENT_BUILD $*" "$R/exp/libatgpu_$name.so"
