#!/bin/bash
# Profiling aid: build an engine variant with extra -D flags into build/alt/lib_<name>.so
# (only the fast-kernel objects are rebuilt; A/B them with FQ_ENGINE_LIB, tools/ab.sh).
#   tools/ab_build.sh <name> -DFQ_PREFETCH=0 ...
set -eu
cd "$(dirname "$0")/.."
name=$1; shift
out=build/alt/$name; mkdir -p $out
HIPFLAGS="-std=c++17 -O3 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result"
/opt/rocm/bin/hipcc $HIPFLAGS "$@" -c fqtool_amd/csrc/${PE_FAST_SRC:-pe_fast.hip} -o $out/pe_fast.o &
/opt/rocm/bin/hipcc $HIPFLAGS "$@" -c fqtool_amd/csrc/pe_fast_long.hip -o $out/pe_fast_long.o &
wait
objs=""
for o in engine pe_kernel synth dup kmer text raw; do objs="$objs build/obj/$o.o"; done
/opt/rocm/bin/hipcc $HIPFLAGS -shared -o build/alt/lib_$name.so $objs $out/pe_fast.o $out/pe_fast_long.o
echo built build/alt/lib_$name.so
