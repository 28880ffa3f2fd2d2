#!/bin/bash
# Probe build (not product): the library as of git revision REV, as abl/libtkv_NAME.so, for
# in-process A/B runs against the working tree's build. Usage: tools/build_at.sh REV NAME [-DFLAG ...]
# (REV "WT": the working tree's sources as they are now; REV a directory: its tinykvpp_amd/csrc and include)
set -e
cd "$(dirname "$0")/.."
REV=$1; NAME=$2; shift 2
T=$(mktemp -d)
if [ "$REV" = WT ] || [ -d "$REV" ]; then
  S=.; [ -d "$REV" ] && S=$REV
  mkdir -p "$T/tinykvpp_amd" && cp -r $S/tinykvpp_amd/csrc "$T/tinykvpp_amd/" && cp -r $S/include "$T/" && rm -rf "$T/tinykvpp_amd/csrc/build"
else
  git archive "$REV" tinykvpp_amd/csrc include | tar -x -C "$T"
fi
H=$T/tinykvpp_amd/csrc
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$T/include -I$H"
mkdir -p abl
for f in $H/*.hip; do s=$(basename $f); /opt/rocm/bin/hipcc $F "$@" -c $H/$s -o $T/${s%.*}.o & done
for s in tkv_crc32_host.cpp tkv_formats.cpp tkv_crc32_span.cpp; do /opt/rocm/bin/hipcc $F "$@" -x hip -c $H/$s -o $T/${s%.*}.o & done
wait
echo "extern \"C\" const char* tkv_build_id(void) { return \"rev-$REV\"; }" > $T/id.cpp
/opt/rocm/bin/hipcc -O2 -fPIC -c -x c++ $T/id.cpp -o $T/id.o
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o abl/libtkv_$NAME.so $T/*.o -lpthread
rm -rf "$T"
echo "abl/libtkv_$NAME.so"
