#!/bin/bash
# Probe build (not product): the product library with extra -D flags, as tools/ab/libtkv_NAME.so.
# Usage: tools/build_variant.sh NAME [-DFLAG ...]
set -e
cd "$(dirname "$0")/.."
N=$1; shift
H=tinykvpp_amd/csrc
T=$(mktemp -d)
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Iinclude -I$H"
/opt/rocm/bin/hipcc $F "$@" -c $H/tkv_crc32_kernels.hip -o $T/k.o
/opt/rocm/bin/hipcc $F "$@" -c $H/tkv_wal_device.hip -o $T/w.o
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o tools/ab/libtkv_$N.so $T/k.o $T/w.o $H/build/tkv_crc32_host.o $H/build/tkv_formats.o $H/build/tkv_crc32_span.o $H/build/tkv_wal_records.o $H/build/tkv_build_id.o -lpthread
rm -rf $T
