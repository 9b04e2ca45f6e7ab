#!/bin/bash
# Build an A/B variant of libhgx.so from a modified copy of one engine source (in this container):
#   bash tools/build_variant.sh <name> <file.hip> [<file2.hip> ...]
# The files replace the same-named sources of hypergraphdb_amd/csrc for this build only; the result is
# tools/native/build/libhgx_<name>.so, loaded by HGX_LIB_VARIANT=<name> (hypergraphdb_amd/_lib.py).
# With no files given it builds the current sources as an A/B build (environment knobs on).
set -eu
NAME=$1
shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d /tmp/hgxvar.XXXX)
W=$T/pkg/csrc   # hgx_internal.h includes ../../include/hgx.h
mkdir -p "$W"
ln -s "$ROOT/include" "$T/include"
cp "$ROOT"/hypergraphdb_amd/csrc/*.hip "$ROOT"/hypergraphdb_amd/csrc/*.h "$W"/
for f in "$@"; do cp "$f" "$W/$(basename "$f")"; done
mkdir -p "$ROOT/tools/native/build"
cd "$W"
# A/B builds read the engine's A/B knobs from the environment (hgx::ab_env, -DHGX_AB_KNOBS); the product
# library does not
PIDS=()
for f in hgx_graph hgx_bfs hgx_query hgx_seq hgx_part hgx_file; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -DHGX_AB_KNOBS \
        -I"$ROOT/include" -c $f.hip -o $f.o &
    PIDS+=($!)
done
for p in "${PIDS[@]}"; do
    wait "$p" || { echo "build_variant: a compile failed" >&2; rm -rf "$T"; exit 1; }
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,--no-undefined -o "$ROOT/tools/native/build/libhgx_$NAME.so" \
    hgx_*.o -L/opt/rocm/lib -lrccl -lamdhip64 -Wl,-rpath,/opt/rocm/lib
rm -rf "$T"
echo "built tools/native/build/libhgx_$NAME.so"
