#!/bin/bash
# Build libsrbd_qp.so from the sources of a git commit into build/variants/NAME
# (A/B against the working tree with scripts/dev/ab_variants.py).
set -e
REV=$1; NAME=$2
cd "$(dirname "$0")/../.."
ROOT=$(pwd)
TMP=$(mktemp -d)
git archive "$REV" srbd-nmpc-solver_amd/csrc include | tar -x -C "$TMP"
mkdir -p build/variants/$NAME
cd "$TMP"
for f in srbd-nmpc-solver_amd/csrc/*.hip; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-value -Iinclude -c "$f" -o "$ROOT/build/variants/$NAME/$(basename "$f" .hip).o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/build/variants/$NAME/libsrbd_qp.so" "$ROOT"/build/variants/$NAME/*.o
rm -rf "$TMP"
echo "built build/variants/$NAME from $REV"
