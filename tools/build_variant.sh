#!/bin/bash
# Build librrte_hip.so from git revision <rev> into <out.so> (A/B baselines for tools/ab_lib.sh).
# usage: tools/build_variant.sh <rev> <out.so>
set -euo pipefail
REV=${1:?rev}; OUT=${2:?out.so}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d /tmp/rrte_variant.XXXXXX)
git -C "$ROOT" archive "$REV" | tar -x -C "$TMP"
make -s -C "$TMP/rrte_amd/csrc" -j8 > /dev/null
mkdir -p "$(dirname "$OUT")"
cp "$TMP/rrte_amd/lib/librrte_hip.so" "$OUT"
rm -rf "$TMP"
echo "built $REV -> $OUT"
