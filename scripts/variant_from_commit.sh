#!/bin/bash
# Build lib/variants/<name>/libgsr_hip.so from the kernel sources of an earlier commit (a
# before / after A/B through scripts/ab.sh).  usage: scripts/variant_from_commit.sh NAME COMMIT
set -eu
NAME=$1; COMMIT=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
git -C "$ROOT" archive "$COMMIT" 3d_gaussian_splatting_amd/csrc include | tar -x -C "$TMP"
cd "$ROOT"
python3 -c "
import importlib, sys
sys.path.insert(0, '.')
b = importlib.import_module('3d_gaussian_splatting_amd._build')
print(b.build_variant('$NAME', [], csrc='$TMP/3d_gaussian_splatting_amd/csrc'))
"
rm -rf "$TMP"
