#!/bin/bash
# Build the library of another git revision as a measurement variant
# deppy_amd/libdeppy_hip_<tag>.so (loaded by DEPPY_VARIANT_LIB; A/B runs
# only, never the product path).  usage: scripts/mkvariant.sh <rev> <tag> [extra hipcc flags]
set -e
REV=$1; TAG=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
WT=/tmp/deppy_variant_$TAG
rm -rf $WT
git -C $ROOT worktree prune
git -C $ROOT worktree add -f --detach $WT $REV > /dev/null
(cd $WT && python3 -c "from deppy_amd import build as b; b.build(extra=$(python3 -c "import sys,json; print(json.dumps(sys.argv[1:]) if sys.argv[1:] else 'None')" "$@"))")
cp $WT/deppy_amd/libdeppy_hip.so $ROOT/deppy_amd/libdeppy_hip_$TAG.so
git -C $ROOT worktree remove --force $WT
echo "built deppy_amd/libdeppy_hip_$TAG.so from $REV"
