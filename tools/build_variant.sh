#!/bin/bash
# build librtamd.so at git revision $1 into raytracer-server_amd/lib/variants/$2.so (for A/B runs)
set -e
REV=$1; TAG=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
WT=/tmp/rt_wt_$TAG
rm -rf "$WT"; git -C "$ROOT" worktree prune
git -C "$ROOT" worktree add -f "$WT" "$REV" >/dev/null 2>&1
make -s -j8 -C "$WT/raytracer-server_amd" >/dev/null
mkdir -p "$ROOT/raytracer-server_amd/lib/variants"
cp "$WT/raytracer-server_amd/lib/librtamd.so" "$ROOT/raytracer-server_amd/lib/variants/$TAG.so"
git -C "$ROOT" worktree remove --force "$WT"
echo "built $TAG from $REV"
