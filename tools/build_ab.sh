#!/bin/bash
# Build the committed HEAD's library as lib/libgsplat_hip_old.so beside the working tree's
# lib/libgsplat_hip.so (for `tools/gpu_run.sh ab` on the GPU box).  Run from the repo root, with the
# change under test uncommitted (with no local changes there is nothing to compare, and a
# `git stash pop` would restore an unrelated older stash).
set -e
cd "$(git rev-parse --show-toplevel)"
if git diff --quiet && git diff --cached --quiet; then
    echo "build_ab: no local changes to compare against HEAD" >&2
    exit 1
fi
M="make -s -j8 -C openglgaussiansplattingrenderer_amd ARCH=gfx950"
git stash -q
$M
cp openglgaussiansplattingrenderer_amd/lib/libgsplat_hip.so /tmp/libgsplat_hip_old.so
git stash pop -q
$M
cp /tmp/libgsplat_hip_old.so openglgaussiansplattingrenderer_amd/lib/libgsplat_hip_old.so
