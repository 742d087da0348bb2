#!/usr/bin/env bash
# Build libpekf.so of a given commit into ab/<name>.so (for same-box A/B timing with PEKF_LIB=...).
# usage: scripts/ab_build.sh <commit> <name>
set -eu
root=$(cd "$(dirname "$0")/.." && pwd)
wt=/tmp/pekf_ab_$2
rm -rf "$wt"
git -C "$root" worktree add -f --detach "$wt" "$1" >/dev/null
make -s -j8 -C "$wt/poseestimationkf_amd/csrc" ../libpekf.so 2>&1 | grep -v hip-link || true
mkdir -p "$root/ab"
cp "$wt/poseestimationkf_amd/libpekf.so" "$root/ab/$2.so"
git -C "$root" worktree remove --force "$wt"
echo "built ab/$2.so from $(git -C "$root" rev-parse --short "$1")"
