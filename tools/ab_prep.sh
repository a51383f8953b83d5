#!/bin/bash
# Build the committed HEAD's library into zig-bpe_amd/zbpe/ab/libzbpe_head.so (the A/B baseline of
# tools/exp_run.sh) from a temporary worktree, leaving the working tree alone.
set -e
cd "$(dirname "$0")/.."
W=/tmp/zbpe_head_wt
git worktree remove --force "$W" 2>/dev/null || true
git worktree add -q --detach "$W" HEAD
make -s -C "$W/zig-bpe_amd"
mkdir -p zig-bpe_amd/zbpe/ab
cp "$W/zig-bpe_amd/zbpe/libzbpe.so" zig-bpe_amd/zbpe/ab/libzbpe_head.so
git worktree remove --force "$W"
echo "ab baseline: $(git rev-parse --short HEAD)"
