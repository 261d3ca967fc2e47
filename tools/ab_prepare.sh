#!/usr/bin/env bash
# Prepare a same-box A/B baseline: a git worktree of REV under build/ab_base with its own native build.
# Then on the GPU box: (cd build/ab_base && python bench.py ...) vs python bench.py ...
set -e
REV=${1:-HEAD}
here=$(cd "$(dirname "$0")/.." && pwd)
cd "$here"
git worktree remove --force build/ab_base 2>/dev/null || rm -rf build/ab_base
git worktree add -f build/ab_base "$REV" -q
(cd build/ab_base && python tools/build_native.py > /dev/null)
echo "baseline $REV ready in build/ab_base"
