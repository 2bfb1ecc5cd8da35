#!/bin/bash
# Build libtlsgpu.so of a git revision (same ABI as the tree: A/B of kernel changes between
# commits) into tools/ab/<name>/, from a temporary worktree.  CPU box (hipcc cross-compiles).
#   bash tools/build_rev.sh <name> <rev>
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
name=${1:?name}; rev=${2:?rev}
wt=$(mktemp -d /tmp/tg_rev_XXXX)
git -C "$R" worktree add -q --detach "$wt" "$rev"
python "$wt/tlslite_amd/build.py" --force --out "$R/tools/ab/$name" > /dev/null
git -C "$R" worktree remove --force "$wt"
ls -la "$R/tools/ab/$name/libtlsgpu.so"
