#!/bin/bash
# Build the "old" arm of tools/ab_pkg.py: a git worktree of COMMIT (default HEAD), built on the CPU
# here (hipcc cross-compiles gfx950), copied into ab_old/ (git-ignored) so it travels to the GPU box
# with the working tree.  Usage: tools/make_ab_old.sh [commit]
set -eu
cd "$(dirname "$0")/.."
COMMIT=${1:-HEAD}
WT=/tmp/po2q_ab_old_tree
git worktree remove --force "$WT" 2>/dev/null || true
git worktree add --detach "$WT" "$COMMIT" > /dev/null
(cd "$WT" && python -c "import __graft_entry__ as g; g.build()" > /tmp/po2q_ab_old_build.log 2>&1)
rm -rf ab_old
mkdir -p ab_old/po2_quantization_amd/lib ab_old/oracle ab_old/tools
cp -r "$WT"/po2_quantization_amd/*.py "$WT"/po2_quantization_amd/models "$WT"/po2_quantization_amd/utils \
    ab_old/po2_quantization_amd/
cp "$WT"/po2_quantization_amd/lib/*.so ab_old/po2_quantization_amd/lib/
cp "$WT"/bench.py ab_old/
cp -r "$WT"/oracle/*.py "$WT"/oracle/_build ab_old/oracle/
cp "$WT"/tools/*.py ab_old/tools/
git worktree remove --force "$WT"
echo "ab_old/ = $(git rev-parse --short "$COMMIT")"
