#!/bin/bash
# Build libbos.so of a git revision (e.g. HEAD: the last commit, against the working tree's
# changes) into gpurun_exp/libbos_<name>.so for A/B runs (tools/gn_ab.py), from a temporary
# worktree. Usage: tools/build_rev_variant.sh name rev
set -e
cd "$(dirname "$0")/.."
name=$1; rev=${2:-HEAD}
wt=/tmp/bos_wt_$name
rm -rf $wt; git worktree prune
git worktree add -q --detach $wt $rev
make -C $wt/prb-project-bearing-only-slam_amd -j8 lib/libbos.so > /tmp/bos_wt_$name.log 2>&1
mkdir -p gpurun_exp
cp $wt/prb-project-bearing-only-slam_amd/lib/libbos.so gpurun_exp/libbos_$name.so
git worktree remove --force $wt
echo built gpurun_exp/libbos_$name.so from $(git rev-parse --short $rev)
