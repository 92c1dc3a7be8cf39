#!/bin/bash
# Build libbos.so of the working tree with extra compile flags (e.g. -DBOS_MF_MIXB=0) into
# gpurun_exp/libbos_<name>.so for A/B runs (tools/gn_ab.py), from a temporary copy of the package.
# Usage: tools/build_flag_variant.sh name "FLAGS"
set -e
cd "$(dirname "$0")/.."
name=$1; flags=$2
tmp=/tmp/bos_var_$name
rm -rf $tmp; mkdir -p $tmp
cp -r prb-project-bearing-only-slam_amd $tmp/
rm -rf $tmp/prb-project-bearing-only-slam_amd/build $tmp/prb-project-bearing-only-slam_amd/lib
cp -r include oracle $tmp/ 2>/dev/null || true
sed -i "s|^HIPFLAGS ?= \(.*\)|HIPFLAGS ?= \1 $flags|" $tmp/prb-project-bearing-only-slam_amd/Makefile
make -C $tmp/prb-project-bearing-only-slam_amd -j8 lib/libbos.so > $tmp.log 2>&1
mkdir -p gpurun_exp
cp $tmp/prb-project-bearing-only-slam_amd/lib/libbos.so gpurun_exp/libbos_$name.so
rm -rf $tmp
echo built gpurun_exp/libbos_$name.so with $flags
