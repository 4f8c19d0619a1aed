#!/bin/bash
# Regenerates tools/patches/lab.patch after a product change: three-way
# merges the lab's changes (the committed patch over the committed sources)
# onto the working-tree sources, then diffs them. Conflicts are reported and
# left for a hand fix in $W/lab (re-run with FINISH=1 to only re-diff).
cd "$(dirname "$0")/.." || exit 1
W=${W:-/tmp/lab_regen}
FILES="zero-packet_amd/csrc/zp_parse.hip zero-packet_amd/csrc/zp_stream.h zero-packet_amd/csrc/zp_build.hip zero-packet_amd/csrc/zp_ctx.hip"
if [ -z "$FINISH" ]; then
  rm -rf $W && mkdir -p $W/base $W/other $W/lab
  git archive HEAD zero-packet_amd/csrc include | tar -x -C $W/base
  git archive HEAD zero-packet_amd/csrc include | tar -x -C $W/other
  git show HEAD:tools/patches/lab.patch | patch -s -p1 -d $W/other || exit 1
  rc=0
  for f in $FILES; do
    mkdir -p $W/lab/$(dirname $f)
    git merge-file -p $f $W/base/$f $W/other/$f > $W/lab/$f || { echo "conflict: $W/lab/$f"; rc=1; }
  done
  [ $rc -ne 0 ] && exit 1
fi
{ sed -n '1,/^--- a\//p' tools/patches/lab.patch | sed '$d'
  for f in $FILES; do diff -u --label a/$f --label b/$f $f $W/lab/$f; done; } > $W/lab.patch
cp $W/lab.patch tools/patches/lab.patch && echo "tools/patches/lab.patch regenerated"
