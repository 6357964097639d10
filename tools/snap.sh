#!/bin/bash
# Freeze the committed tree plus its built libraries under build/snap, so a GPU run can
# use it while the working tree is being edited.  Usage: tools/snap.sh [REV]
set -e
REV=${1:-HEAD}
rm -rf build/snap && mkdir -p build/snap
git archive "$REV" | tar -x -C build/snap
make -s -C build/snap -j8 all experimental > build/snap/make.log 2>&1
echo "build/snap = $(git rev-parse --short $REV)"
