#!/bin/bash
# Run a command inside build/snap (tools/snap.sh) on the GPU box, with gpurun_out/ and the
# round-2 tree (build/ab_r2) shared with the repository root.  Usage: tools/gpu_snap_run.sh CMD...
set -e
ROOTDIR=$(pwd)
mkdir -p gpurun_out
cd build/snap
ln -sfn "$ROOTDIR/gpurun_out" gpurun_out
mkdir -p build && ln -sfn "$ROOTDIR/build/ab_r2" build/ab_r2
exec bash -c "$*"
