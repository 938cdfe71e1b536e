#!/bin/bash
# The GPU suite + interleaved P-run A/B of the in-tree library against one variant ($1), plain then VBS.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
AB="default $1" TAG=${TAG:-pair} ROUNDS=${ROUNDS:-3} PYTEST=${PYTEST:-1} bash tools/gpu_ab.sh || exit $?
SO_AB_VBS=1 AB="default $1" TAG=${TAG:-pair}_vbs ROUNDS=2 PYTEST=0 bash tools/gpu_ab.sh
