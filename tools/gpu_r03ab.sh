#!/bin/bash
# integer first pass of the 8-point sub-block transforms: GPU suite, VBS A/B against HEAD's build
cd "$GRAFT_REPO_ROOT" || exit 1
SO_AB_VBS=1 AB="default tools/_ab/head.so" TAG=${TAG:-r03ab} ROUNDS=3 tools/gpu_ab.sh
