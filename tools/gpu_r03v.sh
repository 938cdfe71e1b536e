#!/bin/bash
# integer first pass of the transforms: GPU suite, then interleaved A/B against HEAD's build
cd "$GRAFT_REPO_ROOT" || exit 1
AB="default tools/_ab/base.so" TAG=r03v ROUNDS=3 tools/gpu_ab.sh
