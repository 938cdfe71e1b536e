#!/bin/bash
# SEA U refinement past the cap: GPU suite, interleaved A/B on the bench content and on low texture
cd "$GRAFT_REPO_ROOT" || exit 1
AB="default tools/_ab/norefine.so" TAG=r03aa ROUNDS=3 tools/gpu_ab.sh || exit $?
SO_AB_CONTENT=lowtex AB="default tools/_ab/norefine.so" TAG=r03aa_lowtex ROUNDS=2 PYTEST=0 tools/gpu_ab.sh
