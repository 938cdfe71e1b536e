#!/bin/bash
# survivors past the cap in list windows: GPU suite, interleaved A/B on the bench content and on low texture
cd "$GRAFT_REPO_ROOT" || exit 1
AB="default tools/_ab/chunk384.so tools/_ab/head.so" TAG=r03ak ROUNDS=3 tools/gpu_ab.sh || exit $?
SO_AB_CONTENT=lowtex AB="default tools/_ab/head.so" TAG=r03ak_lowtex ROUNDS=2 PYTEST=0 tools/gpu_ab.sh
