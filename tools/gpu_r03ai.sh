#!/bin/bash
# transform phase at a raised wave priority: interleaved P-run A/B
cd "$GRAFT_REPO_ROOT" || exit 1
AB="default tools/_ab/prio1.so tools/_ab/prio3.so" TAG=r03ai ROUNDS=3 PYTEST=0 tools/gpu_ab.sh
