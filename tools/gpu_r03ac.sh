#!/bin/bash
# tile phase stamps of the VBS persistent run and of the plain one (4K)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03ac; mkdir -p $O
SO_LIB_PATH=tools/_ab/stamps.so timeout -k 10 300 python -u tools/run_stamps.py --heights 2160 --vbs > $O/stamps_vbs.log 2>&1
rc=$?; echo "vbs rc=$rc"; grep "^H=" $O/stamps_vbs.log | cut -c1-2000; [ $rc -ne 0 ] && exit $rc
SO_LIB_PATH=tools/_ab/stamps.so timeout -k 10 300 python -u tools/run_stamps.py --heights 2160 > $O/stamps.log 2>&1
rc=$?; echo "plain rc=$rc"; grep "^H=" $O/stamps.log | cut -c1-2000; exit $rc
