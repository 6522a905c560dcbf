#!/bin/bash
set -o pipefail
O=gpurun_out/r05n; mkdir -p $O
ICAP_LIB=tools/ab/_libs/libicap_echo.so timeout -k 10 300 python -u tools/ab/ln_echo_probe.py 2>&1 | grep -v amdgpu.ids > $O/echo.txt; rc=$?
cat $O/echo.txt; exit $rc
