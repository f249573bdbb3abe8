#!/bin/bash
# Round 3: native D&C tridiagonal solver + default eigensolver tiers on the
# GPU, then the serialized graph-fault locator (last: it may fault)
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r3f; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_tridiag.py > $O/tridiag.log 2>&1; rc=$?; tail -15 $O/tridiag.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_eigh_native_gpu.py > $O/eigh.log 2>&1; rc=$?; tail -12 $O/eigh.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/r3_fault.sh
