#!/bin/bash
# Round 3 re-entry: full GPU suite, default bench (fp32 headline, graphs on),
# reference fp32 on the same harness.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r3r; mkdir -p $O
export KFAC_REFERENCE_PATH="$R/_refbench"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -6 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 600 python -u bench.py --impl reference --no-channels-last --dtype fp32 --secondary-bf16 0 --graphs 0 > $O/ref_fp32.json 2> $O/ref_fp32.err || { tail -5 $O/ref_fp32.err; exit 1; }
cat $O/ref_fp32.json
