#!/bin/bash
# Round 3: two-stage eigensolver v3 (coalesced bulge-chase loads, faster panel QR reductions); profile; bench
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r3y; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_twostage_gpu.py > $O/ts_pytest.log 2>&1; rc=$?; tail -3 $O/ts_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/twostage_probe.py > $O/ts_probe.jsonl 2> $O/ts_probe.err || { echo "probe rc=$?"; tail -5 $O/ts_probe.err; exit 1; }
cat $O/ts_probe.jsonl
timeout -k 10 300 python -u tools/twostage_probe.py --sizes 4608,2304 --batch 3 > $O/ts_probe_b3.jsonl 2> $O/ts_probe_b3.err || { echo "probe rc=$?"; tail -5 $O/ts_probe_b3.err; exit 1; }
cat $O/ts_probe_b3.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o ts -- python3 $R/tools/twostage_probe.py --sizes 4608 --batch 3 --reps 1 > $R/$O/prof.log 2>&1 || { echo "prof rc=$?"; tail -5 $R/$O/prof.log; exit 1; }
cd $R
timeout -k 10 600 python -u bench.py --secondary-bf16 0 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
