#!/bin/bash
# Round 3: two-stage eigensolver (v2 bulge chasing, rocBLAS strided stage-1 / BT1); graph-replay fix; default bench.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r3u; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_twostage_gpu.py > $O/ts_pytest.log 2>&1; rc=$?; tail -15 $O/ts_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/twostage_probe.py > $O/ts_probe.jsonl 2> $O/ts_probe.err || { echo "probe rc=$?"; tail -5 $O/ts_probe.err; exit 1; }
cat $O/ts_probe.jsonl
timeout -k 10 300 python -u tools/twostage_probe.py --sizes 4608,2304 --batch 3 > $O/ts_probe_b3.jsonl 2> $O/ts_probe_b3.err || { echo "probe rc=$?"; tail -5 $O/ts_probe_b3.err; exit 1; }
cat $O/ts_probe_b3.jsonl
timeout -k 10 200 python -u tools/graph_nan_probe.py --steps 10 > $O/gprobe_bf16.jsonl 2> $O/gprobe_bf16.err || { echo "gprobe rc=$?"; tail -5 $O/gprobe_bf16.err; exit 1; }
python -c "
import json
for l in open('$O/gprobe_bf16.jsonl'):
    d=json.loads(l); print(d['step'], d['kind'], d['how'], 'pbuf', d['pbuf']['maxrel'], 'param', d['param']['maxrel'])"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_graphs_refresh_gpu.py tests/test_graphs.py > $O/g_pytest.log 2>&1; rc=$?; tail -6 $O/g_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
export KFAC_REFERENCE_PATH="$R/_refbench"
timeout -k 10 600 python -u bench.py --impl reference --no-channels-last --dtype fp32 --secondary-bf16 0 --graphs 0 > $O/ref_fp32.json 2> $O/ref_fp32.err || { tail -5 $O/ref_fp32.err; exit 1; }
cat $O/ref_fp32.json
