#!/bin/bash
# Round 3: graph-replay regression tests (sequential twin) + bf16 / fp32 bench on the current tree
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r3gv; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_graphs_refresh_gpu.py tests/test_graphs.py > $O/pytest.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error|passed|failed" $O/pytest.log | tail -12; [ $rc -eq 0 ] || exit $rc
KFAC_BENCH_NANSTEP=1 timeout -k 10 300 python3 -u bench.py --bf16 --steps 100 --warmup 10 --baseline 0 > $O/bench_bf16.json 2> $O/bench_bf16.err || { echo "bf16 rc=$?"; tail -5 $O/bench_bf16.err; exit 1; }
grep "\[nan\]" $O/bench_bf16.err | head -3
python3 -c "import json;d=json.load(open('$O/bench_bf16.json'));print('bf16', d['value'],d['ms_per_step'],d['kind_ms'],d['params_finite'])"
timeout -k 10 400 python3 -u bench.py --steps 100 --warmup 10 > $O/bench_fp32.json 2> $O/bench_fp32.err || { echo "fp32 rc=$?"; tail -5 $O/bench_fp32.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_fp32.json'));print('fp32', d['value'],d['ms_per_step'],d['kind_ms'],d.get('sgd_ms_per_step'),d['params_finite'], 'bf16', d.get('bf16',{}).get('value'), d.get('bf16',{}).get('params_finite'))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/$O/rtrace -o rtrace -- python3 $R/tools/refresh_probe.py --mode-list default_warm --reps 2 --no-acc > $R/$O/rtrace.log 2>&1 || { echo "rtrace rc=$?"; tail -5 $R/$O/rtrace.log; exit 1; }
cd $R && tail -2 $O/rtrace.log && python3 tools/refresh_trace_summary.py $(find $O/rtrace -name "*kernel_trace.csv" | head -1) > $O/rtrace_summary.txt && head -60 $O/rtrace_summary.txt && rm -rf $O/rtrace
