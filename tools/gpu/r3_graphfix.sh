#!/bin/bash
# Round 3: graph-replay NaN root cause (AccumulateGrad nodes kept alive by the
# captured loss), regression tests, fp32 headline + reference fp32 baseline.
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r3a; mkdir -p $O
export KFAC_REFERENCE_PATH="$R/_refbench"
nan() { grep -o '\[nan\][^,]*' "$1" | head -1; grep -o '"params_finite": [a-z]*' "$1" | head -1; }
# 1. old behaviour (keep captured autograd graph): expect non-finite
KFAC_GRAPH_KEEP_AUTOGRAD=1 KFAC_BENCH_NANSTEP=1 timeout -k 10 240 python -u bench.py --bf16 --steps 30 --warmup 5 --baseline 0 --secondary-bf16 0 > $O/keep.log 2>&1 || { tail -5 $O/keep.log; exit 1; }
echo "keep-autograd: $(nan $O/keep.log)"
grep -c "AccumulateGrad node's stream" $O/keep.log
# 2. fix, three runs
for i in 1 2 3; do
KFAC_BENCH_NANSTEP=1 timeout -k 10 240 python -u bench.py --bf16 --steps 30 --warmup 5 --baseline 0 --secondary-bf16 0 > $O/fix$i.log 2>&1 || { tail -5 $O/fix$i.log; exit 1; }
echo "fix run $i: $(nan $O/fix$i.log) warn=$(grep -c "AccumulateGrad node's stream" $O/fix$i.log)"
done
# 3. regression tests
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_graphs_refresh_gpu.py tests/test_graphs.py > $O/pytest.log 2>&1; rc=$?; tail -12 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
# 4. headline bench (fp32 default, graphs, secondary bf16)
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
# 5. reference fp32 on the same harness
timeout -k 10 600 python -u bench.py --impl reference --no-channels-last --dtype fp32 --secondary-bf16 0 --graphs 0 > $O/ref_fp32.json 2> $O/ref_fp32.err || { tail -5 $O/ref_fp32.err; exit 1; }
cat $O/ref_fp32.json
