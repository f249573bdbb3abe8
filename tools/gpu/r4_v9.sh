#!/bin/bash
# Round 4: GPU tests touched this round (graph interleave incl. bf16 GEMM
# mode, eigensolver); symv wave budgets above the chip default (mix);
# solver table for the cost model; default bench (fp32 + bf16 secondary,
# both graphed); eigensolver PMC passes from one host thread (last).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4o; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_graphs_refresh_gpu.py tests/test_eigh_native_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
E="python -u tools/eigh_probe.py --mix resnet50 --no-acc"
for w in 0 6144 12288; do
  KFAC_SYTRD_WAVES=$w timeout -k 10 200 $E > $O/mix_w$w.jsonl 2>> $O/eig.err || exit 1
done
timeout -k 10 400 python -u tools/solver_table.py > $O/solver_table.json 2> $O/solver_table.err || exit 1
timeout -k 10 500 python -u bench.py --steps 100 --warmup 10 > $O/bench_default.json 2> $O/bench_default.err || exit 1
bash tools/gpu/r4_pmc.sh > $O/pmc.log 2>&1
du -sh gpurun_out
