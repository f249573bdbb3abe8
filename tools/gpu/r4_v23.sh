#!/bin/bash
# Round 4: kernel-level anatomy of the final default (graphed fp32 plain
# K-FAC step vs graphed SGD step, eager factor step) and MFMA counters of the
# plain step's kernels (one host thread, 5-counter pass).
set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=gpurun_out/r4g2; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/p7 -o p7 -- python3 bench.py --steps 40 --warmup 10 --secondary-bf16 0 > $O/bench_prof.json 2> $O/prof.err || exit 1
T=$(ls /tmp/p7/*kernel_trace.csv /tmp/p7/*/*kernel_trace.csv 2>/dev/null | head -1)
python3 tools/step_kernel_diff.py $T > $O/step_kernel_diff_fp32_final.txt 2>&1 || exit 1
head -50 $O/step_kernel_diff_fp32_final.txt
export KFAC_EIGH_THREADS=0
(cd /tmp && timeout -s KILL 180 rocprofv3 --output-format csv -d /tmp/pm_busy -o pm --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -- python3 $R/bench.py --steps 12 --warmup 3 --secondary-bf16 0 --baseline 0 > /tmp/pm_busy.log 2>&1)
echo "pmc rc=$?"
python3 tools/pmc_summary.py /tmp pm $O/pmc_step_final busy > $O/pmc_summary.json 2> $O/pmc_summary.err || true
head -30 $O/pmc_step_final.md 2>/dev/null
du -sh gpurun_out
