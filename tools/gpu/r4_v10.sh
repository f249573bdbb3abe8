#!/bin/bash
# Round 4: per-kernel diff of the bench's fp32 steps (graphed plain K-FAC vs
# graphed SGD, eager factor-update vs plain) from one rocprofv3 kernel trace;
# host profile of the eager factor-update step.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4p; mkdir -p $O
E="python -u tools/eigh_probe.py --mix resnet50 --no-acc"
for sp in 4000,1000 4000 1000 2000,500 0; do
  KFAC_SYTRD_SPLIT=$sp timeout -k 10 200 $E > $O/mix_split$sp.jsonl 2>> $O/eig.err || exit 1
done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/p6 -o p6 -- python3 bench.py --steps 40 --warmup 10 --secondary-bf16 0 > $O/bench_prof.json 2> $O/prof.err || exit 1
T=$(ls /tmp/p6/*kernel_trace.csv /tmp/p6/*/*kernel_trace.csv 2>/dev/null | head -1)
python3 tools/step_kernel_diff.py $T > $O/step_kernel_diff_fp32.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/host_profile.py --kind factor --steps 5 > $O/host_factor_fp32.txt 2> $O/host.err || exit 1

# PMC crash bisection (one counter; stops at the first stage that fails)
R=$PWD
mkdir -p $O/pmcb
for st in matmul jacobi dc sytrd applyq eigh; do
  (cd /tmp && timeout -s KILL 90 rocprofv3 --output-format csv -d /tmp/pb_$st -o pb --pmc SQ_WAVES -- python3 $R/tools/pmc_bisect.py $st --n 512 > /tmp/pb_$st.log 2>&1)
  rc=$?
  echo "$st rc=$rc" >> $O/pmcb/summary.txt
  if [ $rc -ne 0 ]; then grep -v "^W2026" /tmp/pb_$st.log | tail -60 > $O/pmcb/fail_$st.txt; break; fi
done

du -sh gpurun_out
