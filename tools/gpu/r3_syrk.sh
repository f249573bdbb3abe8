#!/bin/bash
# Round 3: factor SYRK timing on every ResNet-50 factor shape + PMC pass
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r3k; mkdir -p $O
timeout -k 10 240 python3 -u tools/syrk_probe.py --json $O/base.jsonl > $O/base.log 2>&1 || { echo "probe rc=$?"; tail -20 $O/base.log; exit 1; }
KFAC_SYRK_FP32=exact timeout -k 10 240 python3 -u tools/syrk_probe.py --json $O/exact.jsonl > $O/exact.log 2>&1 || { echo "exact rc=$?"; tail -20 $O/exact.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU --output-format csv -d $R/$O/pmc1 -o pmc1 -- python3 $R/tools/syrk_probe.py --reps 3 > $R/$O/pmc1.log 2>&1 || { echo "pmc1 rc=$?"; tail -5 $R/$O/pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $R/$O/pmc2 -o pmc2 -- python3 $R/tools/syrk_probe.py --reps 3 > $R/$O/pmc2.log 2>&1 || { echo "pmc2 rc=$?"; tail -5 $R/$O/pmc2.log; exit 1; }
cd $R; tail -3 $O/base.log; tail -1 $O/exact.log
timeout -k 10 300 python3 -u bench.py --bf16 --steps 100 --warmup 10 > $O/bench_bf16.json 2> $O/bench_bf16.err || { echo "bf16 bench rc=$?"; tail -5 $O/bench_bf16.err; exit 1; }
cat $O/bench_bf16.json
