#!/bin/bash
# Round 4: MIOpen find over the bench's fp32 channels_last convolutions (the
# shipped find-db only holds bf16 entries, so fp32 ran on MIOpen's
# heuristics), merged with the shipped db; fp32 bench A/B old vs new db;
# PMC crash bisection at n = 4608.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=gpurun_out/r4q; mkdir -p $O/tune
for i in 1 2 3; do
  d=/tmp/tune_$i; mkdir -p $d; cp miopen_db/* $d/
  MIOPEN_USER_DB_PATH=$d timeout -k 10 300 python3 bench.py --steps 5 --warmup 3 --cudnn-benchmark 1 --no-kfac --graphs 0 --secondary-bf16 0 --baseline 0 > $O/tune/run_$i.json 2> $O/tune/run_$i.err || exit 1
  cp $d/*.ufdb.txt $O/tune/ufdb_$i.txt
done
mkdir -p /tmp/newdb && cp miopen_db/* /tmp/newdb/
F=$(basename $(ls miopen_db/*.ufdb.txt))
python3 tools/merge_miopen_fdb.py /tmp/newdb/$F miopen_db/$F $O/tune/ufdb_*.txt || exit 1
cp /tmp/newdb/$F $O/tune/merged.ufdb.txt
for i in 1 2; do
  MIOPEN_USER_DB_PATH=$R/miopen_db timeout -k 10 400 python3 bench.py --steps 100 --warmup 10 --secondary-bf16 0 > $O/bench_olddb_$i.json 2> $O/bench.err || exit 1
  MIOPEN_USER_DB_PATH=/tmp/newdb timeout -k 10 400 python3 bench.py --steps 100 --warmup 10 --secondary-bf16 0 > $O/bench_newdb_$i.json 2>> $O/bench.err || exit 1
done
mkdir -p $O/pmcb
(cd /tmp && timeout -s KILL 120 rocprofv3 --output-format csv -d /tmp/pc1 -o pc --pmc SQ_WAVES -- python3 $R/tools/pmc_bisect.py eigh --n 4608 > /tmp/pc1.log 2>&1); rc=$?
echo "eigh4608 SQ_WAVES rc=$rc" >> $O/pmcb/summary.txt
[ $rc -ne 0 ] && { grep -v "^W2026" /tmp/pc1.log | tail -80 > $O/pmcb/fail_eigh4608.txt; exit 0; }
(cd /tmp && timeout -s KILL 120 rocprofv3 --output-format csv -d /tmp/pc2 -o pc --pmc SQ_WAVES -- python3 $R/tools/eigh_probe.py --sizes 4608 --count 1 --reps 1 --no-acc > /tmp/pc2.log 2>&1); rc=$?
echo "eigh_probe4608 SQ_WAVES rc=$rc" >> $O/pmcb/summary.txt
[ $rc -ne 0 ] && { grep -v "^W2026" /tmp/pc2.log | tail -80 > $O/pmcb/fail_probe4608.txt; exit 0; }
(cd /tmp && timeout -s KILL 120 rocprofv3 --output-format csv -d /tmp/pc3 -o pc --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -- python3 $R/tools/pmc_bisect.py eigh --n 4608 > /tmp/pc3.log 2>&1); rc=$?
echo "eigh4608 5 counters rc=$rc" >> $O/pmcb/summary.txt
[ $rc -ne 0 ] && { grep -v "^W2026" /tmp/pc3.log | tail -80 > $O/pmcb/fail_eigh4608_5c.txt; exit 0; }
du -sh gpurun_out
