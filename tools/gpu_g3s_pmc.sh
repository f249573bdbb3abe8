# PMC counters of the grouped pre-split GEMM (benchbin/g3s_t0, ResNet-50 tables)
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd /tmp && export TMPDIR=/tmp
O=$R/gpurun_out/g3s_pmc; mkdir -p $O
for cfg in "0 1 1 g" "0 0 0 a"; do
  tag=$(echo $cfg | tr ' ' '_')
  timeout -s KILL 60 rocprofv3 --kernel-trace --output-format csv -d $O/p1_$tag -o p1 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -- $R/benchbin/g3s_t0 resnet $cfg > $O/p1_$tag.log 2>&1 || { echo "pass1 $tag failed"; tail -5 $O/p1_$tag.log; exit 1; }
  timeout -s KILL 60 rocprofv3 --kernel-trace --output-format csv -d $O/p2_$tag -o p2 --pmc SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE -- $R/benchbin/g3s_t0 resnet $cfg > $O/p2_$tag.log 2>&1 || { echo "pass2 $tag failed"; tail -5 $O/p2_$tag.log; exit 1; }
done
cd $R; python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob('gpurun_out/g3s_pmc/*/**/*counter_collection.csv', recursive=True)):
    agg = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f)):
        if 'gemm3s_kernel' not in r['Kernel_Name']: continue
        agg[r['Counter_Name']] += float(r['Counter_Value'])
        n[r['Counter_Name']] += 1
    print(f.split('/')[2], {k: round(v / max(n[k], 1), 1) for k, v in sorted(agg.items())})
PY
find gpurun_out/g3s_pmc -name "*.csv" -size +5M -delete
