# PMC counters of the grouped GEMM kernel (own pass per counter group; no traces).
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out/pmc"; cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > "$R/gpurun_out/pmc/counters_list.txt" 2>&1 || true
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_BUSY_CYCLES --kernel-trace --output-format csv -d /tmp/pmc1 -o g3 -- python3 "$R/tools/bench_gemm3.py" > "$R/gpurun_out/pmc/run1.txt" 2>&1 || exit $?
find /tmp/pmc1 -name "*counter_collection*.csv" -exec cp {} "$R/gpurun_out/pmc/pass1.csv" \;
timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU --kernel-trace --output-format csv -d /tmp/pmc2 -o g3 -- python3 "$R/tools/bench_gemm3.py" > "$R/gpurun_out/pmc/run2.txt" 2>&1 || exit $?
find /tmp/pmc2 -name "*counter_collection*.csv" -exec cp {} "$R/gpurun_out/pmc/pass2.csv" \;
ls -la "$R/gpurun_out/pmc"
