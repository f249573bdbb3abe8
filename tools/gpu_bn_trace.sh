set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out/prof_keep"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/bn_tr -o bn -- python3 "$R/bench.py" --no-kfac --steps 20 --warmup 5 > /dev/null 2>&1 || exit $?
f=$(find /tmp/bn_tr -name "*kernel_trace*.csv" | head -1)
python3 "$R/tools/kernel_breakdown.py" "$f" bn_ "$R/gpurun_out/prof_keep/bn_breakdown.txt"
head -5 "$f" | cut -c1-400 > "$R/gpurun_out/prof_keep/trace_head.txt"
