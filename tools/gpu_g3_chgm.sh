# CH (tiles per XCD chunk) x GM (tile rows per column group) sweep of the
# grouped bf16x3 GEMM on the ResNet-50 shape set (tools/gemm3_bench.cpp,
# variants prebuilt into g3bin/ on the CPU host).
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"
out="$R/gpurun_out/g3_chgm.jsonl"
: > "$out"
for b in "$R"/g3bin/g3_*; do
  n=$(basename "$b")
  for rep in 1 2; do
    line=$(timeout -k 5 60 "$b") || exit $?
    echo "{\"variant\": \"$n\", \"rep\": $rep, \"r\": $line}" | tee -a "$out"
  done
done
