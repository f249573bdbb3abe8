#!/bin/bash
# gemm3s tile / pipeline-depth variants (correctness-checked) on the NeoX and ResNet sets
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
O=$R/gpurun_out/g3s_stages.jsonl
: > $O
for set in neox resnet; do
  for v in t3_s2 t3_s3 t1_s3 t1_s2 t2_s2; do
    for cfg in "0 1 1" "0 0 0"; do
      echo -n "{\"v\": \"$v\", \"r\": " >> $O
      timeout -k 5 120 $R/benchbin/gemm3s_bench_$v $set $cfg >> $O; rc=$?; echo "}" >> $O
      [ $rc -eq 0 ] || { echo "FAILED $v $set $cfg rc=$rc"; cat $O; exit 1; }
    done
  done
done
cat $O
