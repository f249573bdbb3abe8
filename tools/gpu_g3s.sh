#!/bin/bash
# gemm3s tile-order sweep (XCD chunk CH x grouped rows GM), 128x128 / 2 stages
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
O=$R/gpurun_out/g3s_chgm.jsonl
: > $O
for set in neox resnet; do
  for ch in 2 4 8; do for gm in 4 8 16; do
    echo -n "{\"ch\": $ch, \"gm\": $gm, \"r\": " >> $O
    timeout -k 5 120 $R/benchbin/g3s_ch${ch}_gm${gm} $set 0 1 1 >> $O; rc=$?; echo "}" >> $O
    [ $rc -eq 0 ] || { echo "FAILED ch$ch gm$gm rc=$rc"; exit 1; }
  done; done
done
python3 -c "
import json
for l in open('$O'):
    l=l.strip()
    if not l or l=='}': continue
" 
grep -o '"ch": [0-9]*, "gm": [0-9]*, "r": {"set": "[a-z]*"[^}]*"ms": [0-9.]*' $O
