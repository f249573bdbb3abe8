#!/bin/bash
# gemm3s tile configs (tools/bin/g3s_t<TILE>[s<NSTAGE>], built with -DGEMM3S_TILE
# [-DGEMM3S_NSTAGE]) on
# the NeoX and ResNet-50 layer sets, the four operand layouts of the chain
# (t1/t3e: 0 1 1, t2: 1 1 1 with K = g, t4: 0 0 0).  One JSON line each.
set -o pipefail
for t in "$@"; do
  for set in resnet neox; do
    for cfg in "0 1 1 a" "1 1 1 g" "0 1 1 g" "0 0 0 a"; do
      # T2 (1 1 1 g) with its eigenvalue-scaling epilogue (G3S_SCALE)
      scale=0; [ "$cfg" = "1 1 1 g" ] && scale=1
      echo -n "{\"tile\": \"$t\", \"set\": \"$set\", \"cfg\": \"$cfg\", \"scale\": $scale, \"out\": "
      if [ $scale = 1 ]; then
        G3S_SCALE=1 timeout -k 5 60 tools/bin/g3s_t$t $set $cfg | tail -1 | tr -d '\n'
      else
        timeout -k 5 60 tools/bin/g3s_t$t $set $cfg | tail -1 | tr -d '\n'
      fi
      echo "}"
    done
  done
done
