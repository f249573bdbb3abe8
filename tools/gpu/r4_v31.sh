#!/bin/bash
# Round 4: contribution of the hand-written kernels on the final default
# (env-only): fused BN kernels off, exact-fp32 SYRK instead of bf16x3.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4o2; mkdir -p $O
b() { name=$1; shift; env "$@" timeout -k 10 400 python3 bench.py --steps 100 --warmup 10 --secondary-bf16 0 > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$name.json'));print('$name', d['value'], d['kind_ms'], d.get('sgd_ms_per_step'), d['params_finite'])"; }
b base A=1 && b nofusedbn KFAC_FUSED_BN=0 && b syrk_exact KFAC_SYRK_FP32=exact
