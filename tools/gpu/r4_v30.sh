#!/bin/bash
# Round 4: env-only A/B of the preconditioning GEMM path on the final default.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4n2; mkdir -p $O
b() { name=$1; shift; env "$@" timeout -k 10 400 python3 bench.py --steps 100 --warmup 10 --secondary-bf16 0 --baseline 0 > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$name.json'));print('$name', d['value'], d['kind_ms'], d['params_finite'])"; }
b base A=1 && b torch KFAC_PRECOND_GEMM=torch && b bf16x3 KFAC_PRECOND_GEMM=bf16x3 && b base2 A=1
