#!/bin/bash
# Round 4: env-only A/Bs on the final default (fp32, 100-step window, no SGD
# baseline): factor steps replayed too; symv wave budgets for the chains.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4h2; mkdir -p $O
b() { name=$1; shift; env "$@" timeout -k 10 400 python3 bench.py --steps 100 --warmup 10 --secondary-bf16 0 --baseline 0 > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$name.json'));print('$name', d['value'], d['kind_ms'], d.get('eigen_refresh_ms'), d.get('step_graphs'), d['params_finite'])"; }
b base A=1 && b kinds_pf KFAC_GRAPH_KINDS=plain,factor && b waves12k KFAC_SYTRD_WAVES=12288,6144 && b waves8k KFAC_SYTRD_WAVES=8192 && b base2 A=1
