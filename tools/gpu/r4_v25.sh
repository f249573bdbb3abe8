#!/bin/bash
# Round 4: refresh phase time, eager vs graphed bench (HIP-event phases), and
# every refresh of a 300-step window.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4i2; mkdir -p $O
for g in 0 1; do
  timeout -k 10 400 python3 bench.py --steps 300 --warmup 10 --secondary-bf16 0 --baseline 0 --graphs $g --phase-timing > $O/phase_g$g.json 2> $O/phase_g$g.err || exit 1
  python3 -c "import json;d=json.load(open('$O/phase_g$g.json'));print('graphs $g', d['value'], d['kind_ms'], d.get('inverse_ms_each'), {k: round(v*100,1) for k,v in d.get('phase_ms_per_step',{}).items() if k=='inverse'})"
done
