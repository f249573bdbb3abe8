#!/bin/bash
# Round 3: SYRK v2 (pre-split bf16 planes, buffer-load implicit im2col, two-pass split-K reduce)
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r3k2; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_bnact_gpu.py -k "syrk or cov or bn" > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 240 python3 -u tools/syrk_probe.py --json $O/v2.jsonl > $O/v2.log 2>&1 || { echo "probe rc=$?"; tail -20 $O/v2.log; exit 1; }
tail -1 $O/v2.log
timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -5 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['kind_ms'],d.get('sgd_ms_per_step'),d['params_finite'])"
KFAC_GRAPH_KINDS=plain timeout -k 10 300 python3 -u bench.py --steps 100 --warmup 10 --secondary-bf16 0 > $O/bench_plainonly.json 2> $O/bench_plainonly.err || { echo "bench2 rc=$?"; tail -5 $O/bench_plainonly.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_plainonly.json'));print('plain-only graphs', d['value'],d['ms_per_step'],d['kind_ms'],d['params_finite'])"
timeout -k 10 400 python -u tools/graph_nan_probe.py --steps 26 --image 224 --batch 32 --fused-sgd 1 --factor-steps 10 > $O/nan_bf16.jsonl 2> $O/nan_bf16.err || { echo "nanprobe rc=$?"; tail -3 $O/nan_bf16.err; exit 1; }
python3 -c "
import json
for l in open('$O/nan_bf16.jsonl'):
    d=json.loads(l); print(d['step'], d['kind'], d['how'], d['loss'], 'param', d['param'], 'pbuf', d['pbuf']['maxrel'])
"
