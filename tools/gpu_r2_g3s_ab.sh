#!/bin/bash
# gemm3s integration: GPU tests, then A/B of the precondition GEMM path on
# ResNet-50 and NeoX-125M (same box, alternating)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gemm3_gpu.py tests/test_e2e_gpu.py tests/test_neox_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_g3s.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/pytest_g3s.log | head -20; tail -30 gpurun_out/pytest_g3s.log; exit 1; }
tail -1 gpurun_out/pytest_g3s.log
O=gpurun_out/g3s_ab.txt; : > $O
for mode in bf16x3 split bf16x3 split; do
  KFAC_PRECOND_GEMM=$mode timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --baseline 0 > gpurun_out/ab_rn.json 2> gpurun_out/ab_rn.err || { tail -20 gpurun_out/ab_rn.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/ab_rn.json').read().strip().splitlines()[-1]);print('resnet', '$mode', d['value'], d['kind_ms'])" >> $O
  KFAC_PRECOND_GEMM=$mode timeout -k 10 300 python3 tools/bench_neox.py --steps 12 --warmup 2 --no-sgd > gpurun_out/ab_nx.json 2> gpurun_out/ab_nx.err || { tail -20 gpurun_out/ab_nx.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ab_nx.json'));print('neox', '$mode', d['value'], d['kind_ms'])" >> $O
done
cat $O
