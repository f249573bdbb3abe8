#!/bin/bash
# gemm3 phase pricing (DIAG builds) on the NeoX / ResNet shape sets + torch mm rates
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
O=$R/gpurun_out/g3diag.jsonl
: > $O
for set in neox resnet; do
  for ab in "1 0" "0 0" "1 1"; do
    for d in 0 1 2 3; do
      timeout -k 5 60 $R/benchbin/gemm3_bench_d$d $set $ab >> $O || { echo "FAILED d$d $set $ab"; exit 1; }
    done
  done
done
cat $O
timeout -k 10 120 python3 - <<'PY'
import torch, time, json
dev = 'cuda'
for (m, k, n) in [(2304, 769, 769), (2304, 2304, 769), (3072, 3072, 769), (768, 3073, 3073), (512, 4608, 4608)]:
    for dt in (torch.float32, torch.bfloat16):
        a = torch.randn(m, k, device=dev, dtype=dt); b = torch.randn(k, n, device=dev, dtype=dt)
        for _ in range(3): torch.mm(a, b)
        torch.cuda.synchronize(); t = time.perf_counter()
        for _ in range(20): torch.mm(a, b)
        torch.cuda.synchronize(); ms = (time.perf_counter() - t) / 20 * 1e3
        print(json.dumps({'m': m, 'k': k, 'n': n, 'dtype': str(dt), 'ms': round(ms, 4), 'tflops': round(2*m*k*n/ms/1e9, 1)}))
PY
