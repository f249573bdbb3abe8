#!/bin/bash
# Round 4: env-only A/Bs of the GEMM 1x1 path: weight-gradient slab rows and
# hipBLASLt vs rocBLAS for torch's GEMMs (fp32, 100-step window, no SGD run).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4m2; mkdir -p $O
b() { name=$1; shift; env "$@" timeout -k 10 400 python3 bench.py --steps 100 --warmup 10 --secondary-bf16 0 --baseline 0 > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/$name.json'));print('$name', d['value'], d['kind_ms'], d['params_finite'])"; }
b base A=1 && b slab1k KFAC_CONV1X1_SLAB_ROWS=1024 && b slab4k KFAC_CONV1X1_SLAB_ROWS=4096 && b slab8k KFAC_CONV1X1_SLAB_ROWS=8192 && b rocblas TORCH_BLAS_PREFER_HIPBLASLT=0 && b base2 A=1
