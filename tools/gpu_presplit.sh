set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"; cd "$R"
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for ps in 1 0 1 0; do
  KFAC_GEMM3_PRESPLIT=$ps timeout -k 10 300 python3 bench.py --phase-timing > gpurun_out/presplit_$ps.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.loads(open('gpurun_out/presplit_$ps.json').read().strip().splitlines()[-1]); print('presplit=$ps', d['ms_per_step'], d['value'], d['sgd_ms_per_step'], {k: round(v,3) for k,v in d['phase_ms_per_step'].items()})"
done
