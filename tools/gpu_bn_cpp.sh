set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"; cd "$R"
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for g in 1 0; do
  for f in 1 0; do
    KFAC_FUSED_BN=$f timeout -k 10 300 python3 bench.py --graphs $g > gpurun_out/bn_cpp_g${g}_f$f.json 2>/dev/null || exit $?
    tail -1 gpurun_out/bn_cpp_g${g}_f$f.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('graphs=$g fused=$f', d['ms_per_step'], d['value'], 'sgd', d['sgd_ms_per_step'])"
  done
done
