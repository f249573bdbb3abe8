# fused-BN A/B: SGD-only and K-FAC bench (graphs) with KFAC_FUSED_BN=1 / 0,
# plus a steady-state SGD rocprof summary with the fused kernels
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"; cd "$R"
for f in 1 0 1 0; do
  KFAC_FUSED_BN=$f timeout -k 10 300 python3 bench.py --no-kfac --steps 200 --warmup 20 > gpurun_out/bn_ab_sgd_$f.json 2>/dev/null || exit $?
  tail -1 gpurun_out/bn_ab_sgd_$f.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('sgd fused=$f', d['ms_per_step'], d['value'])"
done
KFAC_FUSED_BN=1 timeout -k 10 300 python3 bench.py > gpurun_out/bn_ab_kfac_1.json 2>/dev/null || exit $?
tail -1 gpurun_out/bn_ab_kfac_1.json
KFAC_FUSED_BN=0 timeout -k 10 300 python3 bench.py > gpurun_out/bn_ab_kfac_0.json 2>/dev/null || exit $?
tail -1 gpurun_out/bn_ab_kfac_0.json
KFAC_FUSED_BN=1 STEPS=100 TAG=sgd_fused EXTRA=--no-kfac bash tools/gpu_profile.sh || exit $?
cd "$R"; head -12 gpurun_out/prof_keep/sgd_fused_steady_summary.txt
