# A/B: MIOpen's ASM NHWC weight-gradient solver (fp32 workspace + zero fill +
# cast kernels) vs forcing the CK grouped wrw solver, on the SGD step.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for rep in 1 2; do
 for v in base ckwrw; do
  if [ $v = ckwrw ]; then export MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0; else unset MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC; fi
  timeout -k 10 300 python3 bench.py --steps 40 --warmup 10 --no-kfac > gpurun_out/wrw_$v.json 2> gpurun_out/wrw_$v.err || { tail -5 gpurun_out/wrw_$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/wrw_$v.json').read().strip().splitlines()[-1]); print('$v', $rep, d['ms_per_step'], d['value'])"
 done
done
