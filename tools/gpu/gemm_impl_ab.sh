# Refresh GEMMs: native gemm_f32 vs hipBLASLt (KFAC_GEMM_IMPL=lib),
# alternating, on 3 x 4608 and the ResNet-50 mix.
set -o pipefail
out=gpurun_out/r6t; mkdir -p $out
for impl in native lib native lib; do
  KFAC_GEMM_IMPL=$impl timeout -k 10 120 python tools/eigh_probe.py --sizes 4608 --count 3 --reps 3 --no-acc > $out/x3_$impl.json 2>/dev/null || exit $?
  echo "$impl x3 $(grep -o '"ms": \[[^]]*\]' $out/x3_$impl.json)"
  KFAC_GEMM_IMPL=$impl timeout -k 10 120 python tools/eigh_probe.py --mix resnet50 --reps 3 --no-acc > $out/mix_$impl.json 2>/dev/null || exit $?
  echo "$impl mix $(grep -o '"ms": \[[^]]*\]' $out/mix_$impl.json)"
done
