# KFAC_SYTRD_MAXBATCH A/B on the eigensolver probe (3 x 4608 and the
# ResNet-50 step-100 mix), alternating, plus float64 accuracy once.
set -o pipefail
out=gpurun_out/r6r; mkdir -p $out

for mb in 0 2 1 0 2 1; do
  KFAC_SYTRD_MAXBATCH=$mb timeout -k 10 120 python tools/eigh_probe.py --sizes 4608 --count 3 --reps 3 --no-acc > $out/x3_mb$mb.json 2>/dev/null || exit $?
  echo "mb=$mb x3 $(tail -c 200 $out/x3_mb$mb.json)"
  KFAC_SYTRD_MAXBATCH=$mb timeout -k 10 120 python tools/eigh_probe.py --mix resnet50 --reps 3 --no-acc > $out/mix_mb$mb.json 2>/dev/null || exit $?
  echo "mb=$mb mix $(grep -o '"ms": \[[^]]*\]' $out/mix_mb$mb.json)"
done
KFAC_SYTRD_MAXBATCH=2 timeout -k 10 200 python tools/eigh_probe.py --mix resnet50 --reps 1 > $out/mix_mb2_acc.json 2>/dev/null || exit $?
echo "acc $(tail -c 600 $out/mix_mb2_acc.json)"
