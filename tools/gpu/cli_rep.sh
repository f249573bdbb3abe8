export OMP_NUM_THREADS=1
mkdir -p $OUT
for i in 1 2 3 4; do
  d=$(mktemp -d)
  timeout -k 10 100 python examples/torch_imagenet_resnet.py --model resnet50 --epochs 2 --image-size 64 --synthetic-train-size 96 --synthetic-val-size 32 --batch-size 8 --val-batch-size 8 --workers 0 --log-dir $d --kfac-inv-update-steps 4 --kfac-factor-update-steps 2 --graphs 1 --checkpoint-freq 2 $CLI_EXTRA > $OUT/cli$i.log 2>&1 || exit 1
  rm -rf $d
  grep -i "capture\|replays\|differs" $OUT/cli$i.log | cut -c1-300
done
