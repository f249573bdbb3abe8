# graph_verify_probe.py over the ImageNet CLI's --graphs 1 configuration, 3 runs
export OMP_NUM_THREADS=1
mkdir -p $OUT
for i in 1 2 3; do
  d=$(mktemp -d)
  timeout -k 10 150 python tools/graph_verify_probe.py -n 6 -- examples/torch_imagenet_resnet.py --model resnet50 --epochs 1 --image-size 64 --synthetic-train-size 96 --synthetic-val-size 32 --batch-size 8 --val-batch-size 8 --workers 0 --log-dir $d --kfac-inv-update-steps 4 --kfac-factor-update-steps 2 --graphs 1 --checkpoint-freq 2 $CLI_EXTRA > $OUT/probe$i.log 2>&1 || exit 1
  rm -rf $d
  grep "\[probe\]" $OUT/probe$i.log | cut -c1-600
done
