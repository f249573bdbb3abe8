# gemm3s tile-config sweep over the four ResNet-50 preconditioning tables
# (binaries built on the CPU side into benchbin/ from tools/gemm3s_bench.cpp)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
: > gpurun_out/g3s_sweep.jsonl
for v in ${VARIANTS:-t0 t4_s2 t4_s3 t5_s2 t5_s3 t6_s2 t6_s3 t7_s2 t7_s3}; do
 for cfg in "0 1 1 a" "1 1 1 g" "0 1 1 g" "0 0 0 a"; do
  out=$(timeout -k 5 60 ./benchbin/g3s_$v ${SET:-resnet} $cfg); rc=$?; if [ $rc != 0 ] && [ $rc != 2 ]; then echo "fail $v $cfg: $out"; exit 1; fi
  echo "{\"v\": \"$v\", ${out#\{}" >> gpurun_out/g3s_sweep.jsonl
 done
done
python3 -c "
import json
for l in open('gpurun_out/g3s_sweep.jsonl'):
    d=json.loads(l); print(d['v'], d['k'], d['a_mc'], d['b_mc'], d['out_split'], d['ms'], d['bf16_mfma_tflops'], d['rel_err'])
"
