# A/B the full training step under different env settings: AB="VAR=val VAR=val2 ..."
set -o pipefail
mkdir -p gpurun_out
for kv in $AB; do
  echo "== $kv"
  env $kv timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-parity > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  python -c "import json; r=json.load(open('gpurun_out/ab.json')); print(r['value'], r['ms_per_step'], r['roofline']['kernel'], r['roofline']['avg_launch_us'])"
done
