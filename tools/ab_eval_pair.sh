set -e
B="python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --skip-256 --skip-config5 --skip-ob02"
for v in 0 1 0 1; do
  IMPLISOLID_EVAL_PAIR=$v timeout -k 10 120 $B > gpurun_out/ab_$v.json 2>/dev/null
  python3 -c "import json;d=json.loads(open('gpurun_out/ab_$v.json').read().splitlines()[-1]);print('pair=$v', d['ms_per_step'], d['kernel_ms'])"
done
