#!/bin/bash
# round-2 check: full GPU suite, OB02 kernel profile, bake A/B of the headline step
set -euo pipefail
out=gpurun_out/${1:-r02d}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > "$out/tests.log" 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/ob02trace" -o run -- python3 tools/ob02_probe.py 3 > "$out/ob02_probe.log" 2>&1
for b in 0 1; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --skip-256 --skip-config5 --skip-ob02 --bake $b > "$out/bench_bake$b.json" 2> "$out/bench_bake$b.err"
done
echo done
