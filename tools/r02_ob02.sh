#!/bin/bash
# round-2 OB02 check: the OB02 / golden / headline GPU tests, the OB02 probe (timings + profiled
# stage breakdown), and a bake A/B of the headline step
set -euo pipefail
out=gpurun_out/${1:-r02h}
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    -k "ob02 or subdiv or golden or headline or progress" > "$out/tests.log" 2>&1
timeout -k 10 200 python tools/ob02_probe.py 5 > "$out/probe.log" 2>&1
for b in 0 1; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --skip-256 --skip-config5 --skip-ob02 --bake $b > "$out/bench_bake$b.json" 2> "$out/bench_bake$b.err"
done
echo done
