#!/bin/bash
# round-3 check: the given GPU tests (default: the whole -m gpu suite), then the default bench line
#   usage: tools/r03_check.sh <tag> [pytest -k expression]
set -euo pipefail
out=gpurun_out/${1:?tag}
mkdir -p "$out"
export TMPDIR=/tmp
if [ -n "${2:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "$2" > "$out/tests.log" 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > "$out/tests.log" 2>&1
fi
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$out/bench.json" 2> "$out/bench.err"
echo done
