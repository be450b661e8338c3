#!/bin/bash
# fold walk check: the fold / OB02 GPU tests, the fold probe with walk statistics, the OB02 probe
set -euo pipefail
out=gpurun_out/${1:?tag}
mkdir -p "$out"
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "fold or ob02 or headline" > "$out/tests.log" 2>&1
tail -2 "$out/tests.log"
IMPLISOLID_FOLD_STATS=1 timeout -k 10 120 python3 tools/fold_probe.py > "$out/fold.log" 2>&1
grep -v amdgpu.ids "$out/fold.log" | tail -12
timeout -k 10 200 python3 tools/ob02_probe.py 5 > "$out/ob02.log" 2>&1
grep -v amdgpu.ids "$out/ob02.log" | head -6
