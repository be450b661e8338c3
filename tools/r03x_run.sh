#!/bin/bash
# round-3 check of the build_geometry host-path changes: the GPU suite, the OB02 timeline (kernel
# trace of config 2 / 3s builds), the OB02 probe and the default bench line.  usage: tools/r03x_run.sh <tag>
set -euo pipefail
tag=${1:?tag}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > "$out/tests.log" 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$out/tl" -o run -- python3 tools/ob02_timeline.py run > "$out/tl.log" 2>&1
python3 tools/ob02_timeline.py analyse "$out/tl" > "$out/tl_analysis.txt" 2>&1
timeout -k 10 200 python3 tools/ob02_probe.py 5 > "$out/ob02_probe.log" 2>&1
timeout -k 10 500 python3 bench.py > "$out/bench.json" 2> "$out/bench.err"
echo done
