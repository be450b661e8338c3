#!/bin/bash
# round-3 evidence run (one gpurun call): the whole -m gpu suite, the round profile
# (tools/profile_round.sh: kernel stats, PMC traffic, VALU, full bench line), and the OB02 kernel
# stats of tools/ob02_probe.py.  usage: tools/r03_profile.sh <tag>
set -euo pipefail
tag=${1:?tag}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
root=$(pwd)
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > "$out/tests.log" 2>&1
cp "$out/tests.log" profiles/${tag}_gpu_tests.log
bash tools/profile_round.sh "$tag"
cp "$out/bench.log" profiles/${tag}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$root/$out/ob02" -o run -- python3 tools/ob02_probe.py 5 > "$out/ob02_probe.log" 2>&1
cp "$out/ob02/run_kernel_stats.csv" profiles/${tag}_ob02_kernel_stats.csv
cp "$out/ob02_probe.log" profiles/${tag}_ob02_probe.log
echo done
