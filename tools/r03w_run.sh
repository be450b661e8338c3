#!/bin/bash
# round-3 evidence run: tools/r03_profile.sh (GPU suite, kernel stats, PMC traffic, VALU, bench,
# OB02 kernel stats), then the OB02 timeline.  usage: tools/r03w_run.sh <tag>
set -euo pipefail
tag=${1:-r03w}
bash tools/r03_profile.sh "$tag"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "gpurun_out/$tag/tl" -o run -- python3 tools/ob02_timeline.py run > "gpurun_out/$tag/tl.log" 2>&1
python3 tools/ob02_timeline.py analyse "gpurun_out/$tag/tl" > "gpurun_out/$tag/tl_analysis.txt" 2>&1
echo done
