#!/bin/bash
# full GPU suite, then the round profile (kernel trace, PMC traffic, SQ pass, full bench)
set -euo pipefail
tag=${1:?tag}
mkdir -p gpurun_out/$tag
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/$tag/gpu_tests.log 2>&1
bash tools/profile_round.sh $tag
