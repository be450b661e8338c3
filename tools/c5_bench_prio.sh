#!/bin/bash
# the bench's config-5 merged leg with the deep class's stream at the lowest priority and at the
# default priority, two alternating rounds.   usage: tools/c5_bench_prio.sh <tag>
set -euo pipefail
tag=${1:?tag}
out=gpurun_out/$tag
mkdir -p "$out"
for rep in 1 2; do
  for v in 1 0; do
    IMPLISOLID_BATCH_DEEP_PRIO=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --skip-ob02 --skip-concurrent \
        --no-cpu-baseline --skip-256 > "$out/b_p${v}_$rep.json" 2> "$out/b_p${v}_$rep.err"
    python3 -c "import json,sys; b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], b['config5']['objects_per_s'], b['config5']['ms_per_stream'])" "$out/b_p${v}_$rep.json"
  done
done
