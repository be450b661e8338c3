#!/bin/bash
# round-3 multi-rank rehearsal on the one-GPU box: the multi-process GPU tests, the slab probe at
# 512^3 (1 and 8 balanced slabs, kernel trace) and a 2-rank bench over gloo (both ranks on cuda:0;
# its timing is not meaningful, it exercises the N > 1 code path of bench.py)
set -euo pipefail
out=gpurun_out/${1:?tag}
mkdir -p "$out"
export TMPDIR=/tmp
IMPLISOLID_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline \
    --skip-config5 > "$out/bench_n2_gloo.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$out/slabtrace" -o run -- \
    python3 tools/slab_probe.py 512 10 1,8 balanced > "$out/slab_probe_512.json" 2> "$out/slab_probe.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/r256trace" -o run -- \
    python3 tools/slab_probe.py 256 10 1 balanced > "$out/slab_probe_256.json" 2> "$out/slab_probe256.err"
echo done
