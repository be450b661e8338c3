#!/bin/bash
# round-2 multi-GPU checks on the one-GPU box: new GPU tests, the slab balance probe at 512^3,
# and a 2-rank bench rehearsal over gloo (both ranks on cuda:0; its timing is not meaningful)
set -euo pipefail
out=gpurun_out/${1:-r02b}
mkdir -p "$out"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    -k "balanced or multi_device or multiprocess or headline or zslab" > "$out/tests.log" 2>&1
timeout -k 10 300 python tools/slab_probe.py 512 10 1,2,4,8 both > "$out/slab_probe_512.json" 2> "$out/slab_probe.err"
IMPLISOLID_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline \
    --skip-config5 --skip-ob02 > "$out/bench_n2_gloo.log" 2>&1
echo done
