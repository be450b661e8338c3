#!/bin/bash
# round-4 profile run (one gpurun call, after the -m gpu suite is green): the round profile
# (tools/profile_round.sh: kernel stats, PMC traffic, VALU, the full bench line), the OB02 kernel
# stats of tools/ob02_probe.py, and a 2-rank bench over gloo (both ranks on cuda:0: it exercises the
# N > 1 code path of bench.py -- strong and weak legs gathered and checked, the stream-ordered
# sharded OB02 -- its timing is not meaningful).   usage: tools/r04_profile.sh <tag>
set -euo pipefail
tag=${1:?tag}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
root=$(pwd)
bash tools/profile_round.sh "$tag"
cp "$out/bench.log" profiles/${tag}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$root/$out/ob02" -o run -- python3 tools/ob02_probe.py 5 > "$out/ob02_probe.log" 2>&1
cp "$out/ob02/run_kernel_stats.csv" profiles/${tag}_ob02_kernel_stats.csv
cp "$out/ob02_probe.log" profiles/${tag}_ob02_probe.log
IMPLISOLID_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline \
    --skip-config5 > "$out/bench_n2_gloo.log" 2> "$out/bench_n2_gloo.err"
cp "$out/bench_n2_gloo.log" profiles/${tag}_n2_gloo_rehearsal.json
echo done
