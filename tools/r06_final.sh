#!/bin/bash
# Round-6 final evidence, one gpurun call (outputs under gpurun_out/<tag>/, copied into profiles/
# by hand afterwards): the whole -m gpu suite, smoke(), the round profile (tools/profile_round.sh:
# kernel stats, PMC traffic, VALU, the default bench line), the OB02 probe's kernel stats, the slab
# trace, and the 2-rank gloo rehearsal of bench.py's N > 1 path.  Each GPU step has its own time
# limit; the first failure ends the script.   usage: tools/r06_final.sh <tag> [part]
#   part: all (default) | a (tests, smoke, profile) | b (OB02 stats, slab trace, gloo rehearsal)
set -euo pipefail
tag=${1:?tag}; part=${2:-all}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
root=$(pwd)
if [ "$part" = all ] || [ "$part" = a ]; then
  bash tools/r06_run.sh "$tag" tests
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$out/smoke.log" 2>&1
  ps -u "$(id -u)" -o pid,ppid,stat,etime,args > "$out/ps_before_profile.txt" || true
  bash tools/profile_round.sh "$tag"
  sleep 2
  ps -u "$(id -u)" -o pid,ppid,stat,etime,args > "$out/ps_after_bench.txt" || true
fi
if [ "$part" = all ] || [ "$part" = b ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$root/$out/ob02" -o run -- \
      python3 tools/ob02_probe.py 5 > "$out/ob02_probe.log" 2>&1
  bash tools/r06_run.sh "$tag" slabtrace
  IMPLISOLID_DIST_BACKEND=gloo timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline \
      --skip-config5 > "$out/bench_n2_gloo.log" 2> "$out/bench_n2_gloo.err"
fi
echo done
