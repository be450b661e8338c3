#!/bin/bash
# round-5 GPU run (one gpurun call).  usage: tools/r05_run.sh <tag> <what...>
#   tests       the whole -m gpu suite
#   tests:<k>   the -m gpu tests matching -k <k>
#   bench       the default bench line (N = 1)
#   benchob     the bench's OB02 legs only (no config 5, no concurrent builds, no CPU baselines)
#   ob02prof    kernel stats of tools/ob02_probe.py (config 2 / 3 / 3s builds)
#   projstats   the projection's evaluations per face, wave balance and late-pass faces
#   fold        the edge-length fold alone on real meshes' edge lengths (stats + kernel trace)
# Each GPU step has its own time limit; the first failure ends the script.
set -euo pipefail
tag=${1:?tag}
shift
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
root=$(pwd)
for what in "$@"; do
  case "$what" in
    tests)
      timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$out/tests.log" 2>&1
      cp "$out/tests.log" profiles/${tag}_gpu_tests.log ;;
    tests:*)
      timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${what#tests:}" \
          > "$out/tests_k.log" 2>&1 ;;
    bench)
      timeout -k 10 600 python3 -u bench.py > "$out/bench.json" 2> "$out/bench.err" ;;
    benchob)
      timeout -k 10 600 python3 -u bench.py --steps 10 --skip-config5 --skip-concurrent --no-cpu-baseline --skip-256 \
          > "$out/bench_ob.json" 2> "$out/bench_ob.err" ;;
    ob02prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$root/$out/ob02" -o run -- \
          python3 tools/ob02_probe.py 5 > "$out/ob02_probe.log" 2>&1 ;;
    fold)
      IMPLISOLID_FOLD_STATS=1 timeout -k 10 200 python3 tools/fold_mesh_probe.py 3 > "$out/fold_stats.log" 2>&1
      timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$root/$out/fold" -o run -- \
          python3 tools/fold_mesh_probe.py 5 > "$out/fold_probe.log" 2>&1 ;;
    projstats)   # the projection's search balance per pass (tools/proj_stats_probe.py)
      IMPLISOLID_PROJ_STATS=1 timeout -k 10 200 python3 -u tools/proj_stats_probe.py > "$out/proj_stats.log" 2>&1 ;;
    shardtrace)   # the 8-shard OB02 loop at 256^3 under a kernel trace (tools/ob02_shard_probe.py)
      timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$root/$out/shard" -o run -- \
          python3 tools/ob02_shard_probe.py 8 256 > "$out/shard_probe.json" 2> "$out/shard_probe.err" ;;
    *) echo "unknown step $what"; exit 2 ;;
  esac
  echo "step $what done"
done
echo done
