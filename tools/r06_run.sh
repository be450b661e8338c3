#!/bin/bash
# round-6 GPU run (one gpurun call).  usage: tools/r06_run.sh <tag> <what...>
#   tests       the whole -m gpu suite
#   tests:<k>   the -m gpu tests matching -k <k>
#   head        the headline alone (512^3 and 256^3, 20 steps; no config 5 / OB02 / CPU baseline)
#   bench       the default bench line (N = 1)
#   benchob     the bench's OB02 legs only
#   slabtrace   kernel trace of tools/slab_probe.py 512 10 1,8 balanced (+ tools/slab_trace.py summary)
#   ob02prof    kernel stats of tools/ob02_probe.py (config 2 / 3 / 3s builds)
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
      timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$out/tests.log" 2>&1 ;;
    tests:*)
      timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${what#tests:}" \
          > "$out/tests_k.log" 2>&1 ;;
    head)
      timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --skip-config5 --skip-ob02 --skip-concurrent \
          --no-cpu-baseline > "$out/head.json" 2> "$out/head.err" ;;
    head2)
      timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --skip-config5 --skip-ob02 --skip-concurrent \
          --no-cpu-baseline --skip-256 > "$out/head2.json" 2> "$out/head2.err" ;;
    bench)
      timeout -k 10 600 python3 -u bench.py > "$out/bench.json" 2> "$out/bench.err" ;;
    benchob)
      timeout -k 10 600 python3 -u bench.py --steps 10 --skip-config5 --skip-concurrent --no-cpu-baseline --skip-256 \
          > "$out/bench_ob.json" 2> "$out/bench_ob.err" ;;
    slabtrace)
      timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$root/$out/slab" -o run -- \
          python3 tools/slab_probe.py 512 10 1,8 balanced > "$out/slab_probe.json" 2> "$out/slab_probe.err"
      python3 tools/slab_trace.py "$out/slab/run_kernel_trace.csv" 10 1,8 > "$out/slab_trace_summary.txt" ;;
    ob02prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$root/$out/ob02" -o run -- \
          python3 tools/ob02_probe.py 5 > "$out/ob02_probe.log" 2>&1 ;;
    *) echo "unknown step $what"; exit 2 ;;
  esac
  echo "step $what done"
done
echo done
