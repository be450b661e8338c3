#!/bin/bash
# Round profile on one MI355X (run from the repo root through gpurun):
#   kernel-trace stats of the bench, four PMC passes (FETCH_SIZE / WRITE_SIZE, pruned bench and the
#   unpruned calibration run), one SQ pass (VALU utilisation per kernel), the traffic summary, and
#   the full bench line with the CPU baseline.
#   usage: tools/profile_round.sh r01
# Each GPU step has its own time limit; the first failure ends the script.
set -euo pipefail
tag=${1:?round tag}
out=gpurun_out/$tag
mkdir -p "$out"
root=$(pwd)
export TMPDIR=/tmp
B="bench.py --steps 10 --warmup 4 --no-cpu-baseline --skip-256 --skip-config5 --skip-ob02 --skip-concurrent"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$root/$out/trace" -o run -- python3 $B > "$out/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$root/$out/fetch" -o run -- python3 $B > "$out/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$root/$out/write" -o run -- python3 $B > "$out/write.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$root/$out/cfetch" -o run -- python3 $B --prune 0 > "$out/cfetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$root/$out/cwrite" -o run -- python3 $B --prune 0 > "$out/cwrite.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU --output-format csv -d "$root/$out/sq" -o run -- python3 $B > "$out/sq.log" 2>&1
python3 tools/pmc_valu.py "$out/sq" > "$out/valu.json"
cp "$out/valu.json" profiles/valu_$tag.json
cp "$out/trace/run_kernel_stats.csv" profiles/${tag}_kernel_stats.csv
python3 tools/pmc_traffic.py --fetch "$out/fetch" --write "$out/write" --cal-fetch "$out/cfetch" --cal-write "$out/cwrite" \
    --R 512 --lib implisolid_amd/lib/libimplisolid_mi355x.so > "$out/traffic.json"
cp "$out/traffic.json" profiles/traffic_$tag.json
timeout -k 10 600 python3 bench.py > "$out/bench.log" 2>&1
echo done
