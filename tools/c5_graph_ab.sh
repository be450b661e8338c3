#!/bin/bash
# config-5 merged pass: the pass captured as one graph (default) against direct launches
# (IMPLISOLID_NO_GRAPH=1), three alternating rounds.   usage: tools/c5_graph_ab.sh <tag>
set -euo pipefail
tag=${1:?tag}
out=gpurun_out/$tag
mkdir -p "$out"
for rep in 1 2 3; do
  for v in graph direct; do
    echo -n "$v $rep " >> "$out/c5_graph.txt"
    if [ $v = direct ]; then export IMPLISOLID_NO_GRAPH=1; else unset IMPLISOLID_NO_GRAPH; fi
    timeout -k 10 120 python3 tools/config5_merged_probe.py 64 128 20 2>/dev/null | grep merged >> "$out/c5_graph.txt"
  done
done
unset IMPLISOLID_NO_GRAPH
cat "$out/c5_graph.txt"
