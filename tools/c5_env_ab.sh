#!/bin/bash
# config-5 merged pass, same-box A/B over library variants and environment settings, three rounds
# alternating:  tools/c5_env_ab.sh <tag> spec ...   with spec = main | <variant> | <label>:VAR=VALUE
# (<variant>: tools/build_variant.sh's variants/<variant>; <label>:VAR=VALUE: the in-tree library
# with VAR=VALUE in the environment)
set -euo pipefail
tag=${1:?tag}; shift
out=gpurun_out/$tag
mkdir -p "$out"
root=$(pwd)
for rep in 1 2 3; do
  for spec in "$@"; do
    lib=""; envs=()
    case "$spec" in
      main) ;;
      *:*=*) envs=("${spec#*:}") ;;
      *) lib=$root/variants/$spec/implisolid_amd/lib/libimplisolid_mi355x.so ;;
    esac
    echo -n "${spec%%:*} $rep " >> "$out/c5_ab.txt"
    env "${envs[@]}" IMPLISOLID_LIB=$lib timeout -k 10 120 python3 tools/config5_merged_probe.py 64 128 20 2>/dev/null \
        | grep merged >> "$out/c5_ab.txt"
  done
done
cat "$out/c5_ab.txt"
