#!/bin/bash
# Build an experimental variant of the library from an edited copy of the sources:
#   tools/build_variant.sh NAME 'sed-expr' [file=csrc/grid.hpp]  (more pairs: 'expr' file ...)
# -> variants/NAME/implisolid_amd/lib/libimplisolid_mi355x.so (IMPLISOLID_LIB=... selects it).
# Edits go into the headers themselves, so the JIT's embedded copies see them too.
# VARIANTS=ab puts the build under ab/ (git-ignored, but not gpurun-ignored: it travels to the box).
# GIT_REF=<rev> takes csrc/ from that commit instead of the working tree (an A/B base).
set -euo pipefail
name=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
d=$root/${VARIANTS:-variants}/$name
rm -rf "$d"; mkdir -p "$d/implisolid_amd" "$d/tools"
cp -r "$root/implisolid_amd/csrc" "$root/implisolid_amd/Makefile" "$d/implisolid_amd/"
rm -f "$d/implisolid_amd/csrc/generated/jit_headers.inc"
cp "$root/tools/embed_headers.py" "$d/tools/"
cp -r "$root/include" "$d/"
if [ -n "${GIT_REF:-}" ]; then   # the sources, Makefile, header embedder and ABI header of that commit
    rm -rf "$d/implisolid_amd/csrc" "$d/include"; mkdir -p "$d/implisolid_amd/csrc"
    (cd "$root" && git archive "$GIT_REF" implisolid_amd/csrc implisolid_amd/Makefile tools/embed_headers.py include) | tar -x -C "$d"
    rm -f "$d/implisolid_amd/csrc/generated/jit_headers.inc"
fi
while [ $# -gt 0 ]; do
    expr=$1; file=${2:-csrc/grid.hpp}; shift; [ $# -gt 0 ] && shift
    sed -i "$expr" "$d/implisolid_amd/$file"
done
# optional: a python script editing the copy (cwd = the copy's implisolid_amd/)
if [ -n "${PATCH_PY:-}" ]; then (cd "$d/implisolid_amd" && python3 "$PATCH_PY"); fi
make -s -j8 -C "$d/implisolid_amd" > "$d/build.log" 2>&1 || { cat "$d/build.log"; exit 1; }
echo "$d/implisolid_amd/lib/libimplisolid_mi355x.so"
