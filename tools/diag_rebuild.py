"""Diagnostic: repeated builds of one shape at different resolutions must match fresh builds."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import implisolid_amd as I
from implisolid_amd import scenes

shape = scenes.config3_tree()
seq = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [64, 32, 64, 48, 64, 32, 64, 64, 32, 48]
out = []
for R in seq:
    v, f = I.make_geometry(shape, scenes.mc_settings(R, 1.0))
    out.append((R, len(v), len(f)))
    I.jit_wait()
print(out, flush=True)
