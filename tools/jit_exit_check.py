#!/usr/bin/env python3
"""Exit with a bitsliced-kernel compile in flight (knob bitslice 1 starts it in the background):
libecamd stops its own compiler children at exit (hip/ecamd_jit.hip, stop_children_at_exit), so
none outlives the process -- check with `ps` right after, as tools/ does on the GPU box."""
import sys, os
sys.path.insert(0, os.getcwd())
import torch
from liberasurecode_amd import _lib, device as D
lay = D.Layout.alloc(21, 65536, 2)
lay.fill_splitmix(nfrags=13)
D.rs_decode(13, 8, [0, 1, 2, 3, 4, 5, 6, 13], lay)   # mode 1: starts a compile in the background
D.synchronize()
print("exiting with a compile in flight")
