#!/usr/bin/env python3
"""Calibrate the oracle restatement (port) against the reference codec on one core
(within +-15% of the reference's per-core C3 figures)."""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import oracle_lib as orc  # noqa: E402
from ecdata import stripe_fragments  # noqa: E402

k, m, F, N = 10, 4, 1 << 20, 6
IP = C.POINTER(C.c_int)
ref = C.CDLL(os.path.join(ROOT, "oracle", "_ref", "liberasurecode_rs_vand.so.1"))
ref.make_systematic_matrix.restype = IP
ref.make_systematic_matrix.argtypes = [C.c_int, C.c_int]
ref.liberasurecode_rs_vand_encode.argtypes = [IP, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int]
ref.init_liberasurecode_rs_vand(k, m)
Gr = ref.make_systematic_matrix(k, m)
Go = orc.ints(orc.generator(k, m))
data = [np.array(x) for x in stripe_fragments(1, k, F)]
par = [np.zeros(F, np.uint8) for _ in range(m)]
dp, pp = orc.ptr_array(data), orc.ptr_array(par)
res = {}
for name, fn, G in (("reference", ref.liberasurecode_rs_vand_encode, Gr),
                    ("port", orc.lib().orc_rs_encode, Go)):
    fn(G, dp, pp, k, m, F)
    t0 = time.perf_counter()
    for _ in range(N):
        fn(G, dp, pp, k, m, F)
    res[name] = round(N * k * F / 1e6 / (time.perf_counter() - t0), 1)
res["ratio_port_over_reference"] = round(res["port"] / res["reference"], 3)
print(json.dumps({"c3_raw_encode_MBps_1core": res}))
