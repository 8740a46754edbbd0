#!/usr/bin/env python3
"""A/B of the bitsliced kernel in one-wave 4 KiB tiles (knob bs_wave, round 4) against the default
kernels (development tool).

C3 (k=10 m=4, 1 MiB, 256 stripes): encode, decode of data {0,1,2,3} and of the mixed {0,5,10,13}
under
  tables      the defaults of round 3 (LDS-table stream kernel for <= 4 outputs)
  wave1       bs_wave 1: outputs that are not consecutive slots (the mixed decode) on the bitsliced
              kernel in one-wave 4 KiB tiles, built with a 2-wave register budget
  wave2_all   bs_wave 2 + bitslice_min_rows 4: every pass on the one-wave bitsliced kernel
  bs4_16k     bitslice_min_rows 4, bs_wave 0: 4-wave 16 KiB tiles (round 3's C3 trial)
C5 (k=20 m=8, 4 MiB, 32 stripes): rebuild of {0..7} and the mixed {0,2,4,6,20,22,24,26} with
bs_wave 0 / 1 / 2.
Every variant's bytes are checked equal to the tables' output first, and the launch counter says
whether the bitsliced kernel ran.  Interleaved rounds after a settle, HIP events per launch, median
fraction of 8 TB/s of the algorithmic bytes ((k + outputs) x F per stripe)."""
import ctypes as C
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from liberasurecode_amd import _lib  # noqa: E402
from liberasurecode_amd import device as D  # noqa: E402

C3 = (10, 4, 1 << 20, 256, {"encode": None, "decode": [0, 1, 2, 3], "decode_mixed": [0, 5, 10, 13]})
C5 = (20, 8, 4 << 20, 32, {"rebuild_data": list(range(8)), "rebuild_mixed": [0, 2, 4, 6, 20, 22, 24, 26]})
C5E = (20, 8, 4 << 20, 32, {"encode": None, "rebuild_data": list(range(8)), "rebuild_mixed": [0, 2, 4, 6, 20, 22, 24, 26]})
C2 = (4, 2, 64 << 10, 4096, {"encode": None, "decode": [0, 1], "decode_mixed": [0, 4]})
# round 5: 1-2-output maps (knob bs_narrow_min_k) -- single-destination reconstruct (Swift's
# reconstructor), 1-2 lost -- and the one-wave LDS-DMA ring (bs_wave_depth)
C3N = (10, 4, 1 << 20, 256, {"rec_data": ("rec", [3], 3), "rec_parity": ("rec", [12], 12),
                             "decode_1": [0], "decode_2": [0, 11]})
C5N = (20, 8, 4 << 20, 32, {"rec_x8_d5": ("rec", list(range(8)), 5),
                            "rec_mixed_d22": ("rec", [0, 2, 4, 6, 20, 22, 24, 26], 22)})
# round 4, first run (profiles/r04_bs_wave_ab1.log): bs_wave 0 (tables), 1 = then only outputs that are
# not consecutive slots, 2 + bitslice_min_rows 4 = every C3 pass, bitslice_min_rows 4 alone = 4-wave
# 16 KiB tiles (decodes spilled there and fell back to the tables).  Now bs_wave 1 is the default
# for 3-4-output maps.
VARIANTS = {"c3": {"tables": {"bs_wave": 0}, "wave1": {}, "bs4_16k": {"bs_wave": 0, "bitslice_min_rows": 4}},
            # round 4, later: the next input's chunks loaded before each network (knob bs_prefetch; measured
            # neutral here, profiles/r04_bs_prefetch_ab.log, so the library now applies it to copy-through maps only)
            "c3pf": {"wave1": {}, "pf2": {"bs_prefetch": 2}, "pf4": {"bs_prefetch": 4}},
            "c2": {"tables": {}, "wave_2rows": {"bs_wave_min_rows": 2}},
            "c5": {"wave0": {}, "wave2": {"bs_wave": 2}},
            "c3ring": {"wave1": {}, "ring2": {"bs_wave_depth": 2}, "ring4": {"bs_wave_depth": 4}},
            "c3n": {"tables": {"bs_narrow_min_k": 0}, "narrow": {"bs_narrow_min_k": 1},
                    "narrow_ring2": {"bs_narrow_min_k": 1, "bs_wave_depth": 2}},
            "c5n": {"tables": {"bs_narrow_min_k": 0}, "narrow": {"bs_narrow_min_k": 1},
                    "narrow_ring2": {"bs_narrow_min_k": 1, "bs_wave_depth": 2}},
            # round 5: amdgpu_waves_per_eu(2, 2) capped the one-wave kernel at 2 waves per SIMD (descriptor
            # VGPRs padded to 176); occupancy variants (knobs bs_wave_wmin / wmax / barrier / depth)
            "c3occ": {"w22": {"bs_wave_wmin": 2, "bs_wave_wmax": 2, "bs_wave_barrier": 0},
                      "w28": {"bs_wave_wmin": 2, "bs_wave_wmax": 8, "bs_wave_barrier": 0},
                      "w28b": {"bs_wave_wmin": 2, "bs_wave_wmax": 8, "bs_wave_barrier": 1},
                      "w58b": {"bs_wave_wmin": 5, "bs_wave_wmax": 8, "bs_wave_barrier": 1},
                      "ring2_w28": {"bs_wave_wmin": 2, "bs_wave_wmax": 8, "bs_wave_depth": 2}},
            # measured: more waves per SIMD run SLOWER (w22 0.742 / w28 0.717 / w28b 0.711, r05_ab_occ.log)
            "c3occ2": {"w22": {"bs_wave_wmin": 2, "bs_wave_wmax": 2, "bs_wave_barrier": 0},
                       "w11": {"bs_wave_wmin": 1, "bs_wave_wmax": 1, "bs_wave_barrier": 0},
                       "w22b": {"bs_wave_wmin": 2, "bs_wave_wmax": 2, "bs_wave_barrier": 1}},
            # resident one-wave workgroups per CU between the register-set occupancies (knob bs_wave_per_cu over
            # a 4-wave-per-SIMD build: (2, 8) + barrier)
            "c3cap": {"w22b": {"bs_wave_wmin": 2, "bs_wave_wmax": 2, "bs_wave_barrier": 1},
                      **{f"cap{n}": {"bs_wave_wmin": 2, "bs_wave_wmax": 8, "bs_wave_barrier": 1, "bs_wave_per_cu": n}
                         for n in (6, 7, 8, 9, 10, 12)}},
            "c5ncap": {"w22": {"bs_narrow_min_k": 1, "bs_wave_wmin": 2, "bs_wave_wmax": 2},
                       **{f"cap{n}": {"bs_narrow_min_k": 1, "bs_wave_wmin": 8, "bs_wave_wmax": 8, "bs_wave_per_cu": n}
                          for n in (6, 7, 8, 9, 10, 12)}},
            # finer: the cap-7 optimum (r05_ab_cap.log: C3 encode 0.80) against w22, on both builds
            "c3cap2": {"w22b": {"bs_wave_wmin": 2, "bs_wave_wmax": 2, "bs_wave_barrier": 1},
                       "cap7": {"bs_wave_wmin": 2, "bs_wave_wmax": 8, "bs_wave_barrier": 1, "bs_wave_per_cu": 7},
                       "cap7_w22b": {"bs_wave_wmin": 2, "bs_wave_wmax": 2, "bs_wave_barrier": 1, "bs_wave_per_cu": 7},
                       "cap7_w28": {"bs_wave_wmin": 2, "bs_wave_wmax": 8, "bs_wave_barrier": 0, "bs_wave_per_cu": 7},
                       "cap5": {"bs_wave_wmin": 2, "bs_wave_wmax": 8, "bs_wave_barrier": 1, "bs_wave_per_cu": 5},
                       "cap7_ring2": {"bs_wave_wmin": 2, "bs_wave_wmax": 8, "bs_wave_depth": 2, "bs_wave_per_cu": 7}},
            "c5cap": {"tiles16k": {},
                      "wave_cap7": {"bs_wave": 2, "bs_wave_wmin": 2, "bs_wave_wmax": 2, "bs_wave_per_cu": 7},
                      "wave_cap6": {"bs_wave": 2, "bs_wave_wmin": 2, "bs_wave_wmax": 2, "bs_wave_per_cu": 6},
                      "wave_w22": {"bs_wave": 2, "bs_wave_wmin": 2, "bs_wave_wmax": 2}},
            # round 5 defaults: (2, 2) + barrier, 7 one-wave workgroups per CU; 1-2-output maps
            "c3ncap": {"tables": {"bs_narrow_min_k": 0},
                       "w22b_cap7": {"bs_narrow_min_k": 1},
                       "w22_cap7": {"bs_narrow_min_k": 1, "bs_wave_barrier": 0},
                       "w88_cap7": {"bs_narrow_min_k": 1, "bs_wave_wmin": 8, "bs_wave_wmax": 8, "bs_wave_barrier": 0},
                       "w22b_cap8": {"bs_narrow_min_k": 1, "bs_wave_per_cu": 8}},
            "c5ncap2": {"tables": {"bs_narrow_min_k": 0},
                        "w22b_cap7": {"bs_narrow_min_k": 1},
                        "w22_cap7": {"bs_narrow_min_k": 1, "bs_wave_barrier": 0},
                        "w88_cap7": {"bs_narrow_min_k": 1, "bs_wave_wmin": 8, "bs_wave_wmax": 8, "bs_wave_barrier": 0},
                        "w22b_cap8": {"bs_narrow_min_k": 1, "bs_wave_per_cu": 8}},
            # the LDS ring at capped residency: fewer waves, each with its next input in flight
            "c3ringcap": {"regs_cap7": {},
                          "ring2_cap7": {"bs_wave_depth": 2},
                          "ring2_cap6": {"bs_wave_depth": 2, "bs_wave_per_cu": 6},
                          "ring2_cap5": {"bs_wave_depth": 2, "bs_wave_per_cu": 5},
                          "ring4_cap6": {"bs_wave_depth": 4, "bs_wave_per_cu": 6}},
            "c2wgs": {"wgs0": {"wgs_per_cu": 0}, "wgs2": {"wgs_per_cu": 2}, "wgs3": {"wgs_per_cu": 3}},
            # round 5: lanes per workgroup of the 16 KiB-tile form (8 / 16 / 32 KiB tiles)
            # the default build ((2, 2) + barrier) at 6 / 7 / 8 resident workgroups per CU, per pattern
            "c3cap3": {"cap6": {"bs_wave_per_cu": 6}, "cap7": {}, "cap8": {"bs_wave_per_cu": 8}},
            "c5ncap3": {"cap6": {"bs_wave_per_cu": 6}, "cap7": {}, "cap8": {"bs_wave_per_cu": 8}},
            "c3pf5": {"pf0": {}, "pf2": {"bs_plain_prefetch": 2}, "pf4": {"bs_plain_prefetch": 4}},
            # robustness of the cap across batch sizes and fragment sizes
            "c3s64": {"cap7": {}, "cap8": {"bs_wave_per_cu": 8}, "cap6": {"bs_wave_per_cu": 6}},
            "c3s1024": {"cap7": {}, "cap8": {"bs_wave_per_cu": 8}, "cap6": {"bs_wave_per_cu": 6}},
            "c3f256k": {"cap7": {}, "cap8": {"bs_wave_per_cu": 8}, "cap6": {"bs_wave_per_cu": 6}},
            "c5tt": {"t256": {}, "t128": {"bs_tile_threads": 128}, "t512": {"bs_tile_threads": 512}},
            "c5tile": {"cap0": {"bs_tile_per_cu": 0}, "cap1": {"bs_tile_per_cu": 1}},
            # the 16 KiB-tile form's LDS-DMA ring (inputs ahead of the network in LDS, not registers)
            "c5depth": {"d0": {}, "d2": {"bitslice_depth": 2}, "d4": {"bitslice_depth": 4}},
            "c5nocc": {"w88": {"bs_narrow_min_k": 1, "bs_wave_wmin": 8, "bs_wave_wmax": 8},
                       "w44": {"bs_narrow_min_k": 1, "bs_wave_wmin": 4, "bs_wave_wmax": 4},
                       "w22": {"bs_narrow_min_k": 1, "bs_wave_wmin": 2, "bs_wave_wmax": 2},
                       "w11": {"bs_narrow_min_k": 1, "bs_wave_wmin": 1, "bs_wave_wmax": 1}},
            "c3nocc": {"w88": {"bs_narrow_min_k": 1, "bs_wave_wmin": 8, "bs_wave_wmax": 8},
                       "w44": {"bs_narrow_min_k": 1, "bs_wave_wmin": 4, "bs_wave_wmax": 4},
                       "w22": {"bs_narrow_min_k": 1, "bs_wave_wmin": 2, "bs_wave_wmax": 2}},
            "c2n": {"tables": {"bs_narrow_min_k": 0}, "narrow": {"bs_narrow_min_k": 1},
                    "narrow_ring2": {"bs_narrow_min_k": 1, "bs_wave_depth": 2}}}
DEFAULTS = {"bs_plain_prefetch": 0, "bs_tile_threads": 256, "wgs_per_cu": 0, "bs_tile_per_cu": 0, "bs_wave_per_cu": -1, "bs_copy_per_cu": 0, "xor_per_cu": 0, "bs_wave": -1, "bitslice_min_rows": 0, "bs_wave_min_rows": 0, "bs_prefetch": -1,
            "bs_narrow_min_k": -1, "bs_wave_depth": 0, "bs_wave_wmin": 0, "bs_wave_wmax": 0, "bs_wave_barrier": -1,
            "bitslice_depth": 0}


def launches():
    f = _lib.dev().ecamd_bitslice_launches
    f.restype = C.c_longlong
    return f()


def apply(d, knobs):
    for k, v in DEFAULTS.items():
        d.ecamd_tune(k.encode(), v)
    for k, v in knobs.items():
        d.ecamd_tune(k.encode(), v)


def run(cfg, rounds=3, n=30, skip=10):
    K, M, F, S, ops = {"c3": C3, "c3pf": C3, "c2": C2, "c5": C5, "c3ring": C3, "c3n": C3N, "c5n": C5N,
                       "c2n": C2, "c3occ": C3, "c3occ2": C3, "c5nocc": C5N, "c3nocc": C3N,
                       "c3cap": C3, "c5ncap": C5N, "c3cap2": C3, "c5cap": C5, "c3ncap": C3N, "c5ncap2": C5N, "c5tile": C5, "c5depth": C5, "c3ringcap": C3, "c2wgs": C2, "c5tt": C5E, "c3cap3": C3, "c5ncap3": C5N, "c3pf5": C3,
                       "c3s64": (10, 4, 1 << 20, 64, C3[4]), "c3s1024": (10, 4, 1 << 20, 1024, C3[4]),
                       "c3f256k": (10, 4, 256 << 10, 1024, C3[4])}[cfg]
    d = _lib.dev()
    d.ecamd_tune(b"bitslice", 2)
    lay = D.Layout.alloc(K + M, F, S)
    st = D.Stream()
    lay.fill_splitmix(nfrags=K, stream=st)
    D.rs_encode(K, M, lay, stream=st)
    st.synchronize()  # the download does not wait for `st`
    src = lay.download_stripes()

    def op_fn(pat):
        if pat is None:
            return lambda: D.rs_encode(K, M, lay, stream=st)
        if isinstance(pat, tuple):  # ("rec", missing, dest): one destination
            return lambda: D.rs_reconstruct(K, M, pat[1], pat[2], lay, stream=st)
        return lambda: D.rs_decode(K, M, pat, lay, stream=st)

    def n_out(pat):
        return M if pat is None else 1 if isinstance(pat, tuple) else len(pat)

    # exactness and which kernel runs: every variant rebuilds every op from the same fragments
    ran = {}
    for vname, knobs in VARIANTS[cfg].items():
        apply(d, knobs)
        for op, pat in ops.items():
            lay.upload_stripes(src)
            n0 = launches()
            op_fn(pat)()
            st.synchronize()
            assert (lay.download_stripes() == src).all(), (vname, op)
            ran[(vname, op)] = launches() - n0
    for _ in range(60):
        op_fn(list(ops.values())[0])()
    st.synchronize()
    res = {}
    for rnd in range(rounds):
        for vname, knobs in VARIANTS[cfg].items():
            apply(d, knobs)
            for op, pat in ops.items():
                fn = op_fn(pat)
                outs = n_out(pat)
                algo = S * (K + outs) * F
                ev = [D.Event() for _ in range(n + 1)]
                ev[0].record(st)
                for i in range(n):
                    fn()
                    ev[i + 1].record(st)
                st.synchronize()
                ms = statistics.median(ev[i].elapsed_ms(ev[i + 1]) for i in range(skip, n))
                res.setdefault((vname, op), []).append(algo / (ms * 1e-3) / 8e12)
                print(json.dumps({"cfg": cfg, "round": rnd, "variant": vname, "op": op, "ms": round(ms, 4),
                                  "frac": round(algo / (ms * 1e-3) / 8e12, 4),
                                  "bitsliced_launches": ran[(vname, op)]}), flush=True)
    for (vname, op), v in res.items():
        print(json.dumps({"cfg": cfg, "summary": vname, "op": op, "median_frac": round(statistics.median(v), 4),
                          "bitsliced_launches": ran[(vname, op)]}), flush=True)
    apply(d, {})
    d.ecamd_tune(b"bitslice", 1)
    lay.buf.free()


if __name__ == "__main__":
    for cfg in (sys.argv[1:] or ["c3", "c2", "c5"]):
        run(cfg)
