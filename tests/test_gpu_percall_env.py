"""GPU: the per-call path's non-default staging modes (host/hostio.cpp), each in a child process
because the settings are read once per process: the kernel reading its inputs from the
pinned slab for every size (ECAMD_PERCALL_ZEROCOPY_MODE 3) or only its outputs (2, inputs by DMA
everywhere: ZEROCOPY_IN_KIB 0), inputs AND outputs by DMA (mode 0 / ZEROCOPY_KIB 0), the kernel
writing its outputs to device memory while reading the slab (mode 1: the CRC pass then copies the
inputs to the device slab), inputs packed through the PCIe BAR (ECAMD_PERCALL_BAR_KIB), and the
checksum pass unfused (ECAMD_PERCALL_FUSE_CRC 0), a small call's input CRC32s left to the frontend
(ECAMD_PERCALL_OVERLAP_CRC 0), the stream synchronized instead of the kernel's
completion flag polled (ECAMD_PERCALL_DONE_FLAG 0), one-launch calls launched instead of posted to the
resident small server (ECAMD_PERCALL_SERVER 0), and the server exiting between calls (a 50 us idle time and
a 1 ms pause after each call) -- RS(10,4) encode / decode / reconstruct at 4 KiB, 64 KiB and 1 MiB with
CHKSUM_NONE and CRC32, byte-exact against the restated framing, and every setting's output digest equal to
the default's.  Plus concurrent callers: 4 threads (a server each) and 12 (more than the library's 8
servers: the rest launch), every result checked."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
SETTINGS = {
    "default": {},
    "zerocopy_mode3": {"ECAMD_PERCALL_ZEROCOPY_MODE": "3"},
    "zerocopy_mode1": {"ECAMD_PERCALL_ZEROCOPY_MODE": "1"},
    "zerocopy_mode0": {"ECAMD_PERCALL_ZEROCOPY_MODE": "0", "ECAMD_PERCALL_ZEROCOPY_IN_KIB": "0"},
    "inputs_by_dma": {"ECAMD_PERCALL_ZEROCOPY_IN_KIB": "0"},
    "zerocopy_off": {"ECAMD_PERCALL_ZEROCOPY_KIB": "0"},
    "bar_64k": {"ECAMD_PERCALL_BAR_KIB": "64", "ECAMD_PERCALL_ZEROCOPY_IN_KIB": "0"},
    "crc_unfused": {"ECAMD_PERCALL_FUSE_CRC": "0"},
    "crc_overlap_off": {"ECAMD_PERCALL_OVERLAP_CRC": "0"},
    "stream_sync": {"ECAMD_PERCALL_DONE_FLAG": "0"},
    "server_off": {"ECAMD_PERCALL_SERVER": "0"},
    "server_idle_exit": {"ECAMD_PERCALL_SERVER_IDLE_US": "50", "PERCALL_SLEEP_US": "1000"},
}


def _run(env_extra):
    env = dict(os.environ, **env_extra)
    r = subprocess.run([sys.executable, os.path.join(HERE, "percall_env_run.py")], env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.fixture(scope="module")
def default_run():
    out = _run({})
    assert out["posts"] > 0 and out["server_launches"] >= 1, out  # the server served the one-launch calls
    return out


@pytest.mark.parametrize("name", [n for n in SETTINGS if n != "default"])
def test_percall_setting_byte_exact(name, default_run):
    out = _run(SETTINGS[name])
    assert out["ok"] and out["digest"] == default_run["digest"], (name, out)
    if name == "server_idle_exit":  # the server exits between calls: launched again for (nearly) every one
        assert out["posts"] == default_run["posts"] and out["server_launches"] > out["posts"] // 2, out
    elif name in ("server_off", "stream_sync", "zerocopy_off", "zerocopy_mode0", "zerocopy_mode1", "inputs_by_dma",
                  "bar_64k"):
        assert out["posts"] == 0, (name, out)  # no call met the server's conditions


@pytest.mark.parametrize("threads", [4, 12])
def test_percall_threads(threads):
    out = _run({"PERCALL_THREADS": str(threads)})
    assert out["ok"] and out["posts"] > 0, out


def test_percall_server_slot_churn():
    """The server's two argument slots and LDS table placements under churn (percall_env_run.churn_main):
    workgroups that sat out 510-514 rewrites keep no stale arguments; alternating operations keep their
    tables apart; every output byte-exact, most calls served."""
    out = _run({"PERCALL_CHURN": "1"})
    assert out["ok"] and out["posted"] > out["calls"] // 2, out
    # 50 alternating encode / decode pairs of one size: no slot rewritten once both blocks are cached (a
    # server idle exit in between, a stall past 2 ms, costs one rewrite of each; one slot would give 100)
    assert all(r <= 4 for r in out["alternating_rewrites"]), out

