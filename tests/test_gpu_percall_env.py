"""GPU: the per-call path's non-default staging modes (host/hostio.cpp), each in a child process
because the settings are read once per process: the kernel reading its inputs from the
pinned slab for every size (ECAMD_PERCALL_ZEROCOPY_MODE 3) or only its outputs (2, inputs by DMA
everywhere: ZEROCOPY_IN_KIB 0), inputs AND outputs by DMA (mode 0 / ZEROCOPY_KIB 0), the kernel
writing its outputs to device memory while reading the slab (mode 1: the CRC pass then copies the
inputs to the device slab), inputs packed through the PCIe BAR (ECAMD_PERCALL_BAR_KIB), and the
checksum pass unfused (ECAMD_PERCALL_FUSE_CRC 0), the stream synchronized instead of the kernel's
completion flag polled (ECAMD_PERCALL_DONE_FLAG 0) -- RS(10,4) encode / decode / reconstruct at 4 KiB,
64 KiB and 1 MiB with CHKSUM_NONE and CRC32, byte-exact against the restated framing, and every
setting's output digest equal to the default's."""
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
    "stream_sync": {"ECAMD_PERCALL_DONE_FLAG": "0"},
}


def _run(env_extra):
    env = dict(os.environ, **env_extra)
    r = subprocess.run([sys.executable, os.path.join(HERE, "percall_env_run.py")], env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.fixture(scope="module")
def default_digest():
    return _run({})["digest"]


@pytest.mark.parametrize("name", [n for n in SETTINGS if n != "default"])
def test_percall_setting_byte_exact(name, default_digest):
    out = _run(SETTINGS[name])
    assert out["ok"] and out["digest"] == default_digest, (name, out)
