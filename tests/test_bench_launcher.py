"""CPU: bench.py's multi-rank launcher and stripe sharding (C4), rehearsed without a GPU.

`bench.py --gpus N` with no WORLD_SIZE in the environment starts N rank processes itself (fresh
interpreters, before anything touches the GPU) with RANK / WORLD_SIZE / LOCAL_RANK / MASTER_*;
`--dry-run` runs the same rank / shard plumbing on gloo and skips the kernels.  Stripes are
independent (src/erasurecode.c:383-477): the shards must cover the batch exactly once."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_bench(*args, env=None):
    e = dict(os.environ)
    for key in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(key, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + list(args),
                          capture_output=True, text=True, timeout=300, env=e, cwd=ROOT)


@pytest.mark.parametrize("gpus,scaling,per_rank", [(2, "weak", [256, 256]),
                                                    (2, "strong", [1024, 1024]),
                                                    (3, "strong", [683, 683, 682])])
def test_launcher_starts_ranks_and_covers_every_stripe(gpus, scaling, per_rank):
    r = run_bench("--gpus", str(gpus), "--dry-run", "--scaling", scaling, "--cpu-seconds", "0.2")
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["dry_run"] and line["covered_once"]
    assert line["n_gpus"] == gpus and line["ranks_seen"] == gpus
    assert line["stripes_per_rank"] == per_rank
    assert line["total_stripes"] == sum(per_rank)
    # north_star: the host-CPU baseline "from the same run" at every GPU count -- rank 0 times it
    # while the other ranks wait on a gloo barrier
    cpu = line["cpu_baseline"]
    assert cpu["value"] > 0 and cpu["cores"] >= 1 and cpu["kind"] in ("reference", "port")
    assert cpu["ranks_idle"] == gpus - 1
    assert "k=10 m=4" in cpu["sample"]


def test_dry_run_without_cpu_baseline():
    r = run_bench("--gpus", "2", "--dry-run", "--no-cpu-baseline")
    assert r.returncode == 0, r.stderr[-2000:]
    assert "cpu_baseline" not in json.loads(r.stdout.strip().splitlines()[-1])


def test_mismatched_world_fails_loudly():
    r = run_bench("--gpus", "1", "--dry-run", env={"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr


def test_single_rank_dry_run():
    r = run_bench("--dry-run", "--cpu-seconds", "0.2")
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 1 and line["stripes_per_rank"] == [256]
    assert line["cpu_baseline"]["ranks_idle"] == 0


@pytest.mark.parametrize("k,width,F,S,cus,want", [
    (10, 4, 1 << 20, 256, 256, 2),     # C3: 65536 tiles, 32 per slot x 1024 slots -> 2 launches
    (10, 4, 1 << 20, 128, 256, 1),
    (10, 4, 1 << 20, 2048, 256, 16),   # strong scaling at one GPU
    (10, 4, (1 << 20) + 6, 256, 256, 3),  # a partial tile per fragment
    (4, 2, 64 << 10, 4096, 256, 1),    # C2: 64 per slot
    (4, 2, 64 << 10, 8192, 256, 2),
    (20, 8, 4 << 20, 32, 256, 1),      # C5: the bitsliced kernel
])
def test_bench_dispatches_per_pass(k, width, F, S, cus, want):
    """bench.py's count of stream-kernel launches per pass mirrors launch_stream_pass
    (ecamd_device.hip): at most 32 (4-output) / 64 tiles of 256 lanes x 16 B per resident
    workgroup (4 per CU) per launch."""
    sys.path.insert(0, ROOT)
    import bench
    assert bench.dispatches_per_pass(k, width, F, S, cus) == want


def test_ranks_sharing_a_gpu_fail_loudly():
    """Two ranks on one GPU while the host shows a GPU per rank: the device check (identities
    all-gathered over gloo before any RCCL collective) stops the job and names the ranks."""
    r = run_bench("--gpus", "2", "--dry-run",
                  env={"ECAMD_FAKE_DEVICES": "0,0", "ECAMD_FAKE_DEVICE_COUNT": "8"})
    assert r.returncode != 0
    assert "ranks 0, 1 on GPU" in r.stderr and "8 GPUs for 2 ranks" in r.stderr


def test_distinct_devices_reported():
    r = run_bench("--gpus", "2", "--dry-run", "--no-cpu-baseline",
                  env={"ECAMD_FAKE_DEVICES": "0,1", "ECAMD_FAKE_DEVICE_COUNT": "8"})
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["coord_backend"] == "gloo" and not line["shared_devices"]
    assert [d["device"] for d in line["devices"]] == [0, 1]
    assert len({d["pci"] for d in line["devices"]}) == 2


def _ident(dev, count, host=1, bus=None):
    return {"host": host, "device": dev, "pci_domain": 0, "pci_bus": 0x40 + dev if bus is None else bus,
            "pci_device": 0, "device_count": count, "local_rank": 0}


def test_check_devices_rules():
    sys.path.insert(0, ROOT)
    from liberasurecode_amd.shard import DeviceCollision, check_devices
    # one GPU each: fine on either backend
    assert check_devices([_ident(d, 8) for d in range(8)], "nccl") is False
    # same PCI address under different indices (e.g. two HIP_VISIBLE_DEVICES views) is a collision
    with pytest.raises(DeviceCollision, match="ranks 0, 1"):
        check_devices([_ident(0, 8, bus=0x40), _ident(1, 8, bus=0x40)], "nccl")
    # fewer GPUs than ranks: a gloo rehearsal is allowed and reported, RCCL is refused
    assert check_devices([_ident(0, 1), _ident(0, 1)], "gloo") is True
    with pytest.raises(DeviceCollision, match="RCCL needs one GPU per rank"):
        check_devices([_ident(0, 1), _ident(0, 1)], "nccl")
    # the same device index on two hosts is two GPUs
    assert check_devices([_ident(0, 1, host=1), _ident(0, 1, host=2)], "nccl") is False
    # unknown PCI address: fall back to the device index
    assert check_devices([_ident(0, 8, bus=-1), _ident(1, 8, bus=-1)], "nccl") is False
    with pytest.raises(DeviceCollision, match="index 3"):
        check_devices([_ident(3, 8, bus=-1), _ident(3, 8, bus=-1)], "gloo")
