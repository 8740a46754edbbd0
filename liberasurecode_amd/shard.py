"""Multi-GPU sharding of independent stripes (one process per GPU).

Stripes have no cross-stripe dependency (each liberasurecode_encode call is self-contained,
src/erasurecode.c:383-477), so a job of N GPUs is N independent shards: rank r owns stripes
[r*S, (r+1)*S) (weak scaling, S per GPU).  The process group carries no fragment data; it is used
for a start barrier and for reducing elapsed times / counters.

On GPUs the process group is "cpu:gloo,cuda:nccl": before the first RCCL collective every rank's
device identity (host, device index, PCI domain:bus:device) is all-gathered over gloo and the job
fails loudly, naming the ranks, when two ranks of one host landed on the same GPU although the host
shows enough GPUs for one each (`check_devices`).  RCCL is initialised by its first collective,
bounded by a watchdog (`ECAMD_RCCL_INIT_TIMEOUT`, default 180 s) that exits the process with a
message instead of hanging -- no retry, no re-exec.
"""
import os
import sys
import threading
import zlib

# device identity vector exchanged over gloo: host hash, device index, PCI domain, bus, device,
# visible device count, local rank
_ID_FIELDS = ("host", "device", "pci_domain", "pci_bus", "pci_device", "device_count", "local_rank")


def stripe_range(rank: int, world: int, per_rank: int):
    """(first stripe id, count) owned by `rank` under weak scaling."""
    if not (0 <= rank < world) or per_rank < 0:
        raise ValueError("bad shard request")
    return rank * per_rank, per_rank


def split_range(rank: int, world: int, total: int):
    """(first, count) of a fixed total split as evenly as possible (strong scaling)."""
    if not (0 <= rank < world) or total < 0:
        raise ValueError("bad shard request")
    base, extra = divmod(total, world)
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


def percall_devices_spec(device):
    """ECAMD_PERCALL_DEVICES value that pins a rank's per-call host-buffer path (hostio.cpp) to
    its own GPU: the device index itself."""
    if device is None or int(device) < 0:
        raise ValueError("a rank without a GPU has no per-call device")
    return str(int(device))


class DeviceCollision(RuntimeError):
    """Two ranks of one host were placed on the same GPU."""


def pci_string(ident):
    return "%04x:%02x:%02x" % (ident["pci_domain"], ident["pci_bus"], ident["pci_device"])


def check_devices(idents, backend):
    """Validate the per-rank device identities (one dict per rank, in rank order, fields
    _ID_FIELDS).  Ranks of one host sharing a GPU -- same PCI address, or same device index when
    the PCI address is unknown (-1) -- raise DeviceCollision naming them when that host shows at
    least as many GPUs as it has ranks (a placement bug: the scaling numbers would be wrong) or
    when RCCL is the backend (RCCL refuses it).  With fewer GPUs than ranks on gloo the sharing is
    a rehearsal and is reported.  Returns True when some GPU is shared."""
    by_host = {}
    for rank, ident in enumerate(idents):
        by_host.setdefault(ident["host"], []).append(rank)
    shared = False
    for host, ranks in by_host.items():
        seen = {}
        for r in ranks:
            ident = idents[r]
            if ident["device"] < 0:
                continue  # a rank without a GPU (CPU dry run)
            key = (pci_string(ident) if ident["pci_bus"] >= 0 else "index %d" % ident["device"])
            seen.setdefault(key, []).append(r)
        dups = sorted((v, k) for k, v in seen.items() if len(v) > 1)
        if not dups:
            continue
        shared = True
        ndev = min(idents[r]["device_count"] for r in ranks)
        desc = "; ".join("ranks %s on GPU %s (device %d)" % (
            ", ".join(str(r) for r in v), k, idents[v[0]]["device"]) for v, k in dups)
        if ndev >= len(ranks):
            raise DeviceCollision(
                "device placement: %s -- the host shows %d GPUs for %d ranks, so every rank must "
                "own one (check LOCAL_RANK / HIP_VISIBLE_DEVICES)" % (desc, ndev, len(ranks)))
        if backend != "gloo":
            raise DeviceCollision(
                "device placement: %s -- %d GPUs for %d ranks; RCCL needs one GPU per rank "
                "(a shared-GPU rehearsal must use ECAMD_DIST_BACKEND=gloo)" % (desc, ndev, len(ranks)))
    return shared


def _fake_identity(local, world):
    """CPU dry runs: ECAMD_FAKE_DEVICES="d0,d1,..." (device index per local rank) and
    ECAMD_FAKE_DEVICE_COUNT stand in for the GPUs a real run would see (tests only)."""
    spec = os.environ.get("ECAMD_FAKE_DEVICES")
    if not spec:
        return None
    devs = [int(x) for x in spec.split(",")]
    dev = devs[local % len(devs)]
    count = int(os.environ.get("ECAMD_FAKE_DEVICE_COUNT", str(max(devs) + 1)))
    return {"device": dev, "pci_domain": 0, "pci_bus": 0x10 + dev, "pci_device": 0,
            "device_count": count, "name": "fake"}


class Coordinator:
    """Launch coordination over torch.distributed (RCCL when on GPUs, gloo on CPU)."""

    def __init__(self, backend=None, timeout_s=None):
        import datetime

        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.on_gpu = False
        self.device = None
        self.shared_devices = False
        ident = {"device": -1, "pci_domain": -1, "pci_bus": -1, "pci_device": -1,
                 "device_count": 0, "name": None}
        if torch.cuda.is_available() and torch.cuda.device_count() > 0:
            # one GPU per rank; ranks beyond the visible GPUs share them (gloo rehearsal only,
            # check_devices refuses it otherwise)
            ndev = torch.cuda.device_count()
            self.device = self.local % ndev
            torch.cuda.set_device(self.device)
            p = torch.cuda.get_device_properties(self.device)
            ident = {"device": self.device, "pci_domain": int(p.pci_domain_id),
                     "pci_bus": int(p.pci_bus_id), "pci_device": int(p.pci_device_id),
                     "device_count": ndev, "name": p.name}
            # the per-call host-buffer path (hostio.cpp) stays on this rank's GPU, whichever
            # thread of the rank calls it (an explicit index: a worker thread's current device
            # would be device 0)
            os.environ.setdefault("ECAMD_PERCALL_DEVICES", percall_devices_spec(self.device))
        fake = _fake_identity(self.local, self.world)
        if fake is not None:
            ident = fake
        self.identity = dict(ident, host=os.environ.get("ECAMD_FAKE_HOST") or _hostname(),
                             local_rank=self.local, rank=self.rank)
        self.devices = [self._public(self.identity)]
        self.coord_backend = None
        if self.world > 1:
            backend = backend or os.environ.get("ECAMD_DIST_BACKEND")
            if backend is None:
                backend = "nccl" if torch.cuda.is_available() else "gloo"
            self.on_gpu = backend == "nccl"
            tmo = datetime.timedelta(seconds=float(timeout_s or os.environ.get(
                "ECAMD_DIST_TIMEOUT", "600")))
            # RCCL is created lazily by the first CUDA collective (no device_id here), so the
            # device check below runs over gloo before any RCCL communicator exists
            self.coord_backend = "cpu:gloo,cuda:nccl" if self.on_gpu else backend
            dist.init_process_group(backend=self.coord_backend, timeout=tmo)
            idents = self._gather_identities()
            self.devices = [self._public(i) for i in idents]
            try:
                self.shared_devices = check_devices(idents, backend)
            except DeviceCollision as e:
                sys.stderr.write("bench rank %d: %s\n" % (self.rank, e))
                sys.stderr.flush()
                raise
            if self.on_gpu:
                self._init_rccl()

    @staticmethod
    def _public(ident):
        out = {"rank": ident.get("rank", 0), "local_rank": ident["local_rank"],
               "device": ident["device"], "device_count": ident["device_count"]}
        if ident["pci_bus"] >= 0:
            out["pci"] = pci_string(ident)
        if ident.get("name"):
            out["name"] = ident["name"]
        return out

    def _gather_identities(self):
        """All-gather every rank's identity vector over gloo (CPU tensors)."""
        torch = self.torch
        mine = self.identity
        vec = torch.tensor([zlib.crc32(mine["host"].encode()), mine["device"], mine["pci_domain"],
                            mine["pci_bus"], mine["pci_device"], mine["device_count"],
                            mine["local_rank"]], dtype=torch.int64)
        bufs = [torch.zeros_like(vec) for _ in range(self.world)]
        self.dist.all_gather(bufs, vec)
        out = []
        for r, b in enumerate(bufs):
            d = dict(zip(_ID_FIELDS, (int(x) for x in b.tolist())))
            d["rank"] = r
            d["name"] = mine["name"] if r == self.rank else None
            out.append(d)
        return out

    def _init_rccl(self):
        """First RCCL collective (communicator creation) under a watchdog: a rank that cannot
        join within ECAMD_RCCL_INIT_TIMEOUT seconds exits non-zero with a message."""
        limit = float(os.environ.get("ECAMD_RCCL_INIT_TIMEOUT", "180"))

        def expire():
            sys.stderr.write("bench rank %d: RCCL communicator not up after %.0f s (device %s); "
                             "exiting\n" % (self.rank, limit, self.device))
            sys.stderr.flush()
            os._exit(3)

        timer = threading.Timer(limit, expire)
        timer.daemon = True
        timer.start()
        try:
            t = self.torch.ones(1, device="cuda")
            self.dist.all_reduce(t)
            self.torch.cuda.synchronize()
            if int(t.item()) != self.world:
                raise RuntimeError("RCCL all-reduce returned %s, expected %d" % (t.item(), self.world))
        finally:
            timer.cancel()

    def _tensor(self, values):
        dev = "cuda" if self.on_gpu else "cpu"
        return self.torch.tensor(values, dtype=self.torch.float64, device=dev)

    def barrier(self):
        if self.world == 1:
            return
        if self.on_gpu:  # RCCL: a one-element all-reduce, complete on return
            t = self._tensor([0.0])
            self.dist.all_reduce(t)
            self.torch.cuda.synchronize()
        else:
            self.dist.barrier()

    def cpu_barrier(self):
        """Barrier over gloo (a CPU tensor, also under "cpu:gloo,cuda:nccl"): ranks waiting here
        block in a socket read rather than in a GPU synchronize, e.g. while rank 0 times the
        host-CPU baseline on the cores they share."""
        if self.world == 1:
            return
        t = self.torch.zeros(1, dtype=self.torch.float64)
        self.dist.all_reduce(t)

    def per_rank(self, value):
        """Every rank's `value` (a float), in rank order, on every rank."""
        v = [float(value) if r == self.rank else 0.0 for r in range(self.world)]
        return self.reduce(v, op="sum")

    def reduce(self, values, op="max"):
        """All-reduce a list of floats (max or sum); identity when world == 1."""
        values = list(values)
        if self.world == 1:
            return values
        t = self._tensor(values)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX if op == "max" else self.dist.ReduceOp.SUM)
        return [float(v) for v in t.cpu().tolist()]

    def close(self):
        if self.world > 1:
            self.dist.destroy_process_group()


def _hostname():
    import socket
    return socket.gethostname()
