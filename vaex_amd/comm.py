"""Inter-process communication for the multi-GPU path, without PyTorch.

One process per GPU.  Two communicators with the same interface:

* :class:`RcclComm` -- the product path: RCCL bound by ``libvaexhip`` itself
  (``vh_comm_*``, ``csrc/comm.hip``).  Grids and groupby partitions are reduced /
  exchanged on HBM buffers over xGMI; small host values (limits, flags, set key arrays)
  go through the same communicator with host staging.
* :class:`HostComm` -- a CPU exchange over TCP (a star through rank 0).  It carries RCCL's
  unique id to the other ranks before ``vh_comm_init``, and it is the CPU fake the
  multi-process tests run the SAME exchange code on (no GPU needed); several ranks
  sharing one GPU (RCCL refuses two ranks on one device) use it too.
* :class:`LoopbackComm` -- N virtual ranks in one process on one GPU (threads), the
  library's loopback communicator (``vh_comm_loopback``): the device-side multi-rank code
  of :class:`RcclComm` runs with N ranks' data where only one GPU exists (tests).

Rendezvous: ``RANK`` / ``WORLD_SIZE`` / ``MASTER_ADDR`` from the environment (what
``torch.distributed.run`` exports); the host channel listens on ``VAEX_AMD_COMM_PORT``, or
``MASTER_PORT + 1`` (the launcher's own store holds ``MASTER_PORT``).

Messages use a small self-describing encoding of None / bool / int / float / str / bytes /
numpy arrays / lists / tuples / dicts -- nothing is unpickled.
"""
import os
import socket
import struct
import time

import numpy as np

OPS = {"sum": 0, "min": 1, "max": 2}


# ---- message encoding ------------------------------------------------------------------
def _enc(obj, out):
    if obj is None:
        out.append(b"N")
    elif isinstance(obj, (bool, np.bool_)):
        out.append(b"B" + (b"\x01" if obj else b"\x00"))
    elif isinstance(obj, (int, np.integer)) and -(1 << 63) <= int(obj) < (1 << 63):
        out.append(b"I" + struct.pack("<q", int(obj)))
    elif isinstance(obj, (float, np.floating)):
        out.append(b"F" + struct.pack("<d", float(obj)))
    elif isinstance(obj, str):
        b = obj.encode()
        out.append(b"S" + struct.pack("<Q", len(b)) + b)
    elif isinstance(obj, (bytes, bytearray)):
        out.append(b"Y" + struct.pack("<Q", len(obj)) + bytes(obj))
    elif isinstance(obj, np.ndarray):
        a = np.ascontiguousarray(obj)
        dt = a.dtype.str.encode()
        out.append(b"A" + struct.pack("<Q", len(dt)) + dt + struct.pack("<Q", a.ndim)
                   + struct.pack(f"<{a.ndim}Q", *a.shape) + struct.pack("<Q", a.nbytes))
        out.append(a.tobytes())
    elif isinstance(obj, (list, tuple)):
        out.append((b"L" if isinstance(obj, list) else b"T") + struct.pack("<Q", len(obj)))
        for o in obj:
            _enc(o, out)
    elif isinstance(obj, dict):
        out.append(b"D" + struct.pack("<Q", len(obj)))
        for k, v in obj.items():
            _enc(k, out)
            _enc(v, out)
    else:
        raise TypeError(f"cannot send {type(obj).__name__}")


def encode(obj):
    out = []
    _enc(obj, out)
    return b"".join(out)


def _dec(buf, at):
    tag = buf[at:at + 1]
    at += 1
    if tag == b"N":
        return None, at
    if tag == b"B":
        return buf[at] != 0, at + 1
    if tag == b"I":
        return struct.unpack_from("<q", buf, at)[0], at + 8
    if tag == b"F":
        return struct.unpack_from("<d", buf, at)[0], at + 8
    if tag in (b"S", b"Y"):
        n = struct.unpack_from("<Q", buf, at)[0]
        at += 8
        b = bytes(buf[at:at + n])
        return (b.decode() if tag == b"S" else b), at + n
    if tag == b"A":
        n = struct.unpack_from("<Q", buf, at)[0]
        at += 8
        dt = np.dtype(bytes(buf[at:at + n]).decode())
        at += n
        nd = struct.unpack_from("<Q", buf, at)[0]
        at += 8
        shape = struct.unpack_from(f"<{nd}Q", buf, at)
        at += 8 * nd
        nb = struct.unpack_from("<Q", buf, at)[0]
        at += 8
        a = np.frombuffer(bytes(buf[at:at + nb]), dtype=dt).reshape(shape).copy()
        return a, at + nb
    if tag in (b"L", b"T"):
        n = struct.unpack_from("<Q", buf, at)[0]
        at += 8
        items = []
        for _ in range(n):
            o, at = _dec(buf, at)
            items.append(o)
        return (items if tag == b"L" else tuple(items)), at
    if tag == b"D":
        n = struct.unpack_from("<Q", buf, at)[0]
        at += 8
        d = {}
        for _ in range(n):
            k, at = _dec(buf, at)
            v, at = _dec(buf, at)
            d[k] = v
        return d, at
    raise ValueError(f"bad message tag {tag!r}")


def decode(buf):
    obj, at = _dec(memoryview(buf), 0)
    if at != len(buf):
        raise ValueError("trailing bytes in message")
    return obj


def reduce_arrays(arrays, op):
    """Fold per-rank arrays in rank order (the reduce order of parts[0].reduce(parts[1:]))."""
    out = np.array(arrays[0], copy=True)
    for a in arrays[1:]:
        if op == "sum":
            out = out + a
        elif op == "min":
            out = np.where(a < out, a, out)
        elif op == "max":
            out = np.where(out < a, a, out)
        else:
            raise ValueError(op)
    return out.astype(np.asarray(arrays[0]).dtype, copy=False)


# ---- host channel -------------------------------------------------------------------------
def _recv_exact(sock, n):
    buf = bytearray(n)
    view = memoryview(buf)
    got = 0
    while got < n:
        k = sock.recv_into(view[got:], n - got)
        if not k:
            raise ConnectionError("peer closed the communicator")
        got += k
    return buf


def _send_msg(sock, obj):
    payload = encode(obj)
    sock.sendall(struct.pack("<Q", len(payload)) + payload)


def _recv_msg(sock):
    n = struct.unpack("<Q", bytes(_recv_exact(sock, 8)))[0]
    return decode(_recv_exact(sock, n))


class HostComm:
    """Collectives through host memory: a TCP star, rank 0 in the middle.  Results are the
    same on every rank, reductions fold in rank order."""

    device = False
    backend = "host"

    def __init__(self, rank, world, addr="127.0.0.1", port=29511, timeout=600.0):
        self.rank, self.world = int(rank), int(world)
        self._peers = {}
        self._sock = None
        if self.world == 1:
            return
        deadline = time.time() + timeout
        if self.rank == 0:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            srv.bind((addr, port))
            srv.listen(self.world)
            srv.settimeout(max(1.0, deadline - time.time()))
            try:
                while len(self._peers) < self.world - 1:
                    conn, _ = srv.accept()
                    conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                    conn.settimeout(None)
                    r = struct.unpack("<q", bytes(_recv_exact(conn, 8)))[0]
                    self._peers[r] = conn
            finally:
                srv.close()
        else:
            while True:
                try:
                    s = socket.create_connection((addr, port), timeout=5.0)
                    break
                except OSError:
                    if time.time() > deadline:
                        raise
                    time.sleep(0.05)
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            s.settimeout(None)
            s.sendall(struct.pack("<q", self.rank))
            self._sock = s

    # ---- primitives (every rank calls them in the same order) ----
    def gather(self, obj):
        """Rank 0: [obj of rank 0, 1, ...]; other ranks: None."""
        if self.world == 1:
            return [obj]
        if self.rank == 0:
            return [obj] + [_recv_msg(self._peers[r]) for r in range(1, self.world)]
        _send_msg(self._sock, obj)
        return None

    def bcast(self, obj=None):
        """Rank 0's obj on every rank."""
        if self.world == 1:
            return obj
        if self.rank == 0:
            for r in range(1, self.world):
                _send_msg(self._peers[r], obj)
            return obj
        return _recv_msg(self._sock)

    def allgather(self, obj):
        return self.bcast(self.gather(obj))

    def alltoall(self, objs):
        """objs[d] goes to rank d; returns [what rank s sent me for s in ranks]."""
        if len(objs) != self.world:
            raise ValueError("alltoall needs one item per rank")
        if self.world == 1:
            return [objs[0]]
        allv = self.gather(list(objs))
        if self.rank == 0:
            for d in range(1, self.world):
                _send_msg(self._peers[d], [allv[s][d] for s in range(self.world)])
            return [allv[s][0] for s in range(self.world)]
        return _recv_msg(self._sock)

    def allreduce(self, arr, op="sum"):
        """numpy array (or scalar) reduced over the ranks; returns the result."""
        a = np.asarray(arr)
        return reduce_arrays(self.allgather(a), op)

    def barrier(self):
        self.allgather(None)

    def close(self):
        for s in list(self._peers.values()) + ([self._sock] if self._sock else []):
            try:
                s.close()
            except OSError:
                pass
        self._peers, self._sock = {}, None


class ThreadComm:
    """Host collectives among the threads of one process (the object channel of a
    loopback group, :func:`loopback_group`): same interface and results as
    :class:`HostComm`, every rank a thread."""

    device = False
    backend = "threads"

    class Group:
        def __init__(self, world, timeout=120.0):
            import threading
            self.world = world
            self.barrier = threading.Barrier(world, timeout=timeout)
            self.slots = [None] * world

    def __init__(self, rank, group):
        self.rank, self.world = int(rank), group.world
        self._g = group

    def _exchange(self, obj):
        g = self._g
        g.slots[self.rank] = obj
        g.barrier.wait()
        got = list(g.slots)
        g.barrier.wait()  # slots are reused by the next call
        return got

    def gather(self, obj):
        got = self._exchange(obj)
        return got if self.rank == 0 else None

    def bcast(self, obj=None):
        return self._exchange(obj if self.rank == 0 else None)[0]

    def allgather(self, obj):
        return self._exchange(obj)

    def alltoall(self, objs):
        if len(objs) != self.world:
            raise ValueError("alltoall needs one item per rank")
        got = self._exchange(list(objs))
        return [got[s][self.rank] for s in range(self.world)]

    def allreduce(self, arr, op="sum"):
        return reduce_arrays(self.allgather(np.asarray(arr)), op)

    def barrier(self):
        self._exchange(None)

    def close(self):
        pass


class DeviceComm:
    """A libvaexhip communicator (``vh_comm_*``): device collectives on the library stream
    -- in-place grid all-reduce, the groupby partition exchange.  Object exchange (key
    arrays, flags) rides the host channel ``host``."""

    device = True
    backend = "device"

    def __init__(self, host, handle):
        from . import _lib
        self._lib = _lib
        self.host = host
        self.rank, self.world = host.rank, host.world
        self._h = handle

    @property
    def handle(self):
        return self._h

    def allreduce(self, arr, op="sum"):
        a = np.array(arr, copy=True)
        flat = np.ascontiguousarray(a.reshape(-1))
        code, _ = self._lib.dtype_code(flat.dtype)
        self._lib.call("vh_comm_allreduce", self._h, flat.ctypes.data, flat.size, code, OPS[op], self._lib.LOC_HOST)
        return flat.reshape(a.shape)

    def allreduce_device(self, ptr, count, dtype, op="sum"):
        code, _ = self._lib.dtype_code(dtype)
        self._lib.call("vh_comm_allreduce", self._h, ptr, count, code, OPS[op], self._lib.LOC_DEVICE)

    def agg_allreduce(self, agg):
        self._lib.call("vh_comm_agg_allreduce", self._h, agg._handle)

    def gather(self, obj):
        return self.host.gather(obj)

    def bcast(self, obj=None):
        return self.host.bcast(obj)

    def allgather(self, obj):
        return self.host.allgather(obj)

    def alltoall(self, objs):
        return self.host.alltoall(objs)

    def barrier(self):
        self._lib.call("vh_comm_barrier", self._h)

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.call("vh_comm_destroy", self._h)
            self._h = None
        self.host.close()


class RcclComm(DeviceComm):
    """RCCL through libvaexhip: one process per GPU, rank 0's unique id sent to the other
    ranks over the host channel, then ``vh_comm_init`` on this process's GPU."""

    backend = "rccl"

    def __init__(self, host):
        import ctypes
        from . import _lib
        uid = ctypes.create_string_buffer(128)
        if host.rank == 0:
            _lib.call("vh_comm_unique_id", uid)
        raw = host.bcast(uid.raw if host.rank == 0 else None)
        ctypes.memmove(uid, raw, 128)
        h = ctypes.c_void_p()
        _lib.call("vh_comm_init", uid, host.world, host.rank, ctypes.byref(h))
        super().__init__(host, h)


class LoopbackComm(DeviceComm):
    """One virtual rank of a loopback group (``vh_comm_loopback``): N ranks in one process on
    one GPU, one thread per rank.  The collectives are device copies and rank-order device
    folds behind the same C-ABI as RCCL's, so the multi-rank device code (grid all-reduce
    folds, AggFirst across ranks, the groupby all-to-all and its fold) runs with N ranks'
    data on a one-GPU box."""

    backend = "loopback"


def loopback_group(world):
    """``world`` :class:`LoopbackComm` ranks of this process (use each from its own thread)."""
    import ctypes
    from . import _lib
    hs = (ctypes.c_void_p * world)()
    _lib.call("vh_comm_loopback", int(world), hs)
    group = ThreadComm.Group(world)
    return [LoopbackComm(ThreadComm(r, group), ctypes.c_void_p(hs[r])) for r in range(world)]


def select_device(local_rank=None):
    """Make GPU ``LOCAL_RANK`` (mod the device count) this process's device -- for every
    thread of the process (vh_set_device): one process per GPU under torch.distributed.run.
    Returns the device, or None without a GPU."""
    from . import _lib
    n = _lib.device_count()
    if n < 1:
        return None
    lr = _env_int("LOCAL_RANK", 0) if local_rank is None else int(local_rank)
    dev = lr % n
    _lib.call("vh_set_device", dev)
    return dev


_default = None


def _env_int(name, default):
    v = os.environ.get(name)
    return int(v) if v not in (None, "") else default


def init(backend="auto", rank=None, world=None, addr=None, port=None, timeout=600.0):
    """Create this process's communicator (and make it the default).  backend: "rccl"
    (GPU collectives), "host" (CPU exchange), "auto" = rccl when the HIP library sees a GPU."""
    global _default
    rank = _env_int("RANK", 0) if rank is None else rank
    world = _env_int("WORLD_SIZE", 1) if world is None else world
    addr = addr or os.environ.get("MASTER_ADDR", "127.0.0.1")
    if port is None:
        port = _env_int("VAEX_AMD_COMM_PORT", 0) or (_env_int("MASTER_PORT", 29510) + 1)
    if backend in ("auto", "rccl"):
        # the GPU is chosen before any other GPU call: every rank on device 0 would make
        # RCCL refuse the duplicate device
        dev = select_device()
        if backend == "auto":
            backend = "rccl" if dev is not None else "host"
    host = HostComm(rank, world, addr, port, timeout)
    _default = RcclComm(host) if backend == "rccl" else host
    return _default


def get():
    if _default is None:
        raise RuntimeError("no communicator: call vaex_amd.comm.init() in every rank first")
    return _default


def shutdown():
    global _default
    if _default is not None:
        _default.close()
        _default = None
