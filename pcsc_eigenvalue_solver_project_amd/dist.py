"""Row-sharded power iteration across GPUs (one process per GPU, RCCL over xGMI).

Python view of ``eigsol_ctx_create_dist`` / ``eigsol_csr_create_dist`` (include/eigsol_hip.h).
The communicator is owned by the C++ library; ``torch.distributed`` (any backend) is only used to
broadcast RCCL's 128-byte unique id at start-up.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import CsrMatrix, Context, EigSolError, PowerSession, _dtype_code, _np_dtype, _ptr
from ._capi import call, lib


def ghost_plan(nranks: int, row_begins, rank: int, colidx_global):
    """Host-only remap of global columns to the local x-space (library function, no device)."""
    rb = np.ascontiguousarray(row_begins, dtype=np.int64)
    cg = np.ascontiguousarray(colidx_global, dtype=np.int32)
    cl = np.empty(max(len(cg), 1), dtype=np.int32)
    gh = np.empty(max(len(cg), 1), dtype=np.int64)
    rc = np.zeros(nranks, dtype=np.int64)
    ng = C.c_int64(0)
    call("eigsol_ghost_plan", int(nranks), _ptr(rb), int(rank), len(cg), _ptr(cg), _ptr(cl),
         C.byref(ng), _ptr(gh), _ptr(rc))
    return cl[: len(cg)], gh[: ng.value], rc


EXCHANGE_HALO, EXCHANGE_ALLGATHER = 0, 1


def exchange_mode(row_begins, ghost_counts) -> int:
    """The x exchange eigsol_csr_create_dist selects from the P x P ghost counts
    (``ghost_counts[r, q]`` = entries rank r reads from rank q); library function, no device."""
    rb = np.ascontiguousarray(row_begins, dtype=np.int64)
    gc = np.ascontiguousarray(ghost_counts, dtype=np.int64)
    m = C.c_int(0)
    call("eigsol_exchange_mode", len(rb) - 1, _ptr(rb), _ptr(gc), C.byref(m))
    return m.value


class DistContext(Context):
    """A Context whose communicator spans one rank per GPU."""

    def __init__(self, device: int, rank: int, world: int, unique_id: bytes, stream=None):
        h = C.c_void_p()
        uid = (C.c_char * len(unique_id)).from_buffer_copy(unique_id)
        call("eigsol_ctx_create_dist", int(device), int(rank), int(world), C.cast(uid, C.c_void_p), C.byref(h))
        self.handle = h
        self.device = device
        self.rank, self.world = rank, world
        if stream is not None:
            self.set_stream(stream)


def unique_id() -> bytes:
    n = lib().eigsol_dist_unique_id_bytes()
    buf = (C.c_char * n)()
    call("eigsol_dist_get_unique_id", C.cast(buf, C.c_void_p))
    return bytes(buf)


def loopback_id(world: int) -> bytes:
    """Id of an in-process loopback world (tests: ``world`` ranks, one thread each, one device)."""
    n = lib().eigsol_dist_unique_id_bytes()
    buf = (C.c_char * n)()
    call("eigsol_dist_loopback_id", int(world), C.cast(buf, C.c_void_p))
    return bytes(buf)


def peer_plan(nranks: int, rank: int, row_begins, ghost_counts, requests) -> np.ndarray:
    """Host-only push plan of the device-side peer exchange (library function, no device): one row
    {local row, peer, slot in the peer's ghost list, 0} per request, sorted by local row."""
    rb = np.ascontiguousarray(row_begins, dtype=np.int64)
    gc = np.ascontiguousarray(ghost_counts, dtype=np.int64)
    rq = np.ascontiguousarray(requests, dtype=np.int64)
    out = np.zeros((max(len(rq), 1), 4), dtype=np.int32)
    call("eigsol_peer_plan", int(nranks), int(rank), _ptr(rb), _ptr(gc), _ptr(rq), len(rq), _ptr(out))
    return out[: len(rq)]


class HostDistContext(Context):
    """A row-sharded context bootstrapped by a host all-gather (``eigsol_ctx_create_dist_host``):
    no RCCL communicator; setup runs over ``allgather(bytes) -> list[bytes]`` (any host transport,
    e.g. torch.distributed gloo) and the per-iteration exchange is device to device."""

    def __init__(self, device: int, rank: int, world: int, allgather, stream=None):
        from ._capi import ALLGATHER_FN

        def _cb(send, recv, nbytes, _user):
            try:
                mine = C.string_at(send, nbytes)
                parts = allgather(mine)
                if len(parts) != world or any(len(p) != nbytes for p in parts):
                    return 1
                C.memmove(recv, b"".join(parts), nbytes * world)
                return 0
            except Exception:   # noqa: BLE001 - reported to the library as a failed collective
                return 1

        self._cb = ALLGATHER_FN(_cb)   # kept alive as long as the context
        h = C.c_void_p()
        call("eigsol_ctx_create_dist_host", int(device), int(rank), int(world), C.cast(self._cb, C.c_void_p),
             None, C.byref(h))
        self.handle = h
        self.device = device
        self.rank, self.world = rank, world
        if stream is not None:
            self.set_stream(stream)


def torch_host_context(device: int, stream=None) -> HostDistContext:
    """HostDistContext over an initialised torch.distributed process group (gloo: CPU tensors)."""
    import torch
    import torch.distributed as dist
    rank, world = dist.get_rank(), dist.get_world_size()

    def allgather(b: bytes):
        n = len(b)
        mine = torch.frombuffer(bytearray(b), dtype=torch.uint8) if n else torch.zeros(0, dtype=torch.uint8)
        out = [torch.zeros(n, dtype=torch.uint8) for _ in range(world)]
        dist.all_gather(out, mine)
        return [bytes(t.numpy().tobytes()) for t in out]

    return HostDistContext(device, rank, world, allgather, stream=stream)


def torch_dist_context(device: int, stream=None) -> DistContext:
    """Bootstrap from an initialised torch.distributed process group (gloo or nccl)."""
    import torch
    import torch.distributed as dist
    rank, world = dist.get_rank(), dist.get_world_size()
    n = lib().eigsol_dist_unique_id_bytes()
    # byte 0: rank 0 obtained the id (a failure there is reported on every rank instead of leaving
    # the others in the broadcast)
    t = torch.zeros(n + 1, dtype=torch.uint8)
    why = ""
    if rank == 0:
        try:
            t[1:] = torch.frombuffer(bytearray(unique_id()), dtype=torch.uint8)
            t[0] = 1
        except EigSolError as e:
            why = str(e)
    dist.broadcast(t, src=0)
    if int(t[0]) != 1:
        raise EigSolError(8, "RCCL unique id unavailable on rank 0" + (": " + why if why else ""))
    return DistContext(device, rank, world, bytes(t[1:].numpy().tobytes()), stream=stream)


class DistCsrMatrix(CsrMatrix):
    """This rank's row block of a row-sharded CSR matrix (collective construction)."""

    def __init__(self, ctx: DistContext, row_begins, rowptr_local, colidx_global, values):
        values = np.ascontiguousarray(values)
        code = _dtype_code(values.dtype)
        rb = np.ascontiguousarray(row_begins, dtype=np.int64)
        rp = np.ascontiguousarray(rowptr_local, dtype=np.int32)
        cg = np.ascontiguousarray(colidx_global, dtype=np.int32)
        if len(rb) != ctx.world + 1:
            raise EigSolError(9, "row_begins must have world + 1 entries")
        h = C.c_void_p()
        call("eigsol_csr_create_dist", ctx.handle, code, _ptr(rb), len(cg), _ptr(rp), _ptr(cg),
             _ptr(values), C.byref(h))
        self.ctx, self.handle = ctx, h
        nloc = int(rb[ctx.rank + 1] - rb[ctx.rank])
        self.shape = (nloc, int(rb[-1]))
        self.n_global = int(rb[-1])
        self.nnz = len(cg)
        self.dtype = _np_dtype(code)

    @property
    def exchange(self) -> int:
        """EXCHANGE_HALO or EXCHANGE_ALLGATHER (chosen collectively at construction)."""
        m, g = C.c_int(0), C.c_int64(0)
        call("eigsol_csr_dist_info", self.handle, C.byref(m), C.byref(g))
        return m.value


def sharded_power_session(ctx: DistContext, rowptr_local, colidx_global, values, n_global: int,
                          row0: int):
    """Equal contiguous row blocks (rows_per_rank = n_global / world); returns (matrix, session)."""
    world = ctx.world
    rows = n_global // world
    rb = np.arange(world + 1, dtype=np.int64) * rows
    rb[-1] = n_global
    assert rb[ctx.rank] == row0
    A = DistCsrMatrix(ctx, rb, rowptr_local, colidx_global, values)
    return A, PowerSession(A)
