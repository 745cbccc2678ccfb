"""Process-per-GPU sharded prove.

Each of the G processes (torch.distributed.run, one per GPU) owns one
Context; a communicator is attached to it and every rank calls
``prove_sharded`` with the same trace.  The proof is byte-identical to
``Context.prove`` (see prove_shard in csrc/prove.cpp for what each rank owns
and what is exchanged).

Two transports:
  * ``attach_rccl``  device-direct RCCL over xGMI (the 8-GPU path); the
    128-byte unique id travels over the torch.distributed control group.
    Import this module before the first Context is created: it loads torch
    first so that liblsp_hip, torch and RCCL share one HIP/HSA runtime.
  * ``GlooComm``     the caller-transport interface (lsp_comm_ops) backed by a
    torch.distributed gloo group on host buffers: slower (device data is
    staged through host memory), but it needs no GPU per rank, so several
    ranks can share one GPU -- how the multi-process path is tested here.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import numpy as np
import torch  # before liblsp_hip.so loads: one HIP/HSA runtime (torch's) serves the process

# RCCL built against that runtime (comm_ext.cpp reads LSP_RCCL_LIB first)
_TORCH_RCCL = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
if os.path.exists(_TORCH_RCCL):
    os.environ.setdefault("LSP_RCCL_LIB", _TORCH_RCCL)

from . import _lib as L
from .air import LineaAIR
from .prover import Context, _fr_arr, _ptr, _take_proof


class GlooComm:
    """lsp_comm_ops over a torch.distributed process group (host tensors)."""

    def __init__(self, group=None):
        import torch.distributed as dist
        if not dist.is_initialized():
            raise RuntimeError("GlooComm needs an initialised torch.distributed process group")
        self.dist, self.group = dist, group
        self.rank, self.size = dist.get_rank(group), dist.get_world_size(group)
        self.error: Optional[BaseException] = None
        # every collective the library issued through this communicator, in
        # order: (op, bytes per rank, root) -- identical on every rank, or a
        # collective transport (RCCL) would deadlock (tests/test_gpu_shard_mp.py)
        self.schedule = []
        self._ag = L.ALLGATHER_FN(self._allgather)
        self._bc = L.BCAST_FN(self._bcast)
        self.ops = L.LspCommOps(self.rank, self.size, None, self._ag, self._bc)

    @staticmethod
    def _view(ptr, nbytes):
        return np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(ptr))

    def _allgather(self, _user, send, recv, nbytes):
        self.schedule.append(("allgather", int(nbytes), None))
        try:
            src = torch.from_numpy(self._view(send, nbytes).copy())
            parts = [torch.empty(nbytes, dtype=torch.uint8) for _ in range(self.size)]
            self.dist.all_gather(parts, src, group=self.group)
            out = self._view(recv, nbytes * self.size)
            for r, t in enumerate(parts):
                out[r * nbytes:(r + 1) * nbytes] = t.numpy()
            return 0
        except BaseException as e:  # the C side turns non-zero into LSP_E_STATE
            self.error = e
            return 1

    def _bcast(self, _user, buf, nbytes, root):
        self.schedule.append(("bcast", int(nbytes), int(root)))
        try:
            v = self._view(buf, nbytes)
            t = torch.from_numpy(v.copy())
            self.dist.broadcast(t, src=self.dist.get_global_rank(self.group, root) if self.group else root,
                                group=self.group)
            v[:] = t.numpy()
            return 0
        except BaseException as e:
            self.error = e
            return 1

    def attach(self, ctx: Context) -> "GlooComm":
        L.check(L.lib().lsp_ctx_attach_comm_ops(ctx.h, ctypes.byref(self.ops)), ctx.h)
        ctx._comm = self  # keep the callbacks alive as long as the context
        selftest(ctx)
        return self


def attach_rccl(ctx: Context, group=None) -> None:
    """Collective: every rank of `group` attaches an RCCL communicator to its
    context (rank 0 makes the id, the control group broadcasts it)."""
    import torch.distributed as dist
    single = not dist.is_initialized()  # a world of one: nothing to distribute
    rank, size = (0, 1) if single else (dist.get_rank(group), dist.get_world_size(group))
    uid = (ctypes.c_uint8 * 128)()
    if rank == 0:
        L.check(L.lib().lsp_comm_rccl_unique_id(uid))
    if not single:
        obj = [bytes(uid)]
        dist.broadcast_object_list(obj, src=dist.get_global_rank(group, 0) if group else 0, group=group)
        uid = (ctypes.c_uint8 * 128).from_buffer_copy(obj[0])
    L.check(L.lib().lsp_ctx_attach_rccl(ctx.h, uid, rank, size), ctx.h)
    selftest(ctx)


def selftest(ctx: Context) -> None:
    """collective: allgather + broadcast of known patterns through the attached communicator"""
    rc = L.lib().lsp_comm_selftest(ctx.h)
    comm = getattr(ctx, "_comm", None)
    if rc != L.LSP_OK and comm is not None and comm.error is not None:
        raise RuntimeError(f"communicator failed: {comm.error!r}") from comm.error
    ctx._chk(rc)


def detach(ctx: Context) -> None:
    L.check(L.lib().lsp_ctx_detach_comm(ctx.h), ctx.h)
    ctx._comm = None


def prove_sharded(ctx: Context, trace, air: LineaAIR, public_values: np.ndarray, h: Optional[int] = None,
                  w: Optional[int] = None, size_only: bool = False):
    """This rank's part of a sharded proof; every rank returns the whole proof.
    `trace`: (h, w, 4) host array or a device pointer (int) with h and w.
    size_only: return the proof's wire size instead (a rehearsal proof under
    lsp_ctx_attach_loopback answers nothing else)."""
    desc = (ctypes.c_int32 * len(air.descriptor()))(*air.descriptor())
    pub = _fr_arr(public_values).reshape(-1, 4)
    proof = ctypes.c_void_p()
    if isinstance(trace, int):
        rc = L.lib().lsp_prove_sharded(ctx.h, trace, h, w, desc, len(desc), _ptr(pub), pub.shape[0],
                                       L.LSP_MEM_DEVICE, ctypes.byref(proof))
    else:
        t = _fr_arr(trace)
        rc = L.lib().lsp_prove_sharded(ctx.h, _ptr(t), t.shape[0], t.shape[1], desc, len(desc), _ptr(pub),
                                       pub.shape[0], L.LSP_MEM_HOST, ctypes.byref(proof))
    comm = getattr(ctx, "_comm", None)
    if rc != L.LSP_OK and comm is not None and comm.error is not None:
        raise RuntimeError(f"communicator failed: {comm.error!r}") from comm.error
    ctx._chk(rc)
    return _take_proof(proof, size_only)
