"""Multi-GPU control plane for independent proofs ("replicas").

One process per GPU (launched by torch.distributed.run). Every rank proves its
own trace; the only cross-rank traffic is a barrier before and after the timed
region and a MAX-reduction of the wall time (gloo, CPU tensors). There is no
data-path collective because independent proofs share nothing.

torch is imported before liblsp_hip.so is loaded so that a single HIP runtime
(the one torch ships, same SONAME) serves the process.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass
from typing import Callable, Optional


@dataclass
class Dist:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    pg: Optional[object] = None   # torch.distributed module when world > 1

    def barrier(self):
        if self.pg is not None:
            self.pg.barrier()

    def max(self, x: float) -> float:
        if self.pg is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.pg.all_reduce(t, op=self.pg.ReduceOp.MAX)
        return float(t.item())

    def sum(self, x: float) -> float:
        if self.pg is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.pg.all_reduce(t, op=self.pg.ReduceOp.SUM)
        return float(t.item())

    def all_gather_object(self, obj) -> list:
        """every rank's `obj`, in rank order (the control group; small objects)"""
        if self.pg is None:
            return [obj]
        out = [None] * self.world
        self.pg.all_gather_object(out, obj)
        return out

    def close(self):
        if self.pg is not None:
            self.pg.destroy_process_group()
            self.pg = None


def init_from_env() -> Dist:
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if world <= 1:
        return Dist(rank, world, local, None)
    import torch  # noqa: F401  (before the HIP library: one runtime per process)
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    dist.init_process_group("gloo", init_method="env://", world_size=world, rank=rank)
    d = Dist(rank, world, local, dist)
    share_host_cpus(d)
    return d


def share_host_cpus(d: Dist) -> Optional[int]:
    """Size every rank's host pool from the ranks that really share its CPUs:
    the ranks on this host with the same affinity set split it, a rank with a
    set of its own keeps it (16 threads at most, as the library's default).
    A cgroup CPU quota is not divided: eight ranks on one box's 16-CPU quota
    ran no faster with strict 2-thread shares (8.26 M rows/s) than with
    16-thread pools each (8.40-8.65 M; profiles/r05r_*, r05z*_*) -- the
    pools' work is bursty latency chains that rarely coincide.
    The library alone can only guess from LOCAL_WORLD_SIZE whether a small
    set is shared or this rank's slice (host.cpp default_host_threads); here
    the ranks compare their sets over the control group and export
    LSP_HOST_THREADS before any context exists.  An LSP_HOST_THREADS the
    caller set wins.  Returns the pool size chosen (None: left to the library)."""
    if d.world <= 1:
        return None
    # every rank takes part in the collective, whatever its own environment
    # says: a rank that skipped it (its own LSP_HOST_THREADS set) would leave
    # the others blocked in the gloo all_gather
    import socket
    mask = tuple(sorted(os.sched_getaffinity(0))) if hasattr(os, "sched_getaffinity") else None
    key = (socket.gethostname(), mask)
    keys = d.all_gather_object(key)
    if "LSP_HOST_THREADS" in os.environ or mask is None:
        return None
    sharers = sum(1 for k in keys if k == key)
    n = max(1, min(16, len(mask) // max(sharers, 1)))
    os.environ["LSP_HOST_THREADS"] = str(n)
    return n


def timed_steps(step: Callable[[], object], steps: int, warmup: int, d: Dist,
                sync: Callable[[], None] = lambda: None, on_step: Callable[[], None] = lambda: None,
                step_times: Optional[list] = None, on_start: Callable[[], object] = lambda: None):
    """W untimed steps, barrier + sync, K timed steps, sync + barrier; returns
    (max-over-ranks elapsed seconds, last step result).  `step_times` (if given)
    receives this rank's wall time of every timed step (the step itself
    returns with its result on the host).  `on_start` runs once after the
    opening barrier + sync, just before the clock starts (bench.py's clock
    sampler)."""
    out = None
    for _ in range(warmup):
        out = step()
    d.barrier()
    sync()
    on_start()
    t0 = time.perf_counter()
    for _ in range(steps):
        ts = time.perf_counter()
        out = step()
        if step_times is not None:
            step_times.append(time.perf_counter() - ts)
        on_step()
    sync()
    d.barrier()
    return d.max(time.perf_counter() - t0), out


def rank_seed(base_seed: int, rank: int) -> int:
    """Each replica proves a distinct synthetic trace."""
    return base_seed + rank
