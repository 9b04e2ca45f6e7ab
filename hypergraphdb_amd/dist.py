"""One process per GPU: rank context, source sharding and the timing reductions of bench.py.

The batched BFS shards by SOURCE: every rank holds a replica of the snapshot (config 2 is 2.5 GB of
CSR on a 288 GB device) and traverses its own batch of start atoms, so the data path has no
collective.  Only the barrier and the max/sum of scalars cross processes, over a CPU gloo group
(torch.distributed is plumbing here; torch's HIP runtime is never initialised, so libhgx drives the
device alone).  The hash-partitioned config-4 path runs its per-level all-to-all over RCCL inside
libhgx (partition.RcclComm); only the 128-byte RCCL unique id crosses this gloo group.
"""
from __future__ import annotations

import os
from dataclasses import dataclass


@dataclass
class RankContext:
    rank: int = 0
    world: int = 1
    local: int = 0
    device: int = 0
    dist: object = None

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def _reduce(self, x, op):
        if self.dist is None:
            return x
        import torch
        t = torch.tensor([float(x)], dtype=torch.float64)
        self.dist.all_reduce(t, op=op)
        return float(t.item())

    def max(self, x):
        return self._reduce(x, self.dist.ReduceOp.MAX) if self.dist is not None else x

    def sum(self, x):
        return self._reduce(x, self.dist.ReduceOp.SUM) if self.dist is not None else x

    def sum_array(self, a):
        """Element-wise int64 sum of a numpy array over the ranks (every rank gets the sum)."""
        import numpy as np
        a = np.ascontiguousarray(a, np.int64)
        if self.dist is None:
            return a.copy()
        import torch
        t = torch.from_numpy(a.copy())
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return t.numpy()

    def broadcast_bytes(self, data: bytes) -> bytes:
        """rank 0's bytes on every rank (the RCCL unique id travels over the gloo group)"""
        if self.dist is None:
            return data
        obj = [data if self.rank == 0 else None]
        self.dist.broadcast_object_list(obj, src=0)
        return obj[0]

    def close(self):
        if self.dist is not None:
            self.dist.destroy_process_group()
            self.dist = None


def init_from_env(backend: str = "gloo") -> RankContext:
    """RANK / WORLD_SIZE / LOCAL_RANK / MASTER_* from torch.distributed.run (or a test harness).
    HGX_DEVICE overrides the device ordinal (rehearsing several ranks on a one-GPU box)."""
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    device = int(os.environ.get("HGX_DEVICE", local))
    ctx = RankContext(rank, world, local, device, None)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group(backend)
        ctx.dist = dist
    return ctx


def rank_sources(graph, n_sources: int, rank: int, base_seed: int = 7):
    """The start atoms of one rank: rank 0 uses the config's own source draw (seed 7, SURVEY.md
    8(d)); rank r > 0 draws an independent batch (weak scaling: fixed work per GPU)."""
    from . import synth
    if rank == 0 and "seeds" in graph and len(graph["seeds"]) == n_sources:
        return graph["seeds"]
    return synth.sources(graph, n_sources, base_seed + 1000 * rank)
