"""Hash-partitioned snapshot and BFS over several GPUs (config 4).

The reference's incidence index (HGStore.getIncidenceResultSet, C/HGStore.java:253) is split by
atom: owner(atom) = atom % n_parts.  Part p holds the incidence rows of its atoms and the target
rows of every link with an owned target; each BFS level it sends the rows it discovered for atoms
owned elsewhere to their owners (one all-to-all per level: RCCL between processes, device copies
inside one process).  Results are identical to ``bfs_batch`` on the whole snapshot
(HGBreadthFirstTraversal + DefaultALGenerator, C/algorithms/HGBreadthFirstTraversal.java:49-66).

  Shard.build(graph arrays, n_parts, part)      host partition (C ABI hgx_shard_build)
  ShardSnapshot(shard, device)                  one part on one device
  pbfs_batch_group(shard_snapshots, seeds, d)   every part in this process (one thread per part)
  RcclComm.create(ctx, device) + pbfs_batch     one part per process over RCCL
  PartitionedBfsResult                          the union of the parts' results
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import check, lib, ptr
from .algorithms import BfsResult, DefaultALGenerator


class Shard:
    """Host-side partition of one part (no device work)."""

    def __init__(self, handle, n_parts, part):
        self._h = handle
        self.n_parts, self.part = n_parts, part
        a, o, m, p = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int64()
        check(lib().hgx_shard_info(handle, C.byref(a), C.byref(o), C.byref(m), C.byref(p)))
        self.n_local, self.n_owned, self.n_links, self.n_pins = a.value, o.value, m.value, p.value

    @classmethod
    def build(cls, num_atoms, link_atom, tgt_off, tgt_idx, link_type, n_parts, part):
        link_atom = np.ascontiguousarray(link_atom, np.int32)
        tgt_off = np.ascontiguousarray(tgt_off, np.int64)
        tgt_idx = np.ascontiguousarray(tgt_idx, np.int32)
        lt = None if link_type is None else np.ascontiguousarray(link_type, np.int32)
        desc = _lib.GraphDesc(int(num_atoms), len(link_atom), ptr(link_atom), ptr(tgt_off), ptr(tgt_idx), ptr(lt))
        h = C.c_void_p()
        check(lib().hgx_shard_build(C.byref(desc), int(n_parts), int(part), C.byref(h)))
        return cls(h, int(n_parts), int(part))

    def export(self) -> dict:
        """The local tables (l2g, link_atom, link_type, tgt_off, tgt_idx in local ids, ghost_count)."""
        d = {"l2g": np.empty(max(self.n_local, 1), np.int32), "link_atom": np.empty(max(self.n_links, 1), np.int32),
             "link_type": np.empty(max(self.n_links, 1), np.int32), "tgt_off": np.empty(self.n_links + 1, np.int64),
             "tgt_idx": np.empty(max(self.n_pins, 1), np.int32), "ghost_count": np.empty(self.n_parts, np.int64)}
        check(lib().hgx_shard_export(self._h, ptr(d["l2g"]), ptr(d["link_atom"]), ptr(d["link_type"]),
                                     ptr(d["tgt_off"]), ptr(d["tgt_idx"]), ptr(d["ghost_count"])))
        d["l2g"] = d["l2g"][: self.n_local]
        d["link_atom"] = d["link_atom"][: self.n_links]
        d["link_type"] = d["link_type"][: self.n_links]
        d["tgt_idx"] = d["tgt_idx"][: self.n_pins]
        return d

    def close(self):
        if getattr(self, "_h", None) is not None:
            lib().hgx_shard_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ShardSnapshot:
    """One part placed on a device (hgx_shard_graph_create)."""

    def __init__(self, shard: Shard, device=0):
        h = C.c_void_p()
        check(lib().hgx_shard_graph_create(shard._h, int(device), C.byref(h)))
        self._h = h
        self.device = device
        self.n_parts, self.part = shard.n_parts, shard.part

    @property
    def handle(self):
        if self._h is None:
            raise ValueError("shard snapshot closed")
        return self._h

    def set_timing(self, on=True):
        check(lib().hgx_set_timing(self.handle, 1 if on else 0))

    def set_option(self, option, value):
        check(lib().hgx_set_option(self.handle, int(option), int(value)))

    def close(self):
        if getattr(self, "_h", None) is not None:
            lib().hgx_graph_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class RcclComm:
    """RCCL communicator of one process per GPU (the unique id travels over an existing
    torch.distributed group, e.g. the gloo group of bench.py)."""

    def __init__(self, handle, world, rank):
        self._h, self.world, self.rank = handle, world, rank

    @classmethod
    def create(cls, world, rank, device, broadcast=None):
        """``broadcast(bytes) -> bytes`` ships rank 0's id to every rank (identity when world == 1)."""
        buf = (C.c_uint8 * 128)()
        if rank == 0:
            check(lib().hgx_comm_rccl_unique_id(buf))
        uid = bytes(buf)
        if world > 1:
            uid = broadcast(uid)
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        h = C.c_void_p()
        check(lib().hgx_comm_rccl_create(buf, int(world), int(rank), int(device), C.byref(h)))
        return cls(h, world, rank)

    def close(self):
        if getattr(self, "_h", None) is not None:
            lib().hgx_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _md(max_depth):
    return _lib.HGX_UNBOUNDED if max_depth is None or max_depth >= 2**31 - 1 else int(max_depth)


def pbfs_batch(shard_snap: ShardSnapshot, comm: RcclComm, seeds, max_depth=None,
               generator: DefaultALGenerator | None = None) -> BfsResult:
    """This process's part of a partitioned batched BFS (collective over the communicator)."""
    opts = (generator or DefaultALGenerator(None)).options()
    s = np.ascontiguousarray(seeds, np.int32)
    h = C.c_void_p()
    check(lib().hgx_pbfs_batch(shard_snap.handle, comm._h, ptr(s), len(s), _md(max_depth), C.byref(opts),
                               C.byref(h)))
    return BfsResult(shard_snap, h, s)


def pbfs_batch_group(shard_snaps, seeds, max_depth=None, generator: DefaultALGenerator | None = None):
    """Every part in this process: returns a PartitionedBfsResult over the parts' results."""
    opts = (generator or DefaultALGenerator(None)).options()
    s = np.ascontiguousarray(seeds, np.int32)
    n = len(shard_snaps)
    arr = (C.c_void_p * n)(*[x.handle for x in shard_snaps])
    outs = (C.c_void_p * n)()
    check(lib().hgx_pbfs_batch_group(arr, n, ptr(s), len(s), _md(max_depth), C.byref(opts), outs))
    return PartitionedBfsResult([BfsResult(shard_snaps[p], C.c_void_p(outs[p]), s) for p in range(n)])


class PartitionedBfsResult:
    """Union of the parts' results: counts add up, visited lists are disjoint and merge sorted."""

    def __init__(self, parts):
        self.parts = parts
        self.n_seeds = parts[0].n_seeds
        self.n_levels = max(p.n_levels for p in parts)

    def counts(self) -> np.ndarray:
        out = np.zeros((self.n_seeds, self.n_levels), np.int64)
        for p in self.parts:
            c = p.counts()
            out[:, : c.shape[1]] += c
        return out

    def visited(self, seed_index, depth) -> np.ndarray:
        return np.sort(np.concatenate([p.visited(seed_index, depth) for p in self.parts]))

    def depth_of(self, seed_index, atom) -> int:
        p = self.parts[int(atom) % len(self.parts)]
        return p.depth_of(seed_index, atom)

    def stats(self, accounting=True) -> list:
        return [p.stats(accounting) for p in self.parts]

    def close(self):
        for p in self.parts:
            p.close()
