"""Partitioned snapshot and BFS over several GPUs (config 4).

The reference's incidence index (HGStore.getIncidenceResultSet, C/HGStore.java:253) is split by
LINK (vertex cut): every link row lives on one part (partition_plan: greedy placement next to the
low-degree targets it shares), an atom is present on every part holding one of its links and owned
by one of them.  Each BFS level every part expands its own links, ships its partial news for atoms
owned elsewhere to their owners (reduce) and the owners ship the final news back (broadcast): RCCL
between processes, device copies inside one process, or host-staged callbacks (a gloo group).
Results are identical to ``bfs_batch`` on the whole snapshot (HGBreadthFirstTraversal +
DefaultALGenerator, C/algorithms/HGBreadthFirstTraversal.java:49-66).

  partition_plan(graph arrays, n_parts)         link placement (C ABI hgx_partition_plan)
  Shard.build(graph arrays, n_parts, part, plan) host partition (hgx_shard_build)
  ShardSnapshot(shard, device)                  one part on one device
  pbfs_batch_group(shard_snapshots, seeds, d)   every part in this process (one thread per part)
  RcclComm.create(...) + pbfs_batch             one part per process over RCCL
  HostComm.gloo(...) + pbfs_batch               one part per process over a torch.distributed group
  PartitionedBfsResult                          the union of the parts' results
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import check, lib, ptr
from .algorithms import BfsResult, DefaultALGenerator


def _desc(num_atoms, link_atom, tgt_off, tgt_idx, link_type):
    arrs = (np.ascontiguousarray(link_atom, np.int32), np.ascontiguousarray(tgt_off, np.int64),
            np.ascontiguousarray(tgt_idx, np.int32),
            None if link_type is None else np.ascontiguousarray(link_type, np.int32))
    return _lib.GraphDesc(int(num_atoms), len(arrs[0]), ptr(arrs[0]), ptr(arrs[1]), ptr(arrs[2]), ptr(arrs[3])), arrs


def partition_plan(num_atoms, link_atom, tgt_off, tgt_idx, link_type, n_parts) -> np.ndarray:
    """link_part[r] = the part that stores link row r (deterministic for a snapshot)."""
    desc, keep = _desc(num_atoms, link_atom, tgt_off, tgt_idx, link_type)
    out = np.zeros(max(len(keep[0]), 1), np.int32)
    check(lib().hgx_partition_plan(C.byref(desc), int(n_parts), ptr(out)))
    return out[: len(keep[0])]


class Shard:
    """Host-side partition of one part (no device work)."""

    def __init__(self, handle, n_parts, part):
        self._h = handle
        self.n_parts, self.part = n_parts, part
        a, o, m, p = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int64()
        check(lib().hgx_shard_info(handle, C.byref(a), C.byref(o), C.byref(m), C.byref(p)))
        self.n_local, self.n_owned, self.n_links, self.n_pins = a.value, o.value, m.value, p.value

    @classmethod
    def build(cls, num_atoms, link_atom, tgt_off, tgt_idx, link_type, n_parts, part, plan=None):
        """plan: link_part from partition_plan (computed here when None)."""
        if plan is None:
            plan = partition_plan(num_atoms, link_atom, tgt_off, tgt_idx, link_type, n_parts)
        plan = np.ascontiguousarray(plan, np.int32)
        desc, keep = _desc(num_atoms, link_atom, tgt_off, tgt_idx, link_type)
        h = C.c_void_p()
        check(lib().hgx_shard_build(C.byref(desc), int(n_parts), int(part), ptr(plan), C.byref(h)))
        return cls(h, int(n_parts), int(part))

    def exchange_tables(self) -> dict:
        """xo_part / xo_lid (owner and the atom's local id there, -1 for owned atoms), bc_off /
        bc_part / bc_lid (each owned atom's other holders and its local id on each), bc_count."""
        n = self.n_local
        d = {"xo_part": np.empty(max(n, 1), np.int32), "xo_lid": np.empty(max(n, 1), np.int32),
             "bc_off": np.empty(n + 1, np.int64), "bc_count": np.empty(self.n_parts, np.int64)}
        check(lib().hgx_shard_exchange_tables(self._h, ptr(d["xo_part"]), ptr(d["xo_lid"]), ptr(d["bc_off"]), None,
                                              None, ptr(d["bc_count"])))
        m = int(d["bc_off"][-1])
        d["bc_part"], d["bc_lid"] = np.empty(max(m, 1), np.int32), np.empty(max(m, 1), np.int32)
        check(lib().hgx_shard_exchange_tables(self._h, None, None, None, ptr(d["bc_part"]), ptr(d["bc_lid"]), None))
        d["xo_part"], d["xo_lid"] = d["xo_part"][:n], d["xo_lid"][:n]
        d["bc_part"], d["bc_lid"] = d["bc_part"][:m], d["bc_lid"][:m]
        return d

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

    def set_serial(self, on=True):
        """In-process rehearsal: the group runs its parts' device work one part at a time."""
        self.set_option(_lib.HGX_OPT_PART_SERIAL, 1 if on else 0)

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


def check_allgather(comm, values, device=0):
    """hgx_comm_check_allgather (collective): the transport's device-input all-gather, the default
    read-back path and the host-input all-gather of every rank's ``values`` -> three (world, n) arrays."""
    v = np.ascontiguousarray(values, np.int64)
    n = len(v)
    outs = [np.full(n * comm.world, -1, np.int64) for _ in range(3)]
    check(lib().hgx_comm_check_allgather(comm._h, int(device), ptr(v), n, ptr(outs[0]), ptr(outs[1]), ptr(outs[2])))
    return [o.reshape(comm.world, n) for o in outs]


_AG = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_int64), C.c_int64, C.POINTER(C.c_int64))
_A2A = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.c_void_p,
                   C.POINTER(C.c_int64), C.POINTER(C.c_int64))


class HostComm:
    """Host-staged transport (hgx_comm_host_create): libhgx stages the exchange segments through
    pinned host memory and calls ``allgather(in_array) -> out_array`` and
    ``alltoallv(send_bytes_per_peer: list[bytes]) -> list[bytes]`` (Python callables) for the
    collectives.  HostComm.gloo(group) wires them to a torch.distributed (gloo) group."""

    def __init__(self, world, rank, allgather, alltoallv):
        self.world, self.rank = world, rank
        self._ag_py, self._a2a_py = allgather, alltoallv

        def ag(_user, inp, n, out):
            try:
                a = np.ctypeslib.as_array(inp, (n,)).copy()
                res = np.asarray(self._ag_py(a), np.int64).reshape(-1)
                np.ctypeslib.as_array(out, (n * world,))[:] = res
                return 0
            except Exception:   # noqa: BLE001 -- reported as a transport failure
                return 1

        def a2a(_user, send, soff, sbytes, recv, roff, rbytes):
            try:
                so = np.ctypeslib.as_array(soff, (world,))
                sb = np.ctypeslib.as_array(sbytes, (world,))
                ro = np.ctypeslib.as_array(roff, (world,))
                rb = np.ctypeslib.as_array(rbytes, (world,))
                parts = [C.string_at(send + int(so[p]), int(sb[p])) if sb[p] > 0 else b"" for p in range(world)]
                got = self._a2a_py(parts)
                for p in range(world):
                    if len(got[p]) != int(rb[p]):
                        return 2
                    if rb[p] > 0:
                        C.memmove(recv + int(ro[p]), got[p], int(rb[p]))
                return 0
            except Exception:   # noqa: BLE001
                return 1

        self._cb = (_AG(ag), _A2A(a2a))   # keep the trampolines alive
        h = C.c_void_p()
        check(lib().hgx_comm_host_create(int(world), int(rank), C.cast(self._cb[0], C.c_void_p),
                                         C.cast(self._cb[1], C.c_void_p), None, C.byref(h)))
        self._h = h

    @classmethod
    def gloo(cls, dist, world, rank):
        """Collectives over an initialised torch.distributed (gloo) default group."""
        import torch

        def allgather(a):
            t = torch.from_numpy(a)
            out = [torch.empty_like(t) for _ in range(world)]
            dist.all_gather(out, t)
            return np.concatenate([o.numpy() for o in out])

        def alltoallv(parts):
            sizes = torch.tensor([len(b) for b in parts], dtype=torch.int64)
            allsz = [torch.empty_like(sizes) for _ in range(world)]
            dist.all_gather(allsz, sizes)
            recv_sz = [int(allsz[q][rank]) for q in range(world)]
            reqs, bufs = [], [None] * world
            for q in range(world):
                if q == rank:
                    bufs[q] = parts[q]
                    continue
                if len(parts[q]):
                    reqs.append(dist.isend(torch.frombuffer(bytearray(parts[q]), dtype=torch.uint8), q))
                if recv_sz[q]:
                    bufs[q] = torch.empty(recv_sz[q], dtype=torch.uint8)
                    reqs.append(dist.irecv(bufs[q], q))
                else:
                    bufs[q] = b""
            for r in reqs:
                r.wait()
            return [b if isinstance(b, bytes) else b.numpy().tobytes() for b in bufs]

        return cls(world, rank, allgather, alltoallv)

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
        """Asked of the owner part (the others answer HGX_E_NOTFOUND)."""
        for p in self.parts:
            try:
                return p.depth_of(seed_index, atom)
            except _lib.HGXError as e:
                if e.code != _lib.HGX_E_NOTFOUND:
                    raise
        raise _lib.HGXError(_lib.HGX_E_NOTFOUND, f"no part owns atom {atom}")

    def stats(self, accounting=True) -> list:
        return [p.stats(accounting) for p in self.parts]

    def close(self):
        for p in self.parts:
            p.close()
