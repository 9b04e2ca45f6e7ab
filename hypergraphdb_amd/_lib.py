"""ctypes binding of libhgx.so (the C ABI declared in include/hgx.h).

The engine is native code only: if libhgx.so is missing or cannot be loaded this module
raises -- there is no CPU fallback on the product path.
"""
from __future__ import annotations

import ctypes as C
import os
import re
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# HGX_LIB_VARIANT=<name>: load tools/native/build/libhgx_<name>.so instead (A/B builds of the engine side by
# side in one GPU session; tools only -- tests/conftest.py, smoke() and bench.py refuse to run with it set)
LIB_PATH = os.path.join(_HERE, "libhgx.so")
LIB_VARIANT = os.environ.get("HGX_LIB_VARIANT") or None
if LIB_VARIANT:
    if not re.fullmatch(r"[A-Za-z0-9_]+", LIB_VARIANT):
        raise ImportError(f"HGX_LIB_VARIANT={LIB_VARIANT!r}: variant names are [A-Za-z0-9_]+")
    LIB_PATH = os.path.join(os.path.dirname(_HERE), "tools", "native", "build", f"libhgx_{LIB_VARIANT}.so")
    print(f"hypergraphdb_amd: loading the A/B variant library {LIB_PATH}", file=sys.stderr)
GEN_PATH = os.path.join(_HERE, "libhgx_gen.so")

HGX_OK = 0
HGX_E_INVALID = -1
HGX_E_DEVICE = -2
HGX_E_NOMEM = -3
HGX_E_UNSUPPORTED = -4
HGX_E_NOTFOUND = -5
HGX_ANY_HANDLE = -1
HGX_NO_TYPE = -1
HGX_UNBOUNDED = -1
HGX_OPT_BFS_FLAGS = 1
HGX_OPT_SEQ_BUDGET = 2
HGX_OPT_RANKS_ORDERED = 3
HGX_OPT_PART_SERIAL = 4
HGX_OPT_QUERY_FUSED = 5
HGX_OPT_QUERY_INLINE = 6
HGX_OPT_PUSH_BATCH = 7
HGX_OPT_PART_EXCHANGE = 8
HGX_OPT_QUERY_FLAT = 9
HGX_OPT_CODED = 10
HGX_OPT_QUERY_COALESCE = 11
HGX_OPT_PUSH_INLINE = 12
HGX_OPT_SEQ_ENGINE = 13
HGX_OPT_BFS_BLOCK = 14
HGX_OPT_CO_TIMEOUT = 15
HGX_OPT_SEQ_PULL = 16
HGX_OPT_SEQ_SMALL = 17
HGX_OPT_SEQ_TLIMIT = 18
HGX_OPT_SEQ_PACK_MIN = 19
HGX_OPT_XB_FLAT = 20
HGX_OPT_XB_STATIC = 21

# Every symbol include/hgx.h declares (checked by tests/test_abi.py without a GPU).
EXPORTED = (
    "hgx_version", "hgx_last_error", "hgx_device_synchronize", "hgx_device_count", "hgx_graph_create", "hgx_graph_context", "hgx_graph_destroy", "hgx_graph_info",
    "hgx_graph_degree", "hgx_graph_incidence", "hgx_set_timing", "hgx_set_option", "hgx_bfs_batch", "hgx_bfs_result_info",
    "hgx_bfs_result_counts", "hgx_bfs_result_visited", "hgx_bfs_result_depth_of", "hgx_bfs_result_stats",
    "hgx_bfs_result_free", "hgx_bfs_sequence", "hgx_seq_result_info", "hgx_seq_result_offsets", "hgx_seq_result_pairs",
    "hgx_seq_result_stats", "hgx_seq_result_engine_stats", "hgx_seq_result_level_stats", "hgx_seq_result_grid_stats", "hgx_seq_result_free", "hgx_pattern_batch", "hgx_pattern_batch_packed", "hgx_pattern_batch_ext", "hgx_query_result_count", "hgx_query_result_offsets", "hgx_query_result_ids",
    "hgx_query_result_ms", "hgx_query_result_free",
    "hgx_partition_plan", "hgx_shard_build", "hgx_shard_info", "hgx_shard_export", "hgx_shard_exchange_tables",
    "hgx_shard_free", "hgx_shard_graph_create", "hgx_comm_rccl_unique_id", "hgx_comm_rccl_create",
    "hgx_comm_host_create", "hgx_comm_destroy", "hgx_comm_check_allgather", "hgx_pbfs_batch", "hgx_pbfs_batch_group",
    "hgx_snapshot_write", "hgx_snapshot_info", "hgx_snapshot_read", "hgx_graph_open", "hgx_graph_export",
    "hgx_graph_update", "hgx_query_coalesce_stats", "hgx_query_set_create", "hgx_pattern_batch_set",
    "hgx_query_set_free", "hgx_pattern_batch_set_into", "hgx_query_set_info", "hgx_snapshot_read_handles",
    "hgx_snapshot_writer_begin", "hgx_snapshot_writer_handles", "hgx_snapshot_writer_end", "hgx_snapshot_writer_abort", "hgx_snapshot_writer_handle_bytes",
    "hgx_bfs_result_visited_range", "hgx_seq_result_pairs_range",
)


class GraphDesc(C.Structure):
    _fields_ = [("num_atoms", C.c_int64), ("num_links", C.c_int64), ("link_atom", C.c_void_p),
                ("tgt_off", C.c_void_p), ("tgt_idx", C.c_void_p), ("link_type", C.c_void_p)]


class AlgenOpts(C.Structure):
    _fields_ = [("link_type", C.c_int32), ("return_preceding", C.c_uint8), ("return_succeeding", C.c_uint8),
                ("reverse_order", C.c_uint8), ("return_source", C.c_uint8)]


class AndQuery(C.Structure):
    _fields_ = [("type", C.c_int32), ("n_incident", C.c_int32), ("incident", C.c_void_p),
                ("has_ordered", C.c_int32), ("n_pattern", C.c_int32), ("pattern", C.c_void_p)]


KERNELS = ("hgx_link_gather", "hgx_atom_pull", "hgx_atom_pull_heavy", "hgx_hub_finalize", "hgx_frontier_push",
           "hgx_nf_pull", "hgx_fc_pull", "hgx_fc_pull_heavy")


class BfsStats(C.Structure):
    _fields_ = [("n_levels_expanded", C.c_int32), ("n_batches", C.c_int32), ("ms_total", C.c_double),
                ("ms_kernel", C.c_double * 8), ("launches", C.c_int64 * 8), ("bytes_kernel", C.c_double * 8),
                ("bytes_survey", C.c_double), ("traversed_edges", C.c_double),
                ("union_frontier", C.c_int64 * 64), ("level_ms", C.c_double * 64), ("level_new", C.c_int64 * 64),
                ("level_bytes", C.c_double * 64), ("level_sparse", C.c_int32 * 64),
                ("level_rows", (C.c_int64 * 8) * 64), ("ms_exchange", C.c_double),
                ("bytes_exchanged", C.c_double), ("level_xbytes", C.c_double * 64),
                ("level_xpair_max", C.c_double * 64), ("level_xms", C.c_double * 64),
                ("xwords_nonzero", C.c_double), ("xwords_total", C.c_double), ("bytes_min", C.c_double),
                ("level_xtrips", C.c_int32 * 64), ("ms_block", C.c_double), ("bytes_block", C.c_double),
                ("block_seeds", C.c_int64), ("block_rerun", C.c_int64), ("ms_coop", C.c_double),
                ("bytes_coop", C.c_double), ("block_coop", C.c_int64), ("coop_fallbacks", C.c_int64)]

    def as_dict(self):
        d = {"n_levels_expanded": self.n_levels_expanded, "n_batches": self.n_batches, "ms_total": self.ms_total,
             "bytes_survey": self.bytes_survey, "traversed_edges": self.traversed_edges,
             "ms_exchange": self.ms_exchange, "bytes_exchanged": self.bytes_exchanged, "bytes_min": self.bytes_min,
             "block_seeds": int(self.block_seeds), "block_rerun": int(self.block_rerun),
             "block_coop": int(self.block_coop), "coop_fallbacks": int(self.coop_fallbacks)}
        d["kernels"] = {k: {"ms": self.ms_kernel[i], "launches": int(self.launches[i]),
                            "bytes": self.bytes_kernel[i]} for i, k in enumerate(KERNELS)}
        if self.block_seeds or self.block_rerun:   # the workgroup-per-seed stage: one launch per 4096 seeds
            d["kernels"]["hgx_bfs_block"] = {"ms": self.ms_block, "bytes": self.bytes_block,
                                             "launches": int((self.block_seeds + self.block_rerun + 4095) // 4096)}
        if self.block_coop:   # one persistent launch for the seeds that outgrew a workgroup
            d["kernels"]["hgx_bfs_coop"] = {"ms": self.ms_coop, "bytes": self.bytes_coop, "launches": 1}
        n = min(max(self.n_levels_expanded, 0), 64)   # per-level arrays hold the first 64 levels
        d["union_frontier"] = [int(x) for x in self.union_frontier[:n]]
        d["level_ms"] = [round(float(x), 4) for x in self.level_ms[:n]]
        d["level_new"] = [int(x) for x in self.level_new[:n]]
        d["level_bytes"] = [float(x) for x in self.level_bytes[:n]]
        d["level_sparse"] = [int(x) for x in self.level_sparse[:n]]
        d["level_rows"] = [[int(v) for v in self.level_rows[i]] for i in range(n)]
        d["level_xbytes"] = [float(x) for x in self.level_xbytes[:n]]
        d["level_xpair_max"] = [float(x) for x in self.level_xpair_max[:n]]
        d["level_xms"] = [round(float(x), 4) for x in self.level_xms[:n]]
        d["level_xtrips"] = [int(x) for x in self.level_xtrips[:n]]
        d["xwords_nonzero"], d["xwords_total"] = self.xwords_nonzero, self.xwords_total
        return d


class HGXError(RuntimeError):
    """A failed hgx_* call (the reference maps these to HGException)."""

    def __init__(self, code, msg):
        super().__init__(f"hgx error {code}: {msg}")
        self.code = code


class HGXUnsupported(HGXError):
    """The shape is not accelerated (HGX_E_UNSUPPORTED); a Java shim would delegate to the CPU compiler."""


_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
                          " (make -C hypergraphdb_amd/csrc).  There is no CPU fallback.")
    L = C.CDLL(LIB_PATH)
    vp, i32, i64 = C.c_void_p, C.c_int32, C.c_int64
    sig = {
        "hgx_version": ([], C.c_char_p),
        "hgx_last_error": ([], C.c_char_p),
        "hgx_device_synchronize": ([i32], C.c_int),
        "hgx_device_count": ([C.POINTER(i32)], C.c_int),
        "hgx_graph_create": ([C.POINTER(GraphDesc), i32, C.POINTER(vp)], C.c_int),
        "hgx_graph_context": ([vp, C.POINTER(vp)], C.c_int),
        "hgx_graph_destroy": ([vp], None),
        "hgx_graph_info": ([vp, C.POINTER(i64), C.POINTER(i64), C.POINTER(i64)], C.c_int),
        "hgx_graph_degree": ([vp, vp, i32, vp], C.c_int),
        "hgx_graph_incidence": ([vp, i32, vp, i64, C.POINTER(i64)], C.c_int),
        "hgx_set_timing": ([vp, i32], C.c_int),
        "hgx_set_option": ([vp, i32, i64], C.c_int),
        "hgx_bfs_batch": ([vp, vp, i32, i32, C.POINTER(AlgenOpts), C.POINTER(vp)], C.c_int),
        "hgx_bfs_result_info": ([vp, C.POINTER(i32), C.POINTER(i32)], C.c_int),
        "hgx_bfs_result_counts": ([vp, vp], C.c_int),
        "hgx_bfs_result_visited": ([vp, i32, i32, vp, i64, C.POINTER(i64)], C.c_int),
        "hgx_bfs_result_depth_of": ([vp, i32, i32, C.POINTER(i32)], C.c_int),
        "hgx_bfs_result_stats": ([vp, i32, C.POINTER(BfsStats)], C.c_int),
        "hgx_bfs_result_free": ([vp], None),
        "hgx_bfs_sequence": ([vp, vp, i32, i32, C.POINTER(AlgenOpts), C.POINTER(vp)], C.c_int),
        "hgx_seq_result_info": ([vp, C.POINTER(i32), C.POINTER(i64), C.POINTER(i32)], C.c_int),
        "hgx_seq_result_offsets": ([vp, vp], C.c_int),
        "hgx_seq_result_pairs": ([vp, vp, vp, vp], C.c_int),
        "hgx_seq_result_stats": ([vp, C.POINTER(C.c_double), C.POINTER(C.c_double)], C.c_int),
        "hgx_seq_result_engine_stats": ([vp, C.POINTER(i32), C.POINTER(i32), C.POINTER(C.c_double),
                                         C.POINTER(C.c_double)], C.c_int),
        "hgx_seq_result_level_stats": ([vp, C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(i64)], C.c_int),
        "hgx_seq_result_grid_stats": ([vp, C.POINTER(i32), C.POINTER(C.c_double), C.POINTER(C.c_double)], C.c_int),
        "hgx_seq_result_free": ([vp], None),
        "hgx_pattern_batch": ([vp, C.POINTER(AndQuery), i32, C.POINTER(vp)], C.c_int),
        "hgx_pattern_batch_packed": ([vp, i32, vp, vp, vp, vp, vp, vp, C.POINTER(vp)], C.c_int),
        "hgx_pattern_batch_ext": ([vp, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, C.POINTER(vp)], C.c_int),
        "hgx_query_result_count": ([vp, C.POINTER(i64)], C.c_int),
        "hgx_query_result_offsets": ([vp, vp], C.c_int),
        "hgx_query_result_ids": ([vp, vp], C.c_int),
        "hgx_query_result_ms": ([vp, C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_double)], C.c_int),
        "hgx_query_result_free": ([vp], None),
        "hgx_partition_plan": ([C.POINTER(GraphDesc), i32, vp], C.c_int),
        "hgx_shard_build": ([C.POINTER(GraphDesc), i32, i32, vp, C.POINTER(vp)], C.c_int),
        "hgx_shard_exchange_tables": ([vp, vp, vp, vp, vp, vp, vp], C.c_int),
        "hgx_comm_host_create": ([i32, i32, vp, vp, vp, C.POINTER(vp)], C.c_int),
        "hgx_shard_info": ([vp, C.POINTER(i64), C.POINTER(i64), C.POINTER(i64), C.POINTER(i64)], C.c_int),
        "hgx_shard_export": ([vp, vp, vp, vp, vp, vp, vp], C.c_int),
        "hgx_shard_free": ([vp], None),
        "hgx_shard_graph_create": ([vp, i32, C.POINTER(vp)], C.c_int),
        "hgx_comm_rccl_unique_id": ([vp], C.c_int),
        "hgx_comm_rccl_create": ([vp, i32, i32, i32, C.POINTER(vp)], C.c_int),
        "hgx_comm_destroy": ([vp], None),
        "hgx_comm_check_allgather": ([vp, i32, vp, i64, vp, vp, vp], C.c_int),
        "hgx_pbfs_batch": ([vp, vp, vp, i32, i32, C.POINTER(AlgenOpts), C.POINTER(vp)], C.c_int),
        "hgx_pbfs_batch_group": ([vp, i32, vp, i32, i32, C.POINTER(AlgenOpts), vp], C.c_int),
        "hgx_snapshot_write": ([C.c_char_p, C.POINTER(GraphDesc), vp, i32], C.c_int),
        "hgx_snapshot_info": ([C.c_char_p, C.POINTER(i64), C.POINTER(i64), C.POINTER(i64), C.POINTER(i32),
                               C.POINTER(i32)], C.c_int),
        "hgx_snapshot_read": ([C.c_char_p, vp, vp, vp, vp, vp], C.c_int),
        "hgx_graph_open": ([C.c_char_p, i32, C.POINTER(vp)], C.c_int),
        "hgx_graph_export": ([vp, vp, vp, vp, vp], C.c_int),
        "hgx_graph_update": ([vp, i64, i64, vp, vp, vp, vp, i64, vp], C.c_int),
        "hgx_query_coalesce_stats": ([vp, C.POINTER(i64), C.POINTER(i64)], C.c_int),
        "hgx_query_set_create": ([vp, i32, vp, vp, vp, vp, vp, vp, C.POINTER(vp)], C.c_int),
        "hgx_pattern_batch_set": ([vp, vp, C.POINTER(vp)], C.c_int),
        "hgx_query_set_free": ([vp], None),
        "hgx_pattern_batch_set_into": ([vp, vp, vp, vp, i64, C.POINTER(i64), vp], C.c_int),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    _lib = L
    return L


def check(rc):
    if rc != HGX_OK:
        msg = lib().hgx_last_error().decode(errors="replace")
        if rc == HGX_E_UNSUPPORTED:
            raise HGXUnsupported(rc, msg)
        raise HGXError(rc, msg)


def device_synchronize(device: int = 0):
    check(lib().hgx_device_synchronize(int(device)))


def device_count() -> int:
    n = C.c_int32(0)
    check(lib().hgx_device_count(C.byref(n)))
    return n.value


def ptr(a: np.ndarray):
    return a.ctypes.data if a is not None and a.size else None


_gen = None


def gen_lib():
    """Synthetic generators (host C, OpenMP) -- benchmark/test input only."""
    global _gen
    if _gen is None:
        if not os.path.exists(GEN_PATH):
            raise ImportError(f"{GEN_PATH} is missing (make -C hypergraphdb_amd/csrc)")
        G = C.CDLL(GEN_PATH)
        vp, i32, i64, u64, dbl = C.c_void_p, C.c_int32, C.c_int64, C.c_uint64, C.c_double
        G.hgx_gen_hypergraph_offsets.argtypes = [i64, i32, i32, u64, vp]
        G.hgx_gen_hypergraph_offsets.restype = i64
        G.hgx_gen_hypergraph_fill.argtypes = [i64, i64, i32, i32, dbl, i32, u64, vp, vp, vp]
        G.hgx_gen_hypergraph_fill.restype = C.c_int
        G.hgx_gen_permutation_prefix.argtypes = [i64, i64, u64, vp]
        G.hgx_gen_permutation_prefix.restype = C.c_int
        G.hgx_gen_sources.argtypes = [i64, i64, vp, i64, u64, vp]
        G.hgx_gen_sources.restype = C.c_int
        G.hgx_gen_queries.argtypes = [i64, i64, vp, vp, vp, i64, dbl, u64, vp, vp, vp, vp, vp]
        G.hgx_gen_queries.restype = C.c_int
        G.hgx_gen_ontology.argtypes = [i64, i64, u64, i32, i32, vp, vp]
        G.hgx_gen_ontology.restype = i64
        _gen = G
    return _gen
