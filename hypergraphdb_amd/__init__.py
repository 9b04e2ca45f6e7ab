"""hypergraphdb_amd -- MI355X-native engine for HyperGraphDB's data-parallel query path.

Native engine: libhgx.so (HIP kernels for gfx950 + the C ABI of include/hgx.h).
This package is the host-side mirror of the reference interfaces on that path:
  snapshot.HyperGraphSnapshot   the store snapshot (bipartite CSR on the device)
  algorithms                    DefaultALGenerator / HGBreadthFirstTraversal / bfs_batch
  query                         hg.and/type/incident/orderedLink, GpuAndToQuery, pattern_batch
"""
from ._lib import HGXError, HGXUnsupported, lib  # noqa: F401
from .algorithms import (AtomTypeCondition, BfsResult, DefaultALGenerator, HGBreadthFirstTraversal,  # noqa: F401
                         SequenceResult, bfs_sequence,
                         HGException, bfs_batch)
from .query import (ArityCondition, GpuAndToQuery, HGQueryConfiguration, LinkCondition,  # noqa: F401
                    PositionedIncidentCondition, TypePlusCondition, find_all, hg, pattern_batch)
from .snapshot import HyperGraphSnapshot, export_store, rank_handles, read_snapshot, write_snapshot  # noqa: F401

__version__ = "0.1.0"
