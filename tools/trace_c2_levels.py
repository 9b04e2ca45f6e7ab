"""Per-level times / counters of one config-2 batch (HGX_BFS_TRACE=1 adds the engine's per-level lines).

  python tools/trace_c2_levels.py
"""
import os, sys
sys.path.insert(0, '/root/repo')
import hypergraphdb_amd as H
from hypergraphdb_amd import synth
g = synth.config2()
snap = H.HyperGraphSnapshot(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
snap.set_timing(True)
import time
for _ in range(4):
    t0 = time.perf_counter()
    r = H.bfs_batch(snap, g["seeds"], 4)
    r.counts()
    wall = (time.perf_counter() - t0) * 1e3
    st = r.stats(accounting=True)
    print("wall ms (traversal + readout)", round(wall, 3), "device ms", round(st["ms_total"], 3),
          "traversed", st["traversed_edges"], flush=True)
    print({k: st[k] for k in ("level_ms", "level_new", "level_sparse")}, flush=True)
    print("level_rows", st.get("level_rows"), flush=True)
    print("kernels", {k: round(v["ms"], 3) for k, v in st["kernels"].items()}, flush=True)
    r.close()
