"""Per-call latency and many-caller throughput of the drop-in paths (VERDICT r2 'what's missing' 4).

The Java drop-ins call the engine once per query (GpuAndToQuery.getQuery(...).execute()) and once per
traversal (HGGpuTraversal: one hgx_bfs_sequence per start atom), from many threads at once
(TC/query/QueryCompilation.java:76-122: 20 threads).  This tool measures, with native caller threads
(tools/native/hgx_callers.cc; Python threads would serialise on the interpreter lock):
  - config 3: single-query latency (1 caller) and q/s of 20 callers each issuing single And queries,
    with HGX_OPT_QUERY_COALESCE on (default) and off, every hit count checked against one 10K batch;
  - configs 2 and 5: single-seed hgx_bfs_sequence latency (1 caller) and 20 callers.
Writes one JSON object (stdout, or --out)."""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
CALLERS = os.path.join(ROOT, "tools", "native", "build", "libhgx_callers.so")


def log(m):
    print(f"[callers {time.strftime('%H:%M:%S')}] {m}", file=sys.stderr, flush=True)


def callers():
    L = C.CDLL(CALLERS)
    vp = C.c_void_p
    L.hgxc_pattern_threads.argtypes = [vp, C.c_int32, C.c_int32, vp, vp, vp, vp, vp, vp, C.c_int32, vp,
                                       C.POINTER(C.c_double)]
    L.hgxc_sequence_threads.argtypes = [vp, C.c_int32, C.c_int32, vp, C.c_int32, vp, vp, C.POINTER(C.c_double),
                                        C.c_int32]
    return L


def ptr(a):
    return a.ctypes.data_as(C.c_void_p)


def packed_config3(Q):
    nq = len(Q["type"])
    return (np.ascontiguousarray(Q["type"], np.int32), np.arange(nq + 1, dtype=np.int64),
            np.ascontiguousarray(Q["a"], np.int32), np.ones(nq, np.int32), np.arange(0, 3 * nq + 1, 3, dtype=np.int64),
            np.ascontiguousarray(np.stack([Q["x"], np.full(nq, -1, np.int32), Q["y"]], 1).reshape(-1), np.int32))


def pattern_leg(L, snap, packed, n, threads, per_call, expect):
    hits = np.zeros(n, np.int64)
    sec = C.c_double()
    rc = L.hgxc_pattern_threads(snap.handle, threads, n, *(ptr(a) for a in packed), per_call, ptr(hits), C.byref(sec))
    if rc != 0:
        from hypergraphdb_amd._lib import lib
        raise RuntimeError(f"hgxc_pattern_threads rc={rc}: {lib().hgx_last_error().decode()}")
    ok = bool(np.array_equal(hits, expect[:n]))
    return {"threads": threads, "queries_per_call": per_call, "queries": n, "seconds": round(sec.value, 5),
            "qps": round(n / sec.value, 1), "us_per_call": round(sec.value / (n / per_call) * 1e6 * threads, 2),
            "hits_match_batch": ok}


def seq_leg(L, snap, seeds, depth, opts, threads, contexts=0):
    from hypergraphdb_amd._lib import AlgenOpts
    o = AlgenOpts(*opts)
    pairs = np.zeros(len(seeds), np.int64)
    sec = C.c_double()
    s = np.ascontiguousarray(seeds, np.int32)
    rc = L.hgxc_sequence_threads(snap.handle, threads, len(s), ptr(s), depth, C.cast(C.pointer(o), C.c_void_p),
                                 ptr(pairs), C.byref(sec), contexts)
    if rc != 0:
        from hypergraphdb_amd._lib import lib
        raise RuntimeError(f"hgxc_sequence_threads rc={rc}: {lib().hgx_last_error().decode()}")
    return {"threads": threads, "contexts": bool(contexts), "seeds": len(s), "seconds": round(sec.value, 5),
            "traversals_per_s": round(len(s) / sec.value, 1),
            "ms_per_traversal_per_caller": round(sec.value / len(s) * threads * 1e3, 4),
            "pairs": int(pairs.sum())}, pairs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--threads", type=int, default=20)
    ap.add_argument("--single", type=int, default=2000, help="queries of the 1-caller latency leg")
    ap.add_argument("--seq-seeds", type=int, default=200)
    ap.add_argument("--no-seq", action="store_true")
    ap.add_argument("--out")
    args = ap.parse_args()
    import hypergraphdb_amd as H
    from hypergraphdb_amd import _lib, synth
    from hypergraphdb_amd.query import pattern_batch_arrays
    L = callers()
    out = {"tool": "tools/bench_callers.py", "caller_threads": args.threads}

    g3 = synth.config3(scale=args.scale, n_queries=10_000)
    snap = H.HyperGraphSnapshot(g3["num_atoms"], g3["link_atom"], g3["tgt_off"], g3["tgt_idx"], g3["link_type"])
    packed = packed_config3(g3["queries"])
    nq = len(packed[0])
    ref = pattern_batch_arrays(snap, *packed)   # one 10K batch: the expected hit counts (+ warm-up)
    expect = np.diff(np.asarray(ref.offsets, np.int64))
    pattern_batch_arrays(snap, *packed)
    legs = []
    legs.append(("batch_10k_1_caller", pattern_leg(L, snap, packed, nq, 1, nq, expect)))
    legs.append(("single_1_caller", pattern_leg(L, snap, packed, min(args.single, nq), 1, 1, expect)))
    for on in (1, 0):
        snap.set_option(_lib.HGX_OPT_QUERY_COALESCE, on)
        d0, c0 = C.c_int64(), C.c_int64()
        _lib.lib().hgx_query_coalesce_stats(snap.handle, C.byref(d0), C.byref(c0))
        leg = pattern_leg(L, snap, packed, nq, args.threads, 1, expect)
        d1, c1 = C.c_int64(), C.c_int64()
        _lib.lib().hgx_query_coalesce_stats(snap.handle, C.byref(d1), C.byref(c1))
        leg["device_batches"] = d1.value - d0.value
        leg["caller_batches"] = c1.value - c0.value
        legs.append((f"single_{args.threads}_callers_coalesce_{'on' if on else 'off'}", leg))
    snap.set_option(_lib.HGX_OPT_QUERY_COALESCE, 1)
    out["config3_pattern"] = dict(legs)
    for k, v in legs:
        log(f"config3 {k}: {v['qps']:.0f} q/s ({v['us_per_call']} us per call per caller), hits ok {v['hits_match_batch']}")
    snap.close()
    del g3

    if not args.no_seq:
        for name, mk, depth, opts in (("config2_depth2", lambda: synth.config2(scale=args.scale), 2, (-1, 1, 1, 0, 0)),
                                      ("config5_subsumed", lambda: synth.config5(scale=args.scale), -1, None),
                                      ("config5_subsumes", lambda: synth.config5(scale=args.scale), -1, None)):
            g = mk()
            if opts is None:
                opts = (int(g["subsumes_type"]), 0, 1, 1 if name.endswith("subsumes") else 0, 0)
            snap = H.HyperGraphSnapshot(g["num_atoms"], g["link_atom"], g["tgt_off"], g["tgt_idx"], g["link_type"])
            seeds = np.asarray(g["seeds"][: args.seq_seeds], np.int32)
            seq_leg(L, snap, seeds[:8], depth, opts, 1)   # warm-up (index + yield flags on first use)
            one, p1 = seq_leg(L, snap, seeds, depth, opts, 1)
            many, pm = seq_leg(L, snap, seeds, depth, opts, args.threads)
            manyc, pc = seq_leg(L, snap, seeds, depth, opts, args.threads, contexts=1)
            one["pairs_match_many"] = bool(np.array_equal(p1, pm) and np.array_equal(p1, pc))
            out[f"{name}_sequence"] = {"single_seed_1_caller": one, f"single_seed_{args.threads}_callers": many,
                                       f"single_seed_{args.threads}_callers_own_contexts": manyc}
            log(f"{name} sequence: 1 caller {one['ms_per_traversal_per_caller']} ms per traversal; "
                f"{args.threads} callers {many['traversals_per_s']:.0f} traversals/s on one graph, "
                f"{manyc['traversals_per_s']:.0f} on their own contexts")
            snap.close()
            del g
    js = json.dumps(out, indent=1)
    if args.out:
        open(args.out, "w").write(js)
    print(js)


if __name__ == "__main__":
    main()
