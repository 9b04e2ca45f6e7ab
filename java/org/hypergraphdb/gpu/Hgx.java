/*
 * Hgx.java -- JNI declarations of the MI355X engine (libhgx.so, C ABI include/hgx.h) for the
 * reference's Java 1.8 target (pom.xml:14).  Every native is implemented in java/jni/hgx_jni.c;
 * a nonzero hgx_* status becomes an HGException, HGX_E_UNSUPPORTED an UnsupportedOperationException
 * (the caller then keeps the reference's CPU class).
 *
 * UNVERIFIED: written against the cited reference interfaces; this build image has no JDK, so the
 * Java side has not been compiled or run here (SURVEY.md section 0.5).
 */
package org.hypergraphdb.gpu;

final class Hgx
{
    static { System.loadLibrary("hgx_jni"); }   // java/jni/hgx_jni.c, linked against libhgx.so

    private Hgx() {}

    static final int NO_TYPE = -1, ANY_HANDLE = -1, UNBOUNDED = -1;
    static final int OPT_BFS_FLAGS = 1, OPT_SEQ_BUDGET = 2, OPT_RANKS_ORDERED = 3, OPT_PART_SERIAL = 4;
    static final int OPT_QUERY_FUSED = 5, OPT_QUERY_INLINE = 6, OPT_PUSH_BATCH = 7, OPT_PART_EXCHANGE = 8,
                     OPT_QUERY_FLAT = 9, OPT_CODED = 10, OPT_QUERY_COALESCE = 11, OPT_PUSH_INLINE = 12,
                     OPT_SEQ_ENGINE = 13, OPT_BFS_BLOCK = 14;   // include/hgx.h

    // ---- snapshot (hgx_graph_create / open / destroy / update / info) ---------------------------
    static native long graphCreate(long numAtoms, int[] linkAtom, long[] tgtOff, int[] tgtIdx, int[] linkType,
                                   int device);
    static native long graphOpen(String path, int device);
    static native void graphDestroy(long g);
    static native long graphContext(long g);                     // hgx_graph_context: one per concurrent caller
    static native long[] graphInfo(long g);                      // {num_atoms, num_links, num_incidences}
    static native void graphUpdate(long g, long numAtoms, int[] addLinkAtom, long[] addTgtOff, int[] addTgtIdx,
                                   int[] addLinkType, int[] removeLinkAtom);
    static native int[] incidence(long g, int atom);            // link atom ids, ascending
    static native long[] degree(long g, int[] atoms);
    static native void setOption(long g, int option, long value);
    static native void snapshotWrite(String path, long numAtoms, int[] linkAtom, long[] tgtOff, int[] tgtIdx,
                                     int[] linkType, byte[] handles, int handleBytes);
    static native long[] snapshotInfo(String path);             // {num_atoms, num_links, num_pins, handle_bytes, has_types}
    static native byte[] snapshotHandles(String path);          // rank-ordered handle bytes (or null)
    static native void snapshotVerify(String path);             // whole-file checksum (throws on mismatch)
    static native byte[] snapshotHandlesRange(String path, long first, long n);   // ranks [first, first + n)
    // streaming writer (hgx_snapshot_writer_*): handle tables beyond one byte[]
    static native long snapshotWriterBegin(String path, long numAtoms, int[] linkAtom, long[] tgtOff, int[] tgtIdx,
                                           int[] linkType, int handleBytes);
    static native void snapshotWriterHandles(long w, byte[] handles, int handleBytes);
    static native void snapshotWriterEnd(long w);               // checksum + atomic replace; frees w
    static native void snapshotWriterAbort(long w);

    // ---- batched BFS (hgx_bfs_batch + readers) ----------------------------------------------
    static native long bfsBatch(long g, int[] seeds, int maxDepth, int linkType, boolean preceding,
                                boolean succeeding, boolean reverse, boolean source);
    static native int[] bfsInfo(long r);                        // {n_seeds, n_levels}
    static native long[] bfsCounts(long r);                     // [n_seeds * n_levels]
    static native int[] bfsVisited(long r, int seedIndex, int depth);
    static native int[] bfsVisitedRange(long r, int seedIndex, int depth, long first, int max);   // paged
    static native int bfsDepthOf(long r, int seedIndex, int atom);
    static native void bfsFree(long r);

    // ---- order-exact traversal (hgx_bfs_sequence + readers) --------------------------------
    static native long bfsSequence(long g, int[] seeds, int maxDepth, int linkType, boolean preceding,
                                   boolean succeeding, boolean reverse, boolean source);
    static native long[] seqOffsets(long s);                    // [n_seeds + 1]
    static native int[] seqLinks(long s);
    static native int[] seqAtoms(long s);
    static native int[] seqDists(long s);
    static native void seqFree(long s);
    static native int[] seqRange(long s, int which, long first, int max);   // 0 links / 1 atoms / 2 dists, paged
    static native long[] seqEngineStats(long s);                // {workgroup seeds, level-synchronous seeds, pull levels, grid-stage seeds}

    // ---- conjunctive pattern batches (hgx_pattern_batch_packed / _ext + readers) -------------
    static native long patternBatch(long g, int[] type, long[] incOff, int[] inc, int[] hasOrdered, long[] patOff,
                                    int[] pat);
    static native long querySetCreate(long g, int[] type, long[] incOff, int[] inc, int[] hasOrdered, long[] patOff,
                                      int[] pat);                // hgx_query_set_create: a batch resident in HBM
    static native long patternBatchSet(long g, long set);       // hgx_pattern_batch_set
    static native void querySetFree(long set);
    static native long patternBatchSetInto(long g, long set, long[] offsets, int[] ids);   // -> hits
    static native long patternBatchExt(long g, long[] typeOff, int[] types, long[] incOff, int[] inc, long[] posOff,
                                       int[] pos, long[] psetOff, long[] patOff, int[] pat, int[] arity);
    static native long[] queryOffsets(long q);                  // [n + 1]
    static native int[] queryIds(long q);
    static native void queryFree(long q);
    static native long[] queryCoalesceStats(long g);            // {device batches, caller batches}

    // ---- partitioned snapshot (config 4: one part per GPU / JVM) -----------------------------
    static native int[] partitionPlan(long numAtoms, int[] linkAtom, long[] tgtOff, int[] tgtIdx, int[] linkType,
                                      int nParts);
    static native long shardBuild(long numAtoms, int[] linkAtom, long[] tgtOff, int[] tgtIdx, int[] linkType,
                                  int nParts, int part, int[] plan);
    static native void shardFree(long s);
    static native long shardGraphCreate(long s, int device);
    static native byte[] rcclUniqueId();                        // 128 bytes (rank 0)
    static native long rcclCreate(byte[] id, int world, int rank, int device);
    static native void commDestroy(long c);
    static native long pbfsBatch(long shard, long comm, int[] seeds, int maxDepth, int linkType, boolean preceding,
                                 boolean succeeding, boolean reverse, boolean source);

    static native long[] shardInfo(long s);                     // {n_local, n_owned, n_local_links, n_local_pins}
    static native int[] shardLocalAtoms(long s);                // l2g: global id of each local atom
    static native int[] shardOwners(long s);                    // owner part of each local atom (-1 = here)
    static native long[] pbfsBatchGroup(long[] shards, int[] seeds, int maxDepth, int linkType, boolean preceding,
                                        boolean succeeding, boolean reverse, boolean source);   // one result per part

    // ---- timing / statistics / device -------------------------------------------------------
    static native void setTiming(long g, boolean on);
    static native double[] bfsStats(long r, boolean accounting); // {ms_total, traversed_edges, bytes_min, ms_exchange, bytes_exchanged}
    static native double[] seqStats(long s);                    // {ms_total, traversed_edges}
    static native double[] queryMs(long q);                     // {ms_total, ms_match, bytes_match}
    static native long[] graphExportOffsets(long g);            // tgt_off of the device snapshot (D2H)
    static native int[] graphExportTargets(long g);             // tgt_idx
    static native int[] graphExportLinks(long g);               // link_atom
    static native long patternBatchStructs(long g, int[] type, long[] incOff, int[] inc, int[] hasOrdered,
                                           long[] patOff, int[] pat);   // the hgx_and_query[] form
    static native int deviceCount();
    static native void deviceSynchronize(int device);

    static native String lastError();
    static native String version();
}
