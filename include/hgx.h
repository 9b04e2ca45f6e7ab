/*
 * hgx.h -- C ABI of the MI355X engine for HyperGraphDB's data-parallel query path.
 *
 * Plain pointers and sizes only; no C++ or torch types.  Every entry point returns an
 * int status (HGX_OK = 0) and never throws or aborts across the ABI; the message of the
 * last failure on the calling thread is hgx_last_error().  All entry points are
 * thread-safe (one mutex per graph; calls on one graph are serialised -- use one execution
 * context per concurrent caller, hgx_graph_context, to run them side by side).
 *
 * Reference interfaces replaced (paths relative to the reference root,
 * C = core/src/java/org/hypergraphdb):
 *   hgx_graph_create      <- the HGStore incidence index + link records read by
 *                            HyperGraph.getIncidenceSet (C/HyperGraph.java:1415-1418) and
 *                            HGStore.getLink (C/HGStore.java:179-191), snapshotted once.
 *   hgx_bfs_batch         <- HGBreadthFirstTraversal(start, DefaultALGenerator, maxDistance)
 *                            (C/algorithms/HGBreadthFirstTraversal.java:122-164) driven to
 *                            exhaustion, for many start atoms at once; HGTraversal
 *                            (C/algorithms/HGTraversal.java:36-63).
 *   hgx_pattern_batch     <- ConditionToQuery.getQuery for And (C/query/cond2qry/AndToQuery.java:102-306)
 *                            on And{AtomTypeCondition?, IncidentCondition*, OrderedLinkCondition?}
 *                            after ExpressionBasedQuery.expand (:603-762), executed
 *                            (ZigZagIntersectionResult + PredicateBasedFilter), for many queries.
 *
 * Identity: every atom (node or link) is an int32 id = its rank in persistent-handle
 * byte order (C/handle/UUID.java:364-376; IntPersistentHandle via C/storage/BAUtils.java:55-80).
 * Rank order preserves every sorted list of the reference, so GPU result order is the
 * reference's result order -- for a snapshot whose ranks were assigned in handle order (see
 * HGX_OPT_RANKS_ORDERED for snapshots grown by hgx_graph_update).  The caller keeps the
 * rank -> handle table.
 */
#ifndef HGX_H
#define HGX_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HGX_OK              0
#define HGX_E_INVALID      -1   /* bad argument (null pointer, id out of range, unsorted ranks) */
#define HGX_E_DEVICE       -2   /* HIP runtime / kernel failure                               */
#define HGX_E_NOMEM        -3   /* device or host allocation failed                           */
#define HGX_E_UNSUPPORTED  -4   /* shape not accelerated: the caller falls back to the CPU path */
#define HGX_E_NOTFOUND     -5   /* no such seed / depth / query in a result                  */

#define HGX_ANY_HANDLE     (-1) /* hg.anyHandle() inside an ordered pattern                  */
#define HGX_NO_TYPE        (-1) /* no AtomTypeCondition / no link predicate                  */
#define HGX_UNBOUNDED      (-1) /* maxDistance == Integer.MAX_VALUE                          */

typedef struct hgx_graph hgx_graph;
typedef struct hgx_bfs_result hgx_bfs_result;
typedef struct hgx_query_result hgx_query_result;

/* Snapshot of the store.  Link row r (0..num_links-1) is atom link_atom[r] (strictly
 * ascending); its layout is [type, value, t0..tk-1] (C/HyperGraph.java:1603-1608) of
 * which link_type[r] = type key and tgt_idx[tgt_off[r] .. tgt_off[r+1]) = t0..tk-1.
 * Targets may be links.  The incidence index (atom -> incident links) is derived on the
 * device: one entry per distinct (target, link), ascending (BJE putNoDupData + sorted
 * duplicates, storage/bdb-je/.../BJEStorageImplementation.java:109-111,300-307).
 * All arrays are deep-copied; the caller may free them on return. */
typedef struct hgx_graph_desc {
    int64_t        num_atoms;   /* A: nodes + links                                 */
    int64_t        num_links;   /* M                                                */
    const int32_t *link_atom;   /* [M]                                              */
    const int64_t *tgt_off;     /* [M+1]                                            */
    const int32_t *tgt_idx;     /* [tgt_off[M]]                                     */
    const int32_t *link_type;   /* [M] type key (>= 0), or NULL = all 0             */
} hgx_graph_desc;

/* DefaultALGenerator configuration (C/algorithms/DefaultALGenerator.java:437-502).
 * link_type: HGX_NO_TYPE = linkPredicate null, else AtomTypeCondition(type) on the
 * incident link (C/query/AtomTypeCondition.java:121-135).  A siblingPredicate or any
 * other link predicate is not accelerated (the caller keeps the CPU traversal). */
typedef struct hgx_algen_opts {
    int32_t link_type;
    uint8_t return_preceding;    /* default 1 */
    uint8_t return_succeeding;   /* default 1 */
    uint8_t reverse_order;       /* default 0 */
    uint8_t return_source;       /* default 0 */
} hgx_algen_opts;

/* One And{type?, incident*, orderedLink?} query after ExpressionBasedQuery.expand. */
typedef struct hgx_and_query {
    int32_t        type;         /* HGX_NO_TYPE or the AtomTypeCondition type key        */
    int32_t        n_incident;   /* IncidentCondition targets                           */
    const int32_t *incident;
    int32_t        has_ordered;  /* 0: no OrderedLinkCondition                          */
    int32_t        n_pattern;    /* OrderedLinkCondition targets (HGX_ANY_HANDLE = any) */
    const int32_t *pattern;
} hgx_and_query;

/* Device-timed breakdown of one hgx_bfs_batch (kernel times are filled when timing is enabled,
 * hgx_set_timing(g, 1)).  Per-kernel arrays are indexed by HGX_K_*.  Bytes are the algorithmic
 * bytes of the implemented kernels; bytes_survey follows SURVEY.md 8(d)'s
 * push model.  traversed_edges is the hyperedge-TEPS numerator
 * sum_s sum_{d<D} sum_{v in F_sd} |inc(v)|. */
#define HGX_K_LINK_GATHER   0   /* hgx_link_gather          */
#define HGX_K_ATOM_PULL     1   /* hgx_atom_pull            */
#define HGX_K_PULL_HEAVY    2   /* hgx_atom_pull_heavy      */
#define HGX_K_HUB_FINALIZE  3   /* hgx_hub_finalize         */
#define HGX_K_FRONTIER_PUSH 4   /* sparse levels: hgx_frontier_list, hgx_opush[_heavy], hgx_push_finalize_list */
#define HGX_K_NF_PULL       5   /* late dense levels: hgx_nonfull_list, hgx_nf_pull                        */
#define HGX_K_FC_PULL       6   /* dense levels over a small frontier: hgx_fc_slots, hgx_fc_codes, hgx_fc_pull */
#define HGX_K_FC_HEAVY      7   /*   and their hub chunks: hgx_fc_pull_heavy, then hgx_hub_finalize          */
#define HGX_K_COUNT         8
typedef struct hgx_bfs_stats {
    int32_t n_levels_expanded;
    int32_t n_batches;
    double  ms_total;                  /* first kernel -> last level counter D2H, device events */
    double  ms_kernel[HGX_K_COUNT];    /* summed over launches                                 */
    int64_t launches[HGX_K_COUNT];
    double  bytes_kernel[HGX_K_COUNT]; /* algorithmic bytes, summed over launches             */
    double  bytes_survey;
    double  traversed_edges;
    int64_t union_frontier[64];        /* |U_d| per expanded level (summed over batches)       */
    double  level_ms[64];              /* device ms of all kernels of level d (timing enabled) */
    int64_t level_new[64];             /* atoms with a new bit at level d+1 (summed over batches) */
    double  level_bytes[64];           /* algorithmic bytes of all kernels of level d          */
    int32_t level_sparse[64];          /* level d ran 0 = dense, 1 = frontier links + lf push, 2 = frontier push,
                                        * 3 = non-full pull, 4 = frontier-code pull */
    /* per level, summed over batches: [0] lf rows written, [1] frontier rows gathered,
     * [2] lf rows pulled (light), [3] vis rows read, [4] new light atoms, [5] lf rows pulled
     * (heavy chunks), [6] heavy atoms finalised, [7] new heavy atoms */
    int64_t level_rows[64][8];
    /* partitioned BFS (hgx_pbfs_batch): device ms of the per-level exchange (pack, transport,
     * apply, frontier count) and the row bytes this part sent (reduce + broadcast) */
    double  ms_exchange;
    double  bytes_exchanged;
    double  level_xbytes[64];          /* bytes this part sent at level d                      */
    double  level_xpair_max[64];       /* sum over the level's two exchange phases (reduce,     */
                                       /* broadcast) of the largest bytes sent to one part      */
    double  level_xms[64];             /* device ms of the exchange kernels of level d (timing on) */
    double  xwords_nonzero, xwords_total;   /* row words shipped: nonzero / all (compression headroom) */
    /* minimum-bytes model of the whole batch (with accounting): per expanded level, the CSR slices
     * of the frontier atoms or every CSR column once (whichever is less) + one S/8-byte row per
     * frontier atom read + one per new atom written */
    double  bytes_min;
    /* partitioned BFS: host round trips of level d's exchange (count / statistics read-backs and
     * count all-gathers; the row transfers are not counted), the largest over the parts' batches */
    int32_t level_xtrips[64];
    /* the workgroup-per-seed stage (HGX_OPT_BFS_BLOCK): device ms of its launches (timing on), their
     * algorithmic bytes, the seeds it finished and the seeds handed to the level engine */
    double  ms_block;
    double  bytes_block;
    int64_t block_seeds;
    int64_t block_rerun;
    /* the multi-workgroup stage that takes the workgroup stage's overflow (<= 64 seeds, one persistent
     * launch, a grid barrier per level): device ms, algorithmic bytes, seeds it finished (counted in
     * block_seeds too) */
    double  ms_coop;
    double  bytes_coop;
    int64_t block_coop;
    /* multi-workgroup launches whose grid barrier timed out (their workgroups were not all resident
     * within the limit): the bitmaps were cleared and the seeds ran on the rows engine instead */
    int64_t coop_fallbacks;
} hgx_bfs_stats;

const char *hgx_version(void);
const char *hgx_last_error(void);
/* hipDeviceSynchronize on one device (benchmark brackets; no graph needed). */
int hgx_device_synchronize(int32_t device);
/* Number of visible HIP devices (0 on a host without GPUs; never fails for that reason). */
int hgx_device_count(int32_t *n);

/* device: HIP device ordinal to place the snapshot on. */
int  hgx_graph_create(const hgx_graph_desc *desc, int32_t device, hgx_graph **out);
void hgx_graph_destroy(hgx_graph *g);
/* An execution context of g's snapshot: an hgx_graph that borrows the device arrays (no copy) but has
 * its own stream, lock, scratch pool, push accumulator, level counters and host staging, so
 * traversals and pattern batches on different contexts of one snapshot run concurrently on the device
 * (e.g. the hg.subsumed and hg.subsumes closures of one step, or the pool threads of
 * TC/query/QueryCompilation.java:76-122).  It takes the snapshot's options at the time of the call;
 * hgx_set_option / hgx_set_timing on it apply to it alone.  Release it with hgx_graph_destroy; it keeps
 * the snapshot alive, and hgx_graph_update is refused while a context exists.  Not for partition
 * shards (HGX_E_UNSUPPORTED). */
int  hgx_graph_context(hgx_graph *g, hgx_graph **out);
int  hgx_graph_info(const hgx_graph *g, int64_t *num_atoms, int64_t *num_links, int64_t *num_incidences);
/* |inc(atom)| for n atoms (HyperGraph.getIncidenceSet(h).size()). */
int  hgx_graph_degree(hgx_graph *g, const int32_t *atoms, int32_t n, int64_t *out_deg);
/* inc(atom) as link ATOM ids, ascending; *n_out = |inc(atom)| even when > cap. */
int  hgx_graph_incidence(hgx_graph *g, int32_t atom, int32_t *out, int64_t cap, int64_t *n_out);
int  hgx_set_timing(hgx_graph *g, int32_t enabled);
/* Engine options (tuning / A-B experiments; defaults are the tuned values):
 *   HGX_OPT_BFS_FLAGS: bit 0 = gather early exit, bit 1 = pull early exit,
 *                      bit 2 = skip atoms / links already visited by every traversal,
 *                      bit 3 = frontier-driven sparse levels (direction optimisation),
 *                      bit 4 = apply bit 2 only once >= 1/16 of the atoms are fully visited,
 *                      bit 5 = sparse levels of the symmetric mode push from the frontier atoms
 *                              (the ordered modes always do),
 *                      bit 6 = keep the one-row-at-a-time dense kernels for >= 512 sources
 *                              (A/B only; the default uses the tile-staged ones),
 *                      bit 7 = dense levels whose frontier covers the links twice write every lf row
 *                              and pull without the active-link probe,
 *                      bit 8 = dense levels with < 1/4 of the incidence on atoms not yet visited by
 *                              every traversal pull those atoms straight from the frontier rows,
 *                      bit 9 = ordered-mode push levels are pipelined: the next level is issued
 *                              before this level's counters reach the host,
 *                      bit 10 = the dense gather built for 5 waves/SIMD (spills VGPRs; diagnostic A/B only),
 *                      bit 11 = the dense pull keeps half of a lane group's rows in flight at
 *                              once (fewer VGPRs, more waves per SIMD; A/B only),
 *                      bits 12 / 13 / 14 = nontemporal loads of the streamed CSR columns / stores of
 *                              the gather's link rows / stores of the pull's atom rows (A/B only),
 *                      bit 15 = the symmetric-mode hub pull keeps two incidence chunks in flight
 *                              without the active-link probe in all-rows levels (A/B only),
 *                      bit 17 = symmetric-mode dense levels whose frontier rows fit the Infinity Cache
 *                              (<= 64 MB) pull through per-entry target records and coded frontier rows
 *                              instead of gather + pull (records: 32 bytes per incidence entry, built on
 *                              first use, at most 16 GiB; snapshots with links of arity > 8 keep gather + pull).
 *                      Default 0x3BE (bit 17 is an A/B: measured slower on config 2). */
#define HGX_OPT_BFS_FLAGS 1
/* HGX_OPT_SEQ_BUDGET: device bytes the order-exact traversal's level-synchronous engine may use for
 * its per-seed key arrays (seeds are processed in chunks that fit; default 48 GiB). */
#define HGX_OPT_SEQ_BUDGET 2
/* HGX_OPT_RANKS_ORDERED: 1 = the rank order equals the persistent-handle order (the default for a
 * fresh snapshot).  An hgx_graph_update that extends the rank space sets it to 0: appended ranks
 * sort after every existing rank, which is handle order only if the new handles sort after the old
 * ones (true for IntHandleFactory's sequential handles, C/handle/IntHandleFactory.java:32-49; not
 * for random UUIDs).  Result SETS stay correct (the shim re-sorts ids >= the old count by handle),
 * but the FIFO order of hgx_bfs_sequence and its discovering links follow the incidence order and
 * cannot be repaired afterwards, so hgx_bfs_sequence returns HGX_E_UNSUPPORTED until the caller
 * re-asserts 1 (or re-exports the snapshot). */
#define HGX_OPT_RANKS_ORDERED 3
int  hgx_set_option(hgx_graph *g, int32_t option, int64_t value);

/* ---- the snapshot on disk (.hgcsr) and batched store updates ------------------------------------
 * The exporter walks the store once -- atom handles from
 * IndexScanQuery(indexByType) (C/query/cond2qry/ToQueryMap.java:101-113), link layouts from
 * HGStore.getLink (C/HGStore.java:179-191) -- ranks the handles and writes the bipartite CSR with
 * hgx_snapshot_write; a later process maps it with hgx_graph_open instead of re-walking the store.
 * File layout (little-endian, 64-byte aligned sections): 64-byte header (magic "HGXCSR1\0",
 * version 1, flags, num_atoms, num_links, num_pins, handle_bytes, checksum), link_atom i32[M],
 * tgt_off i64[M+1], tgt_idx i32[P], link_type i32[M] (if present), handles u8[A*handle_bytes]
 * (if present: the persistent handle bytes of every rank, so ranks map back to handles).
 * The writer validates the rows like hgx_graph_create and replaces the file atomically. */
int hgx_snapshot_write(const char *path, const hgx_graph_desc *desc, const uint8_t *handles,
                       int32_t handle_bytes);
/* The same file written in pieces: begin writes the header and the row sections, handles appends
 * n_ranks handles (rank order; call it until num_atoms handles are written, or never for
 * handle_bytes 0), end writes the checksum and replaces the file atomically; abort (or a failed end)
 * removes the partial file.  For exporters whose handle table does not fit one buffer (a Java byte[]
 * stops at 2^31 bytes: 134M 16-byte UUIDs; config 4 has 300M atoms). */
typedef struct hgx_snapshot_writer hgx_snapshot_writer;
int  hgx_snapshot_writer_begin(const char *path, const hgx_graph_desc *desc, int32_t handle_bytes,
                               hgx_snapshot_writer **out);
int  hgx_snapshot_writer_handles(hgx_snapshot_writer *w, const uint8_t *handles, int64_t n_ranks);
/* The writer's handle width (begin's handle_bytes): a binding that receives a byte array sizes the
 * rank count from this, not from a width the caller passes again. */
int  hgx_snapshot_writer_handle_bytes(const hgx_snapshot_writer *w, int32_t *handle_bytes);
int  hgx_snapshot_writer_end(hgx_snapshot_writer *w);   /* frees w */
void hgx_snapshot_writer_abort(hgx_snapshot_writer *w);
/* Header fields without reading the sections (any output may be NULL). */
int hgx_snapshot_info(const char *path, int64_t *num_atoms, int64_t *num_links, int64_t *num_pins,
                      int32_t *handle_bytes, int32_t *has_types);
/* Checksum-verified copy of the sections into caller buffers sized from hgx_snapshot_info (NULL
 * skips a section; link_type is zero-filled when the file has none). */
int hgx_snapshot_read(const char *path, int32_t *link_atom, int64_t *tgt_off, int32_t *tgt_idx,
                      int32_t *link_type, uint8_t *handles);
/* Handles of ranks [first_rank, first_rank + n) (n * handle_bytes bytes) from the file's handle table,
 * for readers that cannot hold the whole table at once (a Java byte[] stops at 2^31 bytes: 134M
 * 16-byte UUID handles).  verify = 1 also checks the whole file's checksum -- on EVERY call made with it
 * (the call keeps no state), so a paged reader verifies once (the first range, or hgx_graph_open / the
 * JNI snapshotVerify) and reads the other ranges with verify = 0;
 * HGX_E_NOTFOUND when the file has no handle table, HGX_E_INVALID for ranks outside [0, num_atoms). */
int hgx_snapshot_read_handles(const char *path, int64_t first_rank, int64_t n, int32_t verify, uint8_t *out);
/* Map + verify the file and build the device snapshot (as hgx_graph_create). */
int hgx_graph_open(const char *path, int32_t device, hgx_graph **out);
/* D2H copy of the snapshot rows currently on the device (sizes from hgx_graph_info; num_pins =
 * tgt_off[num_links]).  Any output may be NULL. */
int hgx_graph_export(hgx_graph *g, int32_t *link_atom, int64_t *tgt_off, int32_t *tgt_idx, int32_t *link_type);
/* Apply one batch of store events to a device snapshot: HGAtomAddedEvent for links (n_add rows in
 * hgx_graph_desc form: link atom, offsets into add_tgt_idx, type) and HGAtomRemovedEvent for links
 * (their atom ids) (C/event/HGAtomAddedEvent.java, C/event/HGAtomRemovedEvent.java; the store
 * sides are HGStore.store/removeLink, C/HGStore.java:100-170).  New atoms extend the rank space
 * to num_atoms (>= the current count; the exporter assigns new atoms ranks after the existing
 * ones).  An added link must not exist yet; removing an absent link is a no-op, as a removal of a
 * link already gone is in the store.  The incidence index is rebuilt from the merged rows (same
 * device object, same handle).  Refused while a result of this graph is alive. */
int hgx_graph_update(hgx_graph *g, int64_t num_atoms, int64_t n_add, const int32_t *add_link_atom,
                     const int64_t *add_tgt_off, const int32_t *add_tgt_idx, const int32_t *add_link_type,
                     int64_t n_remove, const int32_t *remove_link_atom);

/* Batched multi-source BFS.  Seed i is HGBreadthFirstTraversal(seeds[i], gen, max_depth)
 * (max_depth HGX_UNBOUNDED = Integer.MAX_VALUE).  The result holds, per seed and per
 * distance d, the set V_d of atoms returned by next() at distance d (V_0 = {seed}),
 * which is the reference's per-depth visited set. */
int  hgx_bfs_batch(hgx_graph *g, const int32_t *seeds, int32_t n_seeds, int32_t max_depth,
                   const hgx_algen_opts *opts, hgx_bfs_result **out);
/* n_levels = 1 + the largest distance reached by any seed. */
int  hgx_bfs_result_info(const hgx_bfs_result *r, int32_t *n_seeds, int32_t *n_levels);
/* counts[i * n_levels + d] = |V_d| of seed i: the batch's result readout (one counting launch per
 * level over the device rows, one D2H; cheap enough to sit inside a timed step). */
int  hgx_bfs_result_counts(hgx_bfs_result *r, int64_t *counts);
/* V_d of seed i, ascending atom ids; *n_out = |V_d| even when > cap. */
int  hgx_bfs_result_visited(hgx_bfs_result *r, int32_t seed_index, int32_t depth,
                            int32_t *out, int64_t cap, int64_t *n_out);
/* The same list from position first on: out[0, min(cap, *n_out - first)) = V_d[first, ...); *n_out = |V_d|
 * (paged readers of sets larger than one Java array). */
int  hgx_bfs_result_visited_range(hgx_bfs_result *r, int32_t seed_index, int32_t depth, int64_t first,
                                  int32_t *out, int64_t cap, int64_t *n_out);
/* isVisited after draining (C/algorithms/HGBreadthFirstTraversal.java:137-141):
 * *depth_out = distance of atom from seed i, or -1 when never reached. */
int  hgx_bfs_result_depth_of(hgx_bfs_result *r, int32_t seed_index, int32_t atom, int32_t *depth_out);
/* with_accounting = 0: timing and algorithmic bytes only (cheap); 1: also run the accounting
 * kernels for traversed_edges, bytes_survey and union_frontier (reads every level once). */
int  hgx_bfs_result_stats(hgx_bfs_result *r, int32_t with_accounting, hgx_bfs_stats *stats);
void hgx_bfs_result_free(hgx_bfs_result *r);

/* Order-exact traversal: for every seed the exact sequence of (link, atom) pairs that
 * HGBreadthFirstTraversal(seeds[i], gen, max_depth).next() returns, in the reference's FIFO order
 * (C/algorithms/HGBreadthFirstTraversal.java:49-66,143-156), plus the distance of each atom.
 * The link of a pair is the link through which the atom was first discovered.
 * Large results may still be arriving from the device when hgx_bfs_sequence returns: the readers
 * (hgx_seq_result_pairs / _pairs_range) wait for the part they read, the stats functions for the timing,
 * and hgx_seq_result_free for every copy; a later call on the same graph is ordered after them. */
typedef struct hgx_seq_result hgx_seq_result;
int  hgx_bfs_sequence(hgx_graph *g, const int32_t *seeds, int32_t n_seeds, int32_t max_depth,
                      const hgx_algen_opts *opts, hgx_seq_result **out);
/* n_pairs = total pairs over all seeds; n_levels = 1 + the largest distance returned. */
int  hgx_seq_result_info(const hgx_seq_result *r, int32_t *n_seeds, int64_t *n_pairs, int32_t *n_levels);
/* offsets[n_seeds+1]: seed i's pairs are [offsets[i], offsets[i+1]) of the pair arrays. */
int  hgx_seq_result_offsets(const hgx_seq_result *r, int64_t *offsets);
/* links / atoms / dists: n_pairs entries each (any may be NULL). */
int  hgx_seq_result_pairs(const hgx_seq_result *r, int32_t *links, int32_t *atoms, int32_t *dists);
/* Pairs [first, first + n) of the flattened pair arrays (paged readers; n may run past the end: only
 * the pairs that exist are copied, *n_out says how many). */
int  hgx_seq_result_pairs_range(const hgx_seq_result *r, int64_t first, int64_t n, int32_t *links, int32_t *atoms,
                                int32_t *dists, int64_t *n_out);
/* device ms (timing enabled) and sum over seeds and expanded atoms of |inc(atom)|. */
int  hgx_seq_result_stats(const hgx_seq_result *r, double *ms_total, double *traversed_edges);
/* Which engine finished the seeds (HGX_OPT_SEQ_ENGINE): seeds done by the workgroup-per-seed engine /
 * by the level-synchronous one (the overflow reruns), the device ms of the workgroup launches (from the
 * call's first operation to their end; timing enabled) and their algorithmic bytes (streamed yield
 * flags, the staged entries' type / row / target-offset / link-id / target loads, frontier offsets,
 * pairs written).  Any output may be NULL. */
int  hgx_seq_result_engine_stats(const hgx_seq_result *r, int32_t *n_block, int32_t *n_level, double *ms_block,
                                 double *bytes_block);
/* The order-exact grid stage (one persistent launch for <= 64 of the seeds the workgroup engine handed
 * over, when the generator has a yield adjacency: ordered modes or a link type): seeds it finished, its
 * device ms (timing enabled) and algorithmic bytes.  Any output may be NULL. */
int  hgx_seq_result_grid_stats(const hgx_seq_result *r, int32_t *n_seeds, double *ms, double *bytes);
/* The level-synchronous engine's part of the call (the seeds the workgroup engine handed over):
 * device ms from its first operation to its last (timing enabled; it includes the pairs' copy to the
 * host), its algorithmic bytes (kernel counters: per item its entry, row, type, target offsets and
 * targets, per yield the examined word and the hash slot; per pulled atom its incidence range, examined
 * row, entries, link rows, union bits, frontier rows, pin indices and hash probes; the frontier
 * entries of the pull tables), and how many of its levels ran as pulls.  Any output may be NULL. */
int  hgx_seq_result_level_stats(const hgx_seq_result *r, double *ms_level, double *bytes_level, int64_t *pull_levels);
void hgx_seq_result_free(hgx_seq_result *r);
/* Batched conjunctive pattern queries.  Result of query q = the link atoms L with
 * type(L) == type, every incident/pattern anchor in targets(L) and
 * OrderedLinkCondition(pattern) true on targets(L), ascending.  A query with no
 * incidence anchor returns HGX_E_UNSUPPORTED for the whole batch (the caller keeps
 * AndToQuery, which scans the type index). */
int  hgx_pattern_batch(hgx_graph *g, const hgx_and_query *queries, int32_t n,
                       hgx_query_result **out);
/* The same batch as flat arrays (one call per batch from JNI / FFM): query q has type[q],
 * incident anchors inc[inc_off[q] .. inc_off[q+1]), has_ordered[q], and ordered pattern
 * pat[pat_off[q] .. pat_off[q+1]). */
int  hgx_pattern_batch_packed(hgx_graph *g, int32_t n, const int32_t *type, const int64_t *inc_off,
                              const int32_t *inc, const int32_t *has_ordered, const int64_t *pat_off,
                              const int32_t *pat, hgx_query_result **out);
/* A packed batch resident in device memory: uploaded once (validated like hgx_pattern_batch_packed)
 * and run any number of times without moving the queries again -- an application re-running a fixed
 * set of compiled queries (the reference compiles a query once and executes it repeatedly,
 * TC/query/QueryCompilation.java:76-122), and the bench's config-3 step with its inputs resident in
 * HBM.  The set belongs to the device of g; it may be run on any graph or execution context of that
 * device.  Results as hgx_pattern_batch.  Every per-run word lives in the running graph's scratch, so one
 * set may run on several graphs / contexts at the same time (round 5: the A/B paths that kept an error
 * slot in the set itself are gone). */
typedef struct hgx_query_set hgx_query_set;
int  hgx_query_set_create(hgx_graph *g, int32_t n, const int32_t *type, const int64_t *inc_off, const int32_t *inc,
                          const int32_t *has_ordered, const int64_t *pat_off, const int32_t *pat,
                          hgx_query_set **out);
int  hgx_pattern_batch_set(hgx_graph *g, const hgx_query_set *qs, hgx_query_result **out);
/* The same run with the results written into caller buffers (no result object): offsets[n + 1] always,
 * ids when the hits fit in ids_cap; *n_ids = the number of hits (call again with a larger buffer when
 * it exceeds ids_cap).  The single-pass back end copies straight from the mapped result area.
 * timing (optional, double[3]): what hgx_query_ms reports for a result object -- device ms of the batch,
 * ms of the match kernel, its algorithmic bytes (zeros unless hgx_set_timing is on). */
int  hgx_pattern_batch_set_into(hgx_graph *g, const hgx_query_set *qs, int64_t *offsets, int32_t *ids, int64_t ids_cap,
                                int64_t *n_ids, double *timing);
/* The number of queries of a set (the size of a run's offsets is n_queries + 1). */
int  hgx_query_set_info(const hgx_query_set *qs, int32_t *n_queries);
void hgx_query_set_free(hgx_query_set *qs);
/* The And shapes beyond {type, incident, orderedLink} (flat arrays, one call per batch).  Query q is
 *   And{ Or over types[type_off[q] .. type_off[q+1])        AtomTypeCondition (one type) or
 *                                                          TypePlusCondition (base + subtypes, expanded to an
 *                                                          Or, C/query/cond2qry/ExpressionBasedQuery.java:606-627);
 *                                                          none = no type condition,
 *        IncidentCondition(inc[inc_off[q] .. inc_off[q+1]))  (also LinkCondition targets, :739-746),
 *        PositionedIncidentCondition(target, lb, ub, complement) for the 4-int records
 *                 pos[4k .. 4k+4), k in [pos_off[q], pos_off[q+1])
 *                 (C/query/PositionedIncidentCondition.java:123-177, PositionedIncidentToQuery.java),
 *        OrderedLinkCondition(pat[pat_off[r] .. pat_off[r+1])) for r in [pset_off[q], pset_off[q+1]),
 *        ArityCondition(arity[q]) unless arity[q] < 0 (C/query/ArityCondition.java:49-67) }.
 * Every query needs an incidence anchor (an incident target, a non-ANY pattern target or a positioned
 * target), else HGX_E_UNSUPPORTED for the batch.  Results as hgx_pattern_batch. */
int  hgx_pattern_batch_ext(hgx_graph *g, int32_t n, const int64_t *type_off, const int32_t *types,
                           const int64_t *inc_off, const int32_t *inc, const int64_t *pos_off, const int32_t *pos,
                           const int64_t *pset_off, const int64_t *pat_off, const int32_t *pat,
                           const int32_t *arity, hgx_query_result **out);
/* n = the number of queries of the batch (the size of offsets is n + 1). */
int  hgx_query_result_count(const hgx_query_result *r, int64_t *n_queries);
/* offsets[n+1]: results of query q are ids[offsets[q] .. offsets[q+1]). */
int  hgx_query_result_offsets(const hgx_query_result *r, int64_t *offsets);
int  hgx_query_result_ids(const hgx_query_result *r, int32_t *ids);
/* device milliseconds of the last pattern batch (timing enabled). */
int  hgx_query_result_ms(const hgx_query_result *r, double *ms_total, double *ms_match, double *bytes_match);
void hgx_query_result_free(hgx_query_result *r);

/* ---------------------------------------------------------------------------------------------
 * Partitioned snapshot and BFS (config 4: graphs sharded over the GPUs of a node).
 *
 * Replaces the same HGBreadthFirstTraversal/DefaultALGenerator loop as hgx_bfs_batch
 * (C/algorithms/HGBreadthFirstTraversal.java:49-66, C/algorithms/DefaultALGenerator.java:287-315)
 * when the incidence index (HGStore.getIncidenceResultSet, C/HGStore.java:253) is split over
 * n_parts devices.  Vertex cut: every link row lives on exactly one part (link_part[r]); an atom is
 * present on every part that holds one of its links and is owned by one of them.  Each level every
 * part expands its own links, ships its partial news for atoms owned elsewhere to their owners
 * (reduce) and each owner ships the final news back to the other holders (broadcast).  Results are
 * bit-identical to hgx_bfs_batch on the whole graph.
 * -------------------------------------------------------------------------------------------- */
typedef struct hgx_shard hgx_shard;   /* host-side partition of one part */
typedef struct hgx_comm hgx_comm;     /* the group's transport            */

/* Link placement over n_parts (1..64): greedy streaming vertex cut (a link goes to the part that
 * already holds most of its low-degree targets, within a 2% pin-balance cap).  Deterministic: every
 * rank computes the same link_part[num_links] from the same snapshot.  Host only. */
int  hgx_partition_plan(const hgx_graph_desc *global, int32_t n_parts, int32_t *link_part);
/* Build part `part` of n_parts for a placement (host only, no device work). */
int  hgx_shard_build(const hgx_graph_desc *global, int32_t n_parts, int32_t part, const int32_t *link_part,
                     hgx_shard **out);
/* n_local = atoms present on this part (owned + ghosts); local links / pins = this part's link rows. */
int  hgx_shard_info(const hgx_shard *s, int64_t *n_local, int64_t *n_owned, int64_t *n_local_links,
                    int64_t *n_local_pins);
/* Copies of the local tables (any pointer may be NULL): l2g[n_local] global id of each local atom
 * (ascending); link_atom/link_type[n_local_links] global link atom id / type of each local link;
 * tgt_off[n_local_links+1], tgt_idx[n_local_pins] targets in LOCAL ids; ghost_count[n_parts] = my
 * ghosts owned by each part. */
int  hgx_shard_export(const hgx_shard *s, int32_t *l2g, int32_t *link_atom, int32_t *link_type,
                      int64_t *tgt_off, int32_t *tgt_idx, int64_t *ghost_count);
/* The exchange tables: xo_part/xo_lid[n_local] = owner part and the atom's local id there (-1 for
 * owned atoms); bc_off[n_local+1] / bc_part / bc_lid = for each owned atom its other holders and
 * its local id on each (bc_off[n_local] entries); bc_count[n_parts] = entries per part. */
int  hgx_shard_exchange_tables(const hgx_shard *s, int32_t *xo_part, int32_t *xo_lid, int64_t *bc_off,
                               int32_t *bc_part, int32_t *bc_lid, int64_t *bc_count);
void hgx_shard_free(hgx_shard *s);
/* Upload a part to a device (incidence build as in hgx_graph_create).  The result is an hgx_graph
 * that only hgx_pbfs_batch / hgx_pbfs_batch_group (+ the hgx_bfs_result_* readers) accept.
 * hgx_set_option(shard_graph, HGX_OPT_PART_SERIAL, 1) makes an in-process group run its parts'
 * device work one part at a time (clean per-part device times for a one-GPU rehearsal). */
int  hgx_shard_graph_create(const hgx_shard *s, int32_t device, hgx_graph **out);
#define HGX_OPT_PART_SERIAL 4
/* HGX_OPT_QUERY_FUSED: removed in round 5.  The fused small-batch path (a wavefront per query expands,
 * plans and matches; three launches) measured slower than the general path on config 3 (0.318 vs 0.211 ms
 * wall, profiles/r02v_pattern_ab.log).  hgx_set_option accepts 0 only (HGX_E_UNSUPPORTED otherwise). */
#define HGX_OPT_QUERY_FUSED 5
/* HGX_OPT_QUERY_INLINE (default 1): the type-grouped incidence index carries each link's <= 8
 * targets inline (32 bytes per incidence entry, built with the index on the first pattern query),
 * so a typed candidate is one streamed record instead of two dependent random rows.  0 = read the
 * target rows through tgt_off (A/B; also what a snapshot too large for the extra bytes gets). */
#define HGX_OPT_QUERY_INLINE 6
/* HGX_OPT_PUSH_BATCH: removed in round 5.  K > 0 gave each wavefront of a frontier-push level K atoms
 * at once; config 5 wall ms per direction subsumed / subsumes (profiles/r02zg_c5_push_ab.jsonl): K = 4,
 * 8, 16 1.68 / 2.15, 1.65 / 2.17, 1.67 / 2.48 against 1.71 / 2.05 with one wavefront per atom -- slower
 * on the sum.  hgx_set_option accepts 0 only (HGX_E_UNSUPPORTED otherwise). */
#define HGX_OPT_PUSH_BATCH 7
/* HGX_OPT_PART_EXCHANGE (partition shards; every part of a group must use the same value -- the
 * partitioned BFS checks it collectively before any exchange and fails with HGX_E_INVALID on every
 * part when they differ): 0 or 1 = compressed records (the only format since round 5).  2 = static
 * slots (every ghost's whole row to a fixed slot of its owner) was removed: 42.8 against 34.0 ms per
 * part a step on full config 4 at 8 parts (profiles/r02ze_part_c4x1.json); HGX_E_UNSUPPORTED. */
#define HGX_OPT_PART_EXCHANGE 8
/* HGX_OPT_QUERY_FLAT (2, the only value since round 5): pattern batches match over the batch's flat
 * candidate space, a wavefront per 64 candidates and a lane per candidate whatever query it belongs
 * to, in a single pass: two kernels per batch (normalise + plan + candidate scan with a decoupled
 * look-back; match + hit offsets with a decoupled look-back + result placement).  The A/B back ends 1
 * (separate single-workgroup scan, finish and scatter) and 0 (a wavefront per chunk of one query's
 * candidates) measured slower and were removed; they return HGX_E_UNSUPPORTED. */
#define HGX_OPT_QUERY_FLAT 9
/* HGX_OPT_CODED: removed in round 5.  Coded dense levels (rows of <= 6 source bits as 64-bit codes) were
 * exact but measured slower on config 2's level 1 (16.0 vs 9.0 ms, profiles/r02zn_*_c2_levels.log;
 * DESIGN.md 3.1 item 8b).  hgx_set_option accepts 0 only (HGX_E_UNSUPPORTED otherwise). */
#define HGX_OPT_CODED 10
/* HGX_OPT_QUERY_COALESCE (default 1 = on): concurrent hgx_pattern_batch_packed calls on one graph
 * share device batches.  A caller that finds the device busy queues its batch; the next caller to
 * run takes every queued batch (FIFO, up to 65536 queries; a value > 1 sets that cap) and runs them
 * as ONE batch, then splits the result -- the reference's usage is many threads each executing small
 * compiled queries (QueryCompilation.java:76-122).  Results and errors are exactly those of separate
 * calls (a batch whose merged run reports a bad or unsupported query is re-run on its own).  0 = off. */
#define HGX_OPT_QUERY_COALESCE 11
/* HGX_OPT_PUSH_INLINE: removed in round 5.  Inline target records in incidence order for the frontier
 * push measured no faster on config 5 (profiles/r03n_c5.log) and cost 32 bytes per incidence entry.
 * hgx_set_option accepts 0 only (HGX_E_UNSUPPORTED otherwise). */
#define HGX_OPT_PUSH_INLINE 12
/* HGX_OPT_SEQ_ENGINE (default 0): how hgx_bfs_sequence runs.  0 = one workgroup per seed with the
 * whole traversal in LDS (hash of the examined atoms, frontier and discovery ranks on chip, pairs
 * written into mapped host memory; one launch per 1024 seeds, no host round trip per level), seeds
 * whose traversal outgrows the workgroup's 2046 pairs rerun on the level-synchronous engine (six
 * fixed-grid kernels a level that read every size from device memory; the host polls each level's
 * size one level behind; discoveries ranked by a bitmap over the level's key space);
 * 1 = every seed on the round-1 key-array engine (rocPRIM sort, two host round trips a level; A/B);
 * 2 = every seed on the level-synchronous engine (tests). */
#define HGX_OPT_SEQ_ENGINE 13
/* HGX_OPT_BFS_BLOCK (default 1): hgx_bfs_batch on a whole snapshot first runs every seed in one
 * workgroup (its visited set, frontier and staging in LDS, all its levels in one launch; V_d written
 * into mapped host memory); the seeds whose traversal outgrows the workgroup (more than 1534 atoms,
 * a level wider than 1024 atoms, or a frontier of more than 4M incidence entries) then run on the
 * batched rows engine -- up to 64 of them first on the multi-workgroup stage (one persistent launch,
 * a grid barrier per level, per-seed visited bitmaps).  0 = every seed on the rows engine; 2 (tests) =
 * a batch of <= 64 seeds straight to the multi-workgroup stage.  Results are identical either way.
 * Memory: in an ordered generator mode, or with a link type, both stages and hgx_bfs_sequence's
 * workgroup engine build on first use (kept on the snapshot, shared by its contexts, dropped by
 * hgx_graph_update) the generator's output per atom for that (mode, type, minimum arity, order):
 * (A + 1) * 8 bytes of offsets + 8 bytes per yielded (target, link) pair, skipped above 4 GB; and a
 * list of the entries that can yield, (A + 1) * 8 + 4 per entry.  At most 8 of each per snapshot. */
#define HGX_OPT_BFS_BLOCK 14
/* Test and diagnostic options (per graph; an execution context takes its snapshot's values when made).
 * The library reads no tuning knob from the environment (only tracing switches); the
 * measured-negative A/B variants live in A/B builds only (tools/build_variant.sh).
 *   HGX_OPT_CO_TIMEOUT   the grid stages' barrier limit in s_memrealtime ticks (100 MHz); 0 = 1 s.  A few
 *                        ticks force the fallback path (the seeds rerun on the other engine, exact).
 *   HGX_OPT_SEQ_PULL     order-exact level engine: 0 = push every level, 1 = pull wide levels (default),
 *                        2 = pull every level.
 *   HGX_OPT_SEQ_SMALL    1 = the level engine starts from tiny capacities (every growth path runs).
 *   HGX_OPT_SEQ_TLIMIT   > 0 lowers the level engine's per-chunk stream-key limit (exercises chunk splits).
 *   HGX_OPT_SEQ_PACK_MIN levels of at least this many pairs cross PCIe packed (0 = 2^20).
 *   HGX_OPT_XB_FLAT      partition shards: the broadcast pack walks owned atoms (0), takes the broadcast
 *                        entries on dense levels (1) or on every level (2); -1 = default (1).
 *   HGX_OPT_XB_STATIC    partition shards: static broadcast never (0), when the group's reduce says so (1),
 *                        every level (2); -1 = default (1).  Every part of a group must use the same value. */
#define HGX_OPT_CO_TIMEOUT   15
#define HGX_OPT_SEQ_PULL     16
#define HGX_OPT_SEQ_SMALL    17
#define HGX_OPT_SEQ_TLIMIT   18
#define HGX_OPT_SEQ_PACK_MIN 19
#define HGX_OPT_XB_FLAT      20
#define HGX_OPT_XB_STATIC    21
/* Coalescing statistics of a graph since its creation: device batches run by the packed pattern path
 * and caller batches they served (caller / device = the mean coalescing factor). */
int  hgx_query_coalesce_stats(hgx_graph *g, int64_t *device_batches, int64_t *caller_batches);

/* RCCL transport between processes (one GPU each): rank 0 calls hgx_comm_rccl_unique_id and
 * broadcasts the 128 bytes out of band; every rank then calls hgx_comm_rccl_create. */
int  hgx_comm_rccl_unique_id(uint8_t id[128]);
int  hgx_comm_rccl_create(const uint8_t id[128], int32_t world, int32_t rank, int32_t device, hgx_comm **out);
/* Host-staged transport: the collectives are callbacks on HOST buffers (return 0 on success).
 * allgather: out[r*n + i] = in[i] of rank r.  alltoallv: rank p receives send_bytes[p] bytes of
 * send + send_off[p]; this rank receives recv_bytes[p] bytes from rank p into recv + recv_off[p]. */
typedef int (*hgx_host_allgather_fn)(void *user, const int64_t *in, int64_t n, int64_t *out);
typedef int (*hgx_host_alltoallv_fn)(void *user, const void *send, const int64_t *send_off,
                                     const int64_t *send_bytes, void *recv, const int64_t *recv_off,
                                     const int64_t *recv_bytes);
int  hgx_comm_host_create(int32_t world, int32_t rank, hgx_host_allgather_fn allgather,
                          hgx_host_alltoallv_fn alltoallv, void *user, hgx_comm **out);
void hgx_comm_destroy(hgx_comm *c);
/* Diagnostics of a transport's all-gathers (collective: every rank of the group calls it with its own
 * n values): out_dev = the device-input all-gather the exchange's count vectors take
 * (Transport::allgather_dev: RCCL gathers on the device and reads the block back once), out_base = the
 * same through the default read-back + host all-gather, out_host = the host-input all-gather; each
 * n * world values, rank r's at [r * n, (r + 1) * n).  For tests: the RCCL-only override is compared
 * with the default path on the same inputs. */
int  hgx_comm_check_allgather(hgx_comm *c, int32_t device, const int64_t *values, int64_t n, int64_t *out_dev,
                              int64_t *out_base, int64_t *out_host);

/* One part's share of a partitioned batched BFS (collective: every part calls it with the same
 * seeds, depth and options).  seeds are GLOBAL atom ids.  The result reports this part's OWNED
 * atoms: counts are partial (sum them over parts), visited lists hold global ids (disjoint over
 * parts), depth_of accepts only atoms this part owns (else HGX_E_NOTFOUND); the TEPS numerator of
 * the stats sums over parts to the whole graph's. */
int  hgx_pbfs_batch(hgx_graph *shard, hgx_comm *comm, const int32_t *seeds, int32_t n_seeds,
                    int32_t max_depth, const hgx_algen_opts *opts, hgx_bfs_result **out);
/* All parts in this process: shards[p] is part p (any devices, including one device for all);
 * runs one host thread per part over an in-process transport.  outs[p] receives part p's result. */
int  hgx_pbfs_batch_group(hgx_graph *const *shards, int32_t n_parts, const int32_t *seeds, int32_t n_seeds,
                          int32_t max_depth, const hgx_algen_opts *opts, hgx_bfs_result **outs);

#ifdef __cplusplus
}
#endif
#endif
