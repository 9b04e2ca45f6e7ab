/*
 * hgx_oracle.h -- TEST INFRASTRUCTURE, NOT PRODUCT CODE.
 *
 * A plain-C restatement of the reference (BalterNotz/hypergraphdb, Java) CPU
 * algorithms on the accelerated path.  It is the parity checker for the HIP
 * engine in hypergraphdb_amd/ and the CPU baseline timed by bench.py.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library.  The product path (libhgx.so) never links or calls it.
 *
 * Parity status: the reference is Java and cannot be compiled or run here
 * (no JDK).  This restatement is pinned by the
 * known-answer tests held in the reference's own test-suite (rebuilt as
 * fixtures in tests/golden/) and cross-checked against a second, independent
 * Python restatement (oracle/pyref.py).  BFS visitation ORDER and large-graph
 * result sets are not pinned by any reference test ("parity unpinned" for
 * those aspects).
 *
 * Paths below are relative to the reference root; C = core/src/java/org/hypergraphdb.
 */
#ifndef HGX_ORACLE_H
#define HGX_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* In-memory model of a snapshot.  Atoms (nodes AND links) are ids 0..A-1,
 * equal to their rank in persistent-handle byte order (C/handle/UUID.java:364-376,
 * C/storage/BAUtils.java:55-80).  Link row r (0..M-1) is atom link_atom[r];
 * its layout is [type, value, t0..tk-1] (C/HyperGraph.java:1603-1608), of which
 * the oracle keeps type (link_type[r]) and the targets tgt_idx[tgt_off[r]..tgt_off[r+1]). */
typedef struct og_graph {
    int64_t A, M;
    const int32_t *link_atom;   /* [M] strictly ascending atom ids           */
    const int64_t *tgt_off;     /* [M+1]                                     */
    const int32_t *tgt_idx;     /* [P] target atom ids in layout order        */
    const int32_t *link_type;   /* [M] or NULL (all type 0)                  */
    /* built by og_graph_build */
    int32_t *atom_row;          /* [A] link row of an atom, -1 for a node     */
    int64_t *inc_off;           /* [A+1]                                     */
    int32_t *inc_atom;          /* [I] incident LINK ATOM ids, ascending      */
    /* type index (HGIndexManager.getIndexByType, restricted to links): link atoms of type t
     * are type_atoms[type_off[t] .. type_off[t+1]), ascending; types 0..n_types-1 */
    int64_t n_types;
    int64_t *type_off;
    int32_t *type_atoms;
} og_graph;

/* Builds the incidence index exactly as the BJE store would hold it:
 * one entry per (target, link) even when the target repeats in the link
 * (putNoDupData, storage/bdb-je/.../BJEStorageImplementation.java:300-307),
 * sorted ascending by handle (sorted duplicates, :109-111).  Returns 0 on success. */
int  og_graph_build(og_graph *g, int64_t A, int64_t M, const int32_t *link_atom,
                    const int64_t *tgt_off, const int32_t *tgt_idx, const int32_t *link_type);
void og_graph_free(og_graph *g);
int64_t og_inc_size(const og_graph *g, int32_t atom);
int64_t og_inc_copy(const og_graph *g, int32_t atom, int32_t *out, int64_t cap);

/* DefaultALGenerator options (C/algorithms/DefaultALGenerator.java:437-502).
 * link_type < 0: linkPredicate == null, else AtomTypeCondition(link_type) on the
 * incident link.  siblingPredicate is always null (not supported on the GPU). */
typedef struct og_algen {
    int32_t link_type;
    int32_t preceding, succeeding, reverse, source;
} og_algen;

/* DefaultALGenerator.generate(src): writes the (link atom, target atom) pairs in
 * the reference iteration order.  Returns the number of pairs (may exceed cap). */
int64_t og_generate(const og_graph *g, const og_algen *o, int32_t src,
                    int32_t *out_link, int32_t *out_atom, int64_t cap);

/* HGBreadthFirstTraversal(seed, gen, max_dist) drained through next()
 * (C/algorithms/HGBreadthFirstTraversal.java:42-66,143-156).
 * max_dist < 0 means Integer.MAX_VALUE.  Writes the returned (link, atom) pairs
 * and their distance in FIFO order.  Returns the count (may exceed cap).
 * *traversed (optional) receives sum over expanded atoms of |inc(atom)|. */
int64_t og_bfs(const og_graph *g, const og_algen *o, int32_t seed, int32_t max_dist,
               int32_t *out_link, int32_t *out_atom, int32_t *out_dist, int64_t cap,
               int64_t *traversed);

/* Many independent traversals (the CPU baseline): per seed, counts of atoms
 * returned at each distance 1..max_levels-1 (index 0 = the seed itself, always 1).
 * counts is [n_seeds * max_levels].  traversed[n_seeds] receives the hyperedge
 * TEPS numerator per seed.  nthreads <= 0: all cores (OpenMP).
 * time_budget_s > 0 bounds the sample: a traversal still running that long after the
 * call started stops (its counts/traversed are then partial); *elapsed_s receives the
 * wall time of the call. */
int og_bfs_many(const og_graph *g, const og_algen *o, const int32_t *seeds, int32_t n_seeds,
                int32_t max_dist, int32_t max_levels, int64_t *counts, int64_t *traversed,
                int32_t nthreads, double time_budget_s, double *elapsed_s);

/* OrderedLinkCondition.satisfies on a link's target array
 * (C/query/OrderedLinkCondition.java:92-124); pattern entries < 0 are hg.anyHandle(). */
int og_ordered_link(const int32_t *tgts, int32_t arity, const int32_t *pattern, int32_t m);

/* hg.and(hg.type(T)?, hg.incident(a_i)..., hg.orderedLink(p_0..p_m-1)?) compiled the
 * way ExpressionBasedQuery + AndToQuery compile it (expand :730-737, AndToQuery.java:102-306)
 * and executed with a literal restatement of ZigZagIntersectionResult
 * (C/query/impl/ZigZagIntersectionResult.java) over ArrayBasedSet cursors
 * (C/util/ArrayBasedSet.java:457-543) followed by PredicateBasedFilter(orderedLink).
 * type < 0: no type condition.  has_ordered = 0: no orderedLink condition.
 * Writes result link atom ids (ascending).  Returns the count, or -1 when the
 * reference would throw HGException (no scannable condition), -2 on an
 * out-of-range id. */
int64_t og_and_query(const og_graph *g, int32_t type, const int32_t *incident, int32_t n_incident,
                     const int32_t *pattern, int32_t m, int32_t has_ordered,
                     int32_t *out, int64_t cap);

/* Same as og_and_query but evaluated as plain sorted-set intersection (used by the
 * tests to show the zig-zag restatement and set semantics agree). */
int64_t og_and_query_sets(const og_graph *g, int32_t type, const int32_t *incident, int32_t n_incident,
                          const int32_t *pattern, int32_t m, int32_t has_ordered,
                          int32_t *out, int64_t cap);

/* PositionedIncidentCondition.satisfies on a target array
 * (C/query/PositionedIncidentCondition.java:123-177): x within [lb, ub] (negative bounds count
 * from the end; complement = anywhere outside the range); invalid ranges never match. */
int og_positioned(const int32_t *tgts, int32_t arity, int32_t x, int32_t lb, int32_t ub, int32_t complement);

/* The extended And of hgx_pattern_batch_ext, restated with set semantics:
 *   TypePlusCondition -> Or of AtomTypeConditions (ExpressionBasedQuery.java:606-627), distributed
 *   over the And by toDNF -> one And per type, results united; LinkCondition / OrderedLinkCondition
 *   targets -> IncidentConditions (:730-746); each And = intersection of its ORA sets (type index,
 *   incidence sets, position-filtered incidence sets of PositionedIncidentToQuery) filtered by the
 *   OrderedLinkCondition and ArityCondition predicates (AndToQuery.java:120-294).
 * n_types == 0: no type condition.  pos: 4 ints per positioned condition (target, lb, ub,
 * complement).  Pattern r is pat[pat_off[r] .. pat_off[r+1]), r < n_pat.  arity < 0: none.
 * Returns the ascending result count (may exceed cap), -1 when there is no incidence anchor, -2 on a
 * bad id. */
int64_t og_and_query_ext(const og_graph *g, int32_t n_types, const int32_t *types, int32_t n_inc,
                         const int32_t *inc, int32_t n_pos, const int32_t *pos, int32_t n_pat,
                         const int64_t *pat_off, const int32_t *pat, int32_t arity, int32_t *out, int64_t cap);

/* Batched pattern queries on all cores (CPU baseline).  Queries are packed:
 * q_type[n], q_inc_off[n+1] into q_inc, q_pat_off[n+1] into q_pat, q_has_ordered[n].
 * counts[n] receives result sizes; checksum receives the sum of result ids. */
int og_and_query_many(const og_graph *g, int32_t n, const int32_t *q_type,
                      const int64_t *q_inc_off, const int32_t *q_inc,
                      const int64_t *q_pat_off, const int32_t *q_pat, const int32_t *q_has_ordered,
                      int64_t *counts, int64_t *checksum, int32_t nthreads);

#ifdef __cplusplus
}
#endif
#endif
