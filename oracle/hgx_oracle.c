/*
 * hgx_oracle.c -- TEST INFRASTRUCTURE, NOT PRODUCT CODE (see hgx_oracle.h).
 *
 * CPU restatement of the reference's hot path, written from the Java sources
 * cited inline (paths relative to the reference root, C = core/src/java/org/hypergraphdb).
 * Used by tests/ (parity checker), __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg only.
 */
#include "hgx_oracle.h"

#include <limits.h>
#include <setjmp.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------------- */
/* Snapshot / incidence index                                                 */
/* ------------------------------------------------------------------------- */

int og_graph_build(og_graph *g, int64_t A, int64_t M, const int32_t *link_atom,
                   const int64_t *tgt_off, const int32_t *tgt_idx, const int32_t *link_type)
{
    memset(g, 0, sizeof(*g));
    g->A = A; g->M = M; g->link_atom = link_atom; g->tgt_off = tgt_off;
    g->tgt_idx = tgt_idx; g->link_type = link_type;
    g->atom_row = (int32_t *)malloc(sizeof(int32_t) * (size_t)(A > 0 ? A : 1));
    g->inc_off = (int64_t *)calloc((size_t)A + 1, sizeof(int64_t));
    if (!g->atom_row || !g->inc_off) return -1;
    for (int64_t a = 0; a < A; a++) g->atom_row[a] = -1;
    for (int64_t r = 0; r < M; r++) {
        int32_t la = link_atom[r];
        if (la < 0 || la >= A) return -2;
        if (r > 0 && link_atom[r - 1] >= la) return -3;   /* rank order must be strict */
        g->atom_row[la] = (int32_t)r;
    }
    /* Count one entry per distinct (target, link): addIncidenceLink is called once per
     * target position (C/HyperGraph.java:1622 updateTargetsIncidenceSets) but BJE
     * stores it with putNoDupData (BJE/BJEStorageImplementation.java:300-307). */
    for (int64_t r = 0; r < M; r++) {
        for (int64_t p = tgt_off[r]; p < tgt_off[r + 1]; p++) {
            int32_t t = tgt_idx[p];
            if (t < 0 || t >= A) return -2;
            int dup = 0;
            for (int64_t q = tgt_off[r]; q < p; q++) if (tgt_idx[q] == t) { dup = 1; break; }
            if (!dup) g->inc_off[t + 1]++;
        }
    }
    for (int64_t a = 0; a < A; a++) g->inc_off[a + 1] += g->inc_off[a];
    int64_t I = g->inc_off[A];
    g->inc_atom = (int32_t *)malloc(sizeof(int32_t) * (size_t)(I > 0 ? I : 1));
    int64_t *fill = (int64_t *)malloc(sizeof(int64_t) * (size_t)(A > 0 ? A : 1));
    if (!g->inc_atom || !fill) { free(fill); return -1; }
    memcpy(fill, g->inc_off, sizeof(int64_t) * (size_t)A);
    /* Links are visited in ascending rank, so every incidence row comes out
     * ascending = the BJE sorted-duplicate order (BJE/...:109-111). */
    for (int64_t r = 0; r < M; r++) {
        for (int64_t p = tgt_off[r]; p < tgt_off[r + 1]; p++) {
            int32_t t = tgt_idx[p];
            int dup = 0;
            for (int64_t q = tgt_off[r]; q < p; q++) if (tgt_idx[q] == t) { dup = 1; break; }
            if (!dup) g->inc_atom[fill[t]++] = link_atom[r];
        }
    }
    free(fill);
    /* type index: counting sort of link rows by type key (rows ascending inside a type) */
    int32_t tmax = 0;
    for (int64_t r = 0; r < M; r++) {
        int32_t t = link_type ? link_type[r] : 0;
        if (t < 0 || t >= (1 << 24)) return -4;
        if (t > tmax) tmax = t;
    }
    g->n_types = (int64_t)tmax + 1;
    g->type_off = (int64_t *)calloc((size_t)g->n_types + 1, sizeof(int64_t));
    g->type_atoms = (int32_t *)malloc(sizeof(int32_t) * (size_t)(M > 0 ? M : 1));
    int64_t *tf = (int64_t *)malloc(sizeof(int64_t) * (size_t)g->n_types);
    if (!g->type_off || !g->type_atoms || !tf) { free(tf); return -1; }
    for (int64_t r = 0; r < M; r++) g->type_off[(link_type ? link_type[r] : 0) + 1]++;
    for (int64_t t = 0; t < g->n_types; t++) g->type_off[t + 1] += g->type_off[t];
    memcpy(tf, g->type_off, sizeof(int64_t) * (size_t)g->n_types);
    for (int64_t r = 0; r < M; r++) g->type_atoms[tf[link_type ? link_type[r] : 0]++] = link_atom[r];
    free(tf);
    return 0;
}

void og_graph_free(og_graph *g)
{
    free(g->atom_row); free(g->inc_off); free(g->inc_atom); free(g->type_off); free(g->type_atoms);
    memset(g, 0, sizeof(*g));
}

int64_t og_inc_size(const og_graph *g, int32_t atom)
{
    if (atom < 0 || atom >= g->A) return -1;
    return g->inc_off[atom + 1] - g->inc_off[atom];
}

int64_t og_inc_copy(const og_graph *g, int32_t atom, int32_t *out, int64_t cap)
{
    int64_t n = og_inc_size(g, atom);
    if (n < 0) return n;
    for (int64_t i = 0; i < n && i < cap; i++) out[i] = g->inc_atom[g->inc_off[atom] + i];
    return n;
}

static inline int32_t og_type_of_link(const og_graph *g, int32_t row)
{
    return g->link_type ? g->link_type[row] : 0;
}

/* ------------------------------------------------------------------------- */
/* DefaultALGenerator.AdjIterator (C/algorithms/DefaultALGenerator.java:85-364)*/
/* with siblingPredicate == null.                                             */
/* ------------------------------------------------------------------------- */

typedef struct og_adj {
    const og_graph *g;
    og_algen o;
    int32_t src;
    const int32_t *links;  /* the incidence set iterator (:507 getIncidenceSet(h).getSearchResult()) */
    int64_t nlinks, li;
    int32_t cur_link;      /* hCurrLink; -1 == currLink == null */
    const int32_t *t;      /* currLink target array (TempLink at offset 2, :306) */
    int32_t arity;
    int32_t pos, focus_seen;
    int32_t min_arity;     /* :94, :326-327 */
} og_adj;

/* FTargetSetIterator.reset (:168-203) */
static void f_reset(og_adj *it)
{
    const int32_t *t = it->t;
    it->pos = 0;
    it->focus_seen = 0;
    if (!it->o.preceding) {
        while (t[it->pos++] != it->src) { }
        it->focus_seen = 1;
        if (it->o.source) { it->pos--; return; }          /* siblingPredicate == null */
        else if (it->pos == it->arity) { it->pos = -1; return; }
    }
    if (!it->focus_seen && t[it->pos] == it->src) {
        it->focus_seen = 1;
        if (it->o.source) return;
        else if (!it->o.succeeding) { it->pos = -1; return; }
        else it->pos++;
    }
}

/* FTargetSetIterator.advance (:149-166) */
static void f_advance(og_adj *it)
{
    if (++it->pos == it->arity) { it->pos = -1; return; }
    else if (!it->focus_seen && it->t[it->pos] == it->src) {
        it->focus_seen = 1;
        if (it->o.source) return;
        else if (!it->o.succeeding || ++it->pos == it->arity) it->pos = -1;
    }
}

/* BTargetSetIterator.reset (:235-266) */
static void b_reset(og_adj *it)
{
    const int32_t *t = it->t;
    it->pos = it->arity - 1;
    it->focus_seen = 0;
    if (!it->o.preceding) {
        while (t[it->pos--] != it->src) { }
        it->focus_seen = 1;
        if (it->o.source) { it->pos++; return; }
        else if (it->pos == -1) return;
    }
    if (!it->focus_seen && t[it->pos] == it->src) {
        it->focus_seen = 1;
        if (it->o.source) return;
        else if (!it->o.succeeding) { it->pos = -1; return; }
        else it->pos--;
    }
}

/* BTargetSetIterator.advance (:268-284) */
static void b_advance(og_adj *it)
{
    if (--it->pos == -1) return;
    else if (!it->focus_seen && it->t[it->pos] == it->src) {
        it->focus_seen = 1;
        if (it->o.source) return;
        if (!it->o.succeeding) it->pos = -1;
        else it->pos--;
    }
}

static inline void ts_reset(og_adj *it) { if (it->o.reverse) b_reset(it); else f_reset(it); }
static inline void ts_advance(og_adj *it) { if (it->o.reverse) b_advance(it); else f_advance(it); }

/* AdjIterator.getNextLink (:287-315) */
static void adj_next_link(og_adj *it)
{
    const og_graph *g = it->g;
    for (;;) {
        if (it->li >= it->nlinks) { it->cur_link = -1; return; }
        int32_t h = it->links[it->li++];
        int32_t row = g->atom_row[h];
        /* linkPredicate = AtomTypeCondition: hg.getType(link) == type (C/query/AtomTypeCondition.java:121-135) */
        if (it->o.link_type >= 0 && og_type_of_link(g, row) != it->o.link_type) continue;
        it->cur_link = h;
        it->t = g->tgt_idx + g->tgt_off[row];
        it->arity = (int32_t)(g->tgt_off[row + 1] - g->tgt_off[row]);
        if (it->arity < it->min_arity) continue;
        ts_reset(it);
        if (it->pos != -1) break;       /* tsIter.hasNext() */
    }
}

static void adj_init(og_adj *it, const og_graph *g, const og_algen *o, int32_t src)
{
    it->g = g; it->o = *o; it->src = src;
    it->links = g->inc_atom + g->inc_off[src];
    it->nlinks = g->inc_off[src + 1] - g->inc_off[src];
    it->li = 0;
    it->min_arity = o->source ? 1 : 2;
    adj_next_link(it);
}

static inline int adj_has_next(const og_adj *it) { return it->cur_link != -1; }

/* AdjIterator.next (:338-344) */
static inline void adj_next(og_adj *it, int32_t *link, int32_t *atom)
{
    *link = it->cur_link;
    *atom = it->t[it->pos];          /* TargetSetIterator.next (:113-118) */
    ts_advance(it);
    if (it->pos == -1) adj_next_link(it);
}

int64_t og_generate(const og_graph *g, const og_algen *o, int32_t src,
                    int32_t *out_link, int32_t *out_atom, int64_t cap)
{
    if (src < 0 || src >= g->A) return -2;
    og_adj it;
    adj_init(&it, g, o, src);
    int64_t n = 0;
    while (adj_has_next(&it)) {
        int32_t l, a;
        adj_next(&it, &l, &a);
        if (n < cap) { out_link[n] = l; out_atom[n] = a; }
        n++;
    }
    return n;
}

/* ------------------------------------------------------------------------- */
/* HGBreadthFirstTraversal (C/algorithms/HGBreadthFirstTraversal.java:29-164) */
/* ------------------------------------------------------------------------- */

typedef struct og_bfs_state {
    int64_t A;
    uint32_t *stamp;    /* examined.containsKey(h) <=> stamp[h] == epoch   */
    uint8_t *flag;      /* examined.get(h): 1 = TRUE, 0 = FALSE            */
    int32_t *q_link, *q_atom, *q_dist;   /* to_explore (FIFO)           */
    uint32_t epoch;
} og_bfs_state;

static int bfs_state_init(og_bfs_state *s, int64_t A)
{
    s->A = A; s->epoch = 0;
    size_t n = (size_t)(A > 0 ? A : 1);
    s->stamp = (uint32_t *)calloc(n, sizeof(uint32_t));
    s->flag = (uint8_t *)calloc(n, 1);
    s->q_link = (int32_t *)malloc(n * sizeof(int32_t));
    s->q_atom = (int32_t *)malloc(n * sizeof(int32_t));
    s->q_dist = (int32_t *)malloc(n * sizeof(int32_t));
    return (s->stamp && s->flag && s->q_link && s->q_atom && s->q_dist) ? 0 : -1;
}

static void bfs_state_free(og_bfs_state *s)
{
    free(s->stamp); free(s->flag); free(s->q_link); free(s->q_atom); free(s->q_dist);
}

typedef void (*og_bfs_emit)(void *ctx, int32_t link, int32_t atom, int32_t dist);

/* Returns the number of pairs returned by next(); *traversed = sum of |inc(v)| over
 * the atoms passed to advance() that were below maxDistance (the atoms whose
 * incidence set was iterated, :49-66). */
static double og_now(void)
{
#ifdef _OPENMP
    return omp_get_wtime();
#else
    return 0.0;
#endif
}

static int64_t bfs_run(const og_graph *g, const og_algen *o, og_bfs_state *s, int32_t seed,
                       int32_t max_dist, og_bfs_emit emit, void *ctx, int64_t *traversed,
                       double deadline)
{
    int32_t maxd = max_dist < 0 ? INT_MAX : max_dist;
    uint32_t ep = ++s->epoch;
    if (ep == 0) { memset(s->stamp, 0, sizeof(uint32_t) * (size_t)s->A); ep = s->epoch = 1; }
    int64_t head = 0, tail = 0, returned = 0, trav = 0;

    /* init(): examined.put(start, TRUE); advance(start, 0)   (:42-46) */
    s->stamp[seed] = ep; s->flag[seed] = 1;
    int32_t from = seed, dist = 0;
    for (;;) {
        /* advance(from, distance) (:49-66) */
        if (dist < maxd) {
            og_adj it;
            adj_init(&it, g, o, from);
            trav += g->inc_off[from + 1] - g->inc_off[from];
            int32_t dd = dist + 1;
            while (adj_has_next(&it)) {
                int32_t l, a;
                adj_next(&it, &l, &a);
                if (s->stamp[a] != ep) {                 /* !examined.containsKey */
                    s->q_link[tail] = l; s->q_atom[tail] = a; s->q_dist[tail] = dd; tail++;
                    s->stamp[a] = ep; s->flag[a] = 0;     /* examined.put(.., FALSE) */
                }
            }
        }
        /* next(): x = to_explore.remove(); examined.put(atom, TRUE); advance (:143-156) */
        if (head == tail) break;
        if (deadline > 0 && (head & 1023) == 0 && og_now() > deadline) break;   /* bounded sample */
        int32_t l = s->q_link[head], a = s->q_atom[head], d = s->q_dist[head];
        head++;
        s->flag[a] = 1;
        if (emit) emit(ctx, l, a, d);
        returned++;
        from = a; dist = d;
    }
    if (traversed) *traversed = trav;
    return returned;
}

typedef struct { int32_t *l, *a, *d; int64_t cap, n; } seq_ctx;
static void seq_emit(void *c, int32_t link, int32_t atom, int32_t dist)
{
    seq_ctx *x = (seq_ctx *)c;
    if (x->n < x->cap) {
        if (x->l) x->l[x->n] = link;
        if (x->a) x->a[x->n] = atom;
        if (x->d) x->d[x->n] = dist;
    }
    x->n++;
}

int64_t og_bfs(const og_graph *g, const og_algen *o, int32_t seed, int32_t max_dist,
               int32_t *out_link, int32_t *out_atom, int32_t *out_dist, int64_t cap,
               int64_t *traversed)
{
    if (seed < 0 || seed >= g->A) return -2;
    og_bfs_state s;
    if (bfs_state_init(&s, g->A)) { bfs_state_free(&s); return -1; }
    seq_ctx c = { out_link, out_atom, out_dist, cap, 0 };
    bfs_run(g, o, &s, seed, max_dist, seq_emit, &c, traversed, 0.0);
    bfs_state_free(&s);
    return c.n;
}

typedef struct { int64_t *counts; int32_t levels; } cnt_ctx;
static void cnt_emit(void *c, int32_t link, int32_t atom, int32_t dist)
{
    (void)link; (void)atom;
    cnt_ctx *x = (cnt_ctx *)c;
    if (dist < x->levels) x->counts[dist]++;
}

int og_bfs_many(const og_graph *g, const og_algen *o, const int32_t *seeds, int32_t n_seeds,
                int32_t max_dist, int32_t max_levels, int64_t *counts, int64_t *traversed,
                int32_t nthreads, double time_budget_s, double *elapsed_s)
{
    double t0 = og_now();
    double deadline = time_budget_s > 0 ? t0 + time_budget_s : 0.0;
    for (int32_t i = 0; i < n_seeds; i++) if (seeds[i] < 0 || seeds[i] >= g->A) return -2;
    memset(counts, 0, sizeof(int64_t) * (size_t)n_seeds * (size_t)max_levels);
    int err = 0;
#ifdef _OPENMP
    int nt = nthreads > 0 ? nthreads : omp_get_max_threads();
#pragma omp parallel num_threads(nt) reduction(|:err)
#endif
    {
        og_bfs_state s;
        if (bfs_state_init(&s, g->A)) err = 1;
        else {
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
            for (int32_t i = 0; i < n_seeds; i++) {
                cnt_ctx c = { counts + (size_t)i * (size_t)max_levels, max_levels };
                if (max_levels > 0) c.counts[0] = 1;
                int64_t tr = 0;
                bfs_run(g, o, &s, seeds[i], max_dist, cnt_emit, &c, &tr, deadline);
                if (traversed) traversed[i] = tr;
            }
        }
        bfs_state_free(&s);
    }
    (void)nthreads;
    if (elapsed_s) *elapsed_s = og_now() - t0;
    return err ? -1 : 0;
}

/* ------------------------------------------------------------------------- */
/* OrderedLinkCondition.satisfies (C/query/OrderedLinkCondition.java:92-124)  */
/* ------------------------------------------------------------------------- */

int og_ordered_link(const int32_t *tgts, int32_t arity, const int32_t *pattern, int32_t m)
{
    int32_t i = 0, j = 0;
    while (i < arity && j < m) {
        if (pattern[j] == tgts[i] || pattern[j] < 0) j++;   /* equals(target) || equals(anyHandle) */
        i++;
    }
    return j == m;
}

/* ------------------------------------------------------------------------- */
/* Random-access result sets: ArrayBasedSet.ResultSet (C/util/ArrayBasedSet.java:457-543) */
/* and ZigZagIntersectionResult (C/query/impl/ZigZagIntersectionResult.java)  */
/* ------------------------------------------------------------------------- */

typedef enum { GT_FOUND, GT_CLOSE, GT_NOTHING } gt_res;
#define RS_UNKNOWN INT64_MIN
#define RS_NULL    (-1)

typedef struct rar rar;
struct rar {
    int kind;                       /* 0 = sorted array cursor, 1 = zig-zag */
    const int32_t *a; int64_t n; int64_t pos;
    rar *left, *right;
    int64_t cur, nxt, prv;
};

static __thread jmp_buf *og_throw;  /* NoSuchElementException -> query throws */
static void og_no_such_element(void) { longjmp(*og_throw, 1); }

static int rar_has_next(rar *r);
static int32_t rar_next(rar *r);
static int32_t rar_current(rar *r);
static gt_res rar_goto(rar *r, int32_t v, int exact);

/* ArrayBasedSet.lookup (:60-78) */
static int64_t abs_lookup(const rar *r, int32_t key)
{
    int64_t low = 0, high = r->n - 1;
    while (low <= high) {
        int64_t mid = (low + high) >> 1;
        int32_t mv = r->a[mid];
        if (mv < key) low = mid + 1;
        else if (mv > key) high = mid - 1;
        else return mid;
    }
    return -(low + 1);
}

static gt_res abs_goto(rar *r, int32_t v, int exact)
{
    int64_t idx = abs_lookup(r, v);
    if (idx >= 0) { r->pos = idx; return GT_FOUND; }
    else if (exact) return GT_NOTHING;
    idx = -(idx + 1);
    if (idx >= r->n) return GT_NOTHING;
    r->pos = idx;
    return GT_CLOSE;
}

static void zz_swap(rar *z) { rar *t = z->left; z->left = z->right; z->right = t; }

/* ZigZagIntersectionResult.advance (:37-75) */
static int64_t zz_advance(rar *z)
{
    int use_next = 1;
    for (;;) {
        if ((!rar_has_next(z->left) && use_next) || !rar_has_next(z->right)) return RS_NULL;
        int32_t x;
        if (use_next) x = rar_next(z->left);
        else { x = rar_current(z->left); use_next = 1; }
        switch (rar_goto(z->right, x, 0)) {
        case GT_FOUND: return x;
        case GT_CLOSE: use_next = 0; zz_swap(z); break;
        default: return RS_NULL;
        }
    }
}

/* ZigZagIntersectionResult.positionTo (:100-125) */
static int zz_position_to(rar *z, rar *left_or_right)
{
    if (z->left != left_or_right) zz_swap(z);
    for (;;) {
        switch (rar_goto(z->right, rar_current(z->left), 0)) {
        case GT_FOUND:
            z->cur = rar_current(z->left);
            z->nxt = z->prv = RS_UNKNOWN;
            return 1;
        case GT_CLOSE: zz_swap(z); break;
        default: return 0;
        }
    }
}

/* current() of a child, mapping NoSuchElementException to 'has no current' */
static int rar_try_current(rar *r, int32_t *out)
{
    if (r->kind == 0) {
        if (r->pos < 0 || r->pos >= r->n) return 0;
        *out = r->a[r->pos];
        return 1;
    }
    if (r->cur == RS_UNKNOWN) return 0;
    *out = (int32_t)r->cur;
    return 1;
}

/* ZigZagIntersectionResult.goTo (:155-247) */
static gt_res zz_goto(rar *z, int32_t value, int exact)
{
    rar *starting_left = z->left, *starting_right = z->right;
    int32_t save_left, save_right;
    if (!rar_try_current(z->left, &save_left) || !rar_try_current(z->right, &save_right))
        return GT_NOTHING;
    gt_res r_l = rar_goto(z->left, value, exact);
    if (r_l == GT_NOTHING) return GT_NOTHING;
    gt_res r_r = rar_goto(z->right, value, exact);
    if (r_r == GT_NOTHING) {
        rar_goto(starting_left, save_left, 1);
        return GT_NOTHING;
    }
    if (r_l == GT_FOUND) {
        if (r_r == GT_FOUND) {
            z->cur = rar_current(z->left);
            z->nxt = z->prv = RS_UNKNOWN;
            return GT_FOUND;
        }
        if (zz_position_to(z, z->right)) return GT_CLOSE;
        rar_goto(starting_left, save_left, 1);
        rar_goto(starting_right, save_right, 1);
        return GT_NOTHING;
    }
    if (r_r == GT_FOUND) {
        if (zz_position_to(z, z->left)) return GT_CLOSE;
        rar_goto(starting_left, save_left, 1);
        rar_goto(starting_right, save_right, 1);
        return GT_NOTHING;
    }
    {
        int32_t lc = rar_current(z->left), rc = rar_current(z->right);
        int cmp = (lc > rc) - (lc < rc);
        if ((cmp == 0 && zz_position_to(z, z->left)) || (cmp > 0 && zz_position_to(z, z->left)) ||
            zz_position_to(z, z->right))
            return GT_CLOSE;
        rar_goto(starting_left, save_left, 1);
        rar_goto(starting_right, save_right, 1);
        return GT_NOTHING;
    }
}

static int rar_has_next(rar *r)
{
    if (r->kind == 0) return r->pos + 1 < r->n;
    if (r->nxt == RS_UNKNOWN) r->nxt = zz_advance(r);         /* :283-288 */
    return r->nxt != RS_NULL;
}

static int32_t rar_next(rar *r)
{
    if (r->kind == 0) return r->a[++r->pos];
    if (!rar_has_next(r)) og_no_such_element();
    r->prv = r->cur; r->cur = r->nxt; r->nxt = RS_UNKNOWN;    /* :290-302 */
    return (int32_t)r->cur;
}

static int32_t rar_current(rar *r)
{
    int32_t v;
    if (!rar_try_current(r, &v)) og_no_such_element();
    return v;
}

static gt_res rar_goto(rar *r, int32_t v, int exact)
{
    return r->kind == 0 ? abs_goto(r, v, exact) : zz_goto(r, v, exact);
}

/* ------------------------------------------------------------------------- */
/* hg.and(type, incident..., orderedLink) compile + execute                   */
/* ------------------------------------------------------------------------- */

typedef struct { const int32_t *a; int64_t n; int64_t size; } ora_item;

static int cmp_ora(const void *x, const void *y)
{
    /* AndToQuery.BySizeComparator on sizeExpected; qsort is not stable so ties
     * are broken by the original position (Collections.sort is stable). */
    const ora_item *a = (const ora_item *)x, *b = (const ora_item *)y;
    if (a->size != b->size) return a->size < b->size ? -1 : 1;
    return (a->a > b->a) - (a->a < b->a);
}

/* Common front end: returns anchors (deduped incident targets in condition order,
 * ExpressionBasedQuery.expand :730-737 and toDNF's HashSet :100) or -2 on a bad id. */
static int32_t build_anchors(const og_graph *g, const int32_t *incident, int32_t n_incident,
                             const int32_t *pattern, int32_t m, int32_t *anchors)
{
    int32_t na = 0;
    for (int32_t i = 0; i < n_incident + m; i++) {
        int32_t h = i < n_incident ? incident[i] : pattern[i - n_incident];
        if (i >= n_incident && h < 0) continue;                       /* anyHandle */
        if (h < 0 || h >= g->A) return -2;
        int dup = 0;
        for (int32_t k = 0; k < na; k++) if (anchors[k] == h) { dup = 1; break; }
        if (!dup) anchors[na++] = h;
    }
    return na;
}

typedef struct { rar *nodes; int32_t nn; int64_t nout; } zz_run;

/* Left-deep nest of ZigZag intersections over the size-sorted ORA cursors
 * (AndToQuery.java:164-180), each built by IntersectionQuery.execute
 * (impl/IntersectionQuery.java:45-59: an empty side gives HGSearchResult.EMPTY),
 * drained through PredicateBasedFilter(orderedLink) (impl/PredicateBasedFilter.java:67-86).
 * Returns -3 when the restated Java would throw NoSuchElementException. */
static int64_t zz_execute(const og_graph *g, const ora_item *ora, int32_t nora,
                          const int32_t *pattern, int32_t m, int32_t has_ordered,
                          int32_t *out, int64_t cap)
{
    zz_run st;
    st.nodes = (rar *)calloc((size_t)(2 * nora + 1), sizeof(rar));
    st.nn = 0;
    st.nout = 0;
    zz_run *run = &st;
    for (int32_t i = 0; i < nora; i++) {
        rar *c = &run->nodes[run->nn++];
        c->kind = 0; c->a = ora[i].a; c->n = ora[i].n; c->pos = -1;
    }
    jmp_buf jb;
    jmp_buf *saved = og_throw;
    og_throw = &jb;
    if (setjmp(jb) != 0) {
        og_throw = saved;
        free(run->nodes);
        return -3;
    }
    rar *result = &run->nodes[0];
    int empty = 0;
    for (int32_t i = 1; i < nora; i++) {       /* nora == 1: the single ORA moves to O (:181-217) */
        rar *right = &run->nodes[i];
        if (!rar_has_next(result) || !rar_has_next(right)) { empty = 1; break; }
        rar *z = &run->nodes[run->nn++];
        z->kind = 1; z->left = result; z->right = right;
        z->cur = z->nxt = z->prv = RS_UNKNOWN;
        result = z;
    }
    if (!empty) {
        while (rar_has_next(result)) {
            int32_t h = rar_next(result);
            int ok = 1;
            if (has_ordered) {
                int32_t row = g->atom_row[h];
                ok = og_ordered_link(g->tgt_idx + g->tgt_off[row],
                                     (int32_t)(g->tgt_off[row + 1] - g->tgt_off[row]), pattern, m);
            }
            if (ok) { if (run->nout < cap) out[run->nout] = h; run->nout++; }
        }
    }
    og_throw = saved;
    free(run->nodes);
    return run->nout;
}

static int64_t and_query_impl(const og_graph *g, int32_t type, const int32_t *incident, int32_t n_incident,
                              const int32_t *pattern, int32_t m, int32_t has_ordered,
                              int32_t *out, int64_t cap, int use_zigzag)
{
    int32_t *anchors = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n_incident + m + 1));
    int32_t na = build_anchors(g, incident, n_incident, pattern, has_ordered ? m : 0, anchors);
    if (na < 0) { free(anchors); return na; }
    if (na == 0) { free(anchors); return -1; }   /* not accelerated: no incidence anchor */
    if (has_ordered && m == 0) { free(anchors); return 0; }   /* QueryMetaData.EMPTY in ORA -> HGQuery.NOP */

    /* The type index restricted to links (the incidence anchors drop every node). */
    const int32_t *typed = NULL;
    int64_t ntyped = 0;
    if (type >= 0 && type < g->n_types) {
        typed = g->type_atoms + g->type_off[type];
        ntyped = g->type_off[type + 1] - g->type_off[type];
    }
    int32_t nora = na + (type >= 0 ? 1 : 0);
    ora_item *ora = (ora_item *)malloc(sizeof(ora_item) * (size_t)nora);
    int32_t k = 0;
    if (type >= 0) { ora[k].a = typed ? typed : anchors; ora[k].n = ntyped; ora[k].size = ntyped; k++; }
    for (int32_t i = 0; i < na; i++, k++) {
        ora[k].a = g->inc_atom + g->inc_off[anchors[i]];
        ora[k].n = g->inc_off[anchors[i] + 1] - g->inc_off[anchors[i]];
        ora[k].size = ora[k].n;
    }
    qsort(ora, (size_t)nora, sizeof(ora_item), cmp_ora);

    int64_t nout = 0;
    if (use_zigzag) {
        nout = zz_execute(g, ora, nora, pattern, m, has_ordered, out, cap);
    } else {
        /* plain set semantics: iterate the smallest list, test membership in the rest */
        const ora_item *base = &ora[0];
        for (int64_t i = 0; i < base->n; i++) {
            int32_t h = base->a[i];
            int ok = 1;
            for (int32_t j = 1; j < nora && ok; j++) {
                rar c = { 0 }; c.a = ora[j].a; c.n = ora[j].n; c.pos = -1;
                ok = abs_lookup(&c, h) >= 0;
            }
            if (ok && has_ordered) {
                int32_t row = g->atom_row[h];
                ok = og_ordered_link(g->tgt_idx + g->tgt_off[row],
                                     (int32_t)(g->tgt_off[row + 1] - g->tgt_off[row]), pattern, m);
            }
            if (ok) { if (nout < cap) out[nout] = h; nout++; }
        }
    }
    free(ora); free(anchors);
    return nout;
}

int64_t og_and_query(const og_graph *g, int32_t type, const int32_t *incident, int32_t n_incident,
                     const int32_t *pattern, int32_t m, int32_t has_ordered,
                     int32_t *out, int64_t cap)
{
    return and_query_impl(g, type, incident, n_incident, pattern, m, has_ordered, out, cap, 1);
}

int64_t og_and_query_sets(const og_graph *g, int32_t type, const int32_t *incident, int32_t n_incident,
                          const int32_t *pattern, int32_t m, int32_t has_ordered,
                          int32_t *out, int64_t cap)
{
    return and_query_impl(g, type, incident, n_incident, pattern, m, has_ordered, out, cap, 0);
}

/* ------------------------------------------------------------------------- */
/* Extended And: TypePlus / Link / PositionedIncident / Arity / several orderedLinks */
/* ------------------------------------------------------------------------- */

int og_positioned(const int32_t *t, int32_t n, int32_t x, int32_t lb, int32_t ub, int32_t complement)
{
    /* C/query/PositionedIncidentCondition.java:146-176 */
    if (ub < 0) ub = n + ub;
    if (lb < 0) lb = n + lb;
    if (lb > ub || lb < 0 || ub < 0 || lb >= n || ub >= n) return 0;
    if (complement) {
        for (int32_t i = 0; i < lb; i++) if (t[i] == x) return 1;
        for (int32_t i = ub + 1; i < n; i++) if (t[i] == x) return 1;
        return 0;
    }
    for (int32_t i = lb; i <= ub; i++) if (t[i] == x) return 1;
    return 0;
}

typedef struct { const int32_t *a; int64_t n; int32_t *own; } ext_list;

static int cmp_ext_list(const void *x, const void *y)
{
    const ext_list *a = (const ext_list *)x, *b = (const ext_list *)y;
    return (a->n > b->n) - (a->n < b->n);
}

static int cmp_i32(const void *x, const void *y)
{
    int32_t a = *(const int32_t *)x, b = *(const int32_t *)y;
    return (a > b) - (a < b);
}

static int64_t bsearch_i32(const int32_t *a, int64_t n, int32_t key)
{
    int64_t lo = 0, hi = n - 1;
    while (lo <= hi) {
        int64_t mid = (lo + hi) >> 1;
        if (a[mid] < key) lo = mid + 1;
        else if (a[mid] > key) hi = mid - 1;
        else return mid;
    }
    return -1;
}

/* One And of the DNF (one type or none): the ascending intersection of its ORA sets
 * (AndToQuery.java:164-217) filtered by its predicates (:277-293).  Appends to buf. */
static int64_t ext_one_and(const og_graph *g, int32_t type, const int32_t *anchors, int32_t na,
                           const int32_t *pos, int32_t n_pos, int32_t n_pat, const int64_t *pat_off,
                           const int32_t *pat, int32_t arity, int32_t **buf, int64_t *bcap, int64_t nb)
{
    int32_t nl = na + n_pos + (type >= 0 ? 1 : 0);
    ext_list *L = (ext_list *)calloc((size_t)(nl > 0 ? nl : 1), sizeof(ext_list));
    int32_t k = 0;
    if (type >= 0) {   /* the type index (links only) */
        if (type < g->n_types) { L[k].a = g->type_atoms + g->type_off[type]; L[k].n = g->type_off[type + 1] - g->type_off[type]; }
        k++;
    }
    for (int32_t i = 0; i < na; i++, k++) {
        L[k].a = g->inc_atom + g->inc_off[anchors[i]];
        L[k].n = g->inc_off[anchors[i] + 1] - g->inc_off[anchors[i]];
    }
    for (int32_t s = 0; s < n_pos; s++, k++) {   /* PositionedIncidentToQuery: inc(target) filtered */
        int32_t x = pos[4 * s];
        const int32_t *inc = g->inc_atom + g->inc_off[x];
        int64_t m = g->inc_off[x + 1] - g->inc_off[x], c = 0;
        int32_t *f = (int32_t *)malloc(sizeof(int32_t) * (size_t)(m > 0 ? m : 1));
        for (int64_t i = 0; i < m; i++) {
            int32_t row = g->atom_row[inc[i]];
            if (og_positioned(g->tgt_idx + g->tgt_off[row], (int32_t)(g->tgt_off[row + 1] - g->tgt_off[row]), x,
                              pos[4 * s + 1], pos[4 * s + 2], pos[4 * s + 3]))
                f[c++] = inc[i];
        }
        L[k].a = f; L[k].n = c; L[k].own = f;
    }
    qsort(L, (size_t)nl, sizeof(ext_list), cmp_ext_list);
    for (int64_t i = 0; i < (nl > 0 ? L[0].n : 0); i++) {
        int32_t h = L[0].a[i];
        int ok = 1;
        for (int32_t j = 1; j < nl && ok; j++) ok = bsearch_i32(L[j].a, L[j].n, h) >= 0;
        if (!ok) continue;
        int32_t row = g->atom_row[h];
        const int32_t *t = g->tgt_idx + g->tgt_off[row];
        int32_t ar = (int32_t)(g->tgt_off[row + 1] - g->tgt_off[row]);
        if (arity >= 0 && ar != arity) continue;   /* ArityCondition: layout.length == arity + 2 */
        for (int32_t r = 0; r < n_pat && ok; r++)
            ok = og_ordered_link(t, ar, pat + pat_off[r], (int32_t)(pat_off[r + 1] - pat_off[r]));
        if (!ok) continue;
        if (nb >= *bcap) {
            *bcap = *bcap * 2 + 64;
            *buf = (int32_t *)realloc(*buf, sizeof(int32_t) * (size_t)*bcap);
        }
        (*buf)[nb++] = h;
    }
    for (int32_t j = 0; j < nl; j++) free(L[j].own);
    free(L);
    return nb;
}

int64_t og_and_query_ext(const og_graph *g, int32_t n_types, const int32_t *types, int32_t n_inc,
                         const int32_t *inc, int32_t n_pos, const int32_t *pos, int32_t n_pat,
                         const int64_t *pat_off, const int32_t *pat, int32_t arity, int32_t *out, int64_t cap)
{
    /* expand: incident targets, then every non-ANY pattern target (deduplicated) */
    int64_t maxa = n_inc + (n_pat > 0 ? pat_off[n_pat] - pat_off[0] : 0) + 1;
    int32_t *anchors = (int32_t *)malloc(sizeof(int32_t) * (size_t)maxa);
    int32_t na = 0;
    for (int64_t i = 0; i < maxa - 1; i++) {
        int32_t h = i < n_inc ? inc[i] : pat[pat_off[0] + (i - n_inc)];
        if (i >= n_inc && h < 0) continue;   /* anyHandle */
        if (h < 0 || h >= g->A) { free(anchors); return -2; }
        int dup = 0;
        for (int32_t k = 0; k < na; k++) if (anchors[k] == h) { dup = 1; break; }
        if (!dup) anchors[na++] = h;
    }
    for (int32_t s = 0; s < n_pos; s++)
        if (pos[4 * s] < 0 || pos[4 * s] >= g->A) { free(anchors); return -2; }
    if (na == 0 && n_pos == 0) { free(anchors); return -1; }
    for (int32_t r = 0; r < n_pat; r++)
        if (pat_off[r + 1] == pat_off[r]) { free(anchors); return 0; }   /* QueryMetaData.EMPTY -> NOP */
    int32_t *buf = NULL;
    int64_t bcap = 0, nb = 0;
    if (n_types == 0) {
        nb = ext_one_and(g, -1, anchors, na, pos, n_pos, n_pat, pat_off, pat, arity, &buf, &bcap, nb);
    } else {
        for (int32_t t = 0; t < n_types; t++) {   /* toDNF: one And per type of the Or, united */
            int dup = 0;
            for (int32_t u = 0; u < t; u++) if (types[u] == types[t]) dup = 1;
            if (!dup) nb = ext_one_and(g, types[t], anchors, na, pos, n_pos, n_pat, pat_off, pat, arity, &buf, &bcap, nb);
        }
        if (nb > 1) qsort(buf, (size_t)nb, sizeof(int32_t), cmp_i32);
    }
    for (int64_t i = 0; i < nb && i < cap; i++) out[i] = buf[i];
    free(buf);
    free(anchors);
    return nb;
}

int og_and_query_many(const og_graph *g, int32_t n, const int32_t *q_type,
                      const int64_t *q_inc_off, const int32_t *q_inc,
                      const int64_t *q_pat_off, const int32_t *q_pat, const int32_t *q_has_ordered,
                      int64_t *counts, int64_t *checksum, int32_t nthreads)
{
    int64_t sum = 0;
    int err = 0;
#ifdef _OPENMP
    int nt = nthreads > 0 ? nthreads : omp_get_max_threads();
#pragma omp parallel num_threads(nt) reduction(+:sum) reduction(|:err)
#endif
    {
        int64_t cap = 1 << 16;
        int32_t *buf = (int32_t *)malloc(sizeof(int32_t) * (size_t)cap);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 4)
#endif
        for (int32_t q = 0; q < n; q++) {
            int64_t c;
            for (;;) {
                c = og_and_query(g, q_type[q], q_inc + q_inc_off[q], (int32_t)(q_inc_off[q + 1] - q_inc_off[q]),
                                 q_pat + q_pat_off[q], (int32_t)(q_pat_off[q + 1] - q_pat_off[q]),
                                 q_has_ordered[q], buf, cap);
                if (c <= cap) break;
                cap = c;
                free(buf);
                buf = (int32_t *)malloc(sizeof(int32_t) * (size_t)cap);
            }
            counts[q] = c;
            if (c < 0) err = 1;
            for (int64_t i = 0; i < c; i++) sum += buf[i];
        }
        free(buf);
    }
    (void)nthreads;
    *checksum = sum;
    return err ? -1 : 0;
}
