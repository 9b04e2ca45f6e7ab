/*
 * hgx_gen.c -- deterministic synthetic hypergraph generators (SURVEY.md section 8(d),
 * configs 1-5).  Host C + OpenMP; results are independent of the thread count
 * because every link draws from its own counter-based stream.
 *
 * Atom ids follow IntHandleFactory add order (C/handle/IntHandleFactory.java:32,49):
 * nodes first (0..N-1), then links (N..N+M-1), so rank order == creation order.
 * The layout of link L is [type, value, t0..tk-1] (C/HyperGraph.java:1603-1608);
 * the generator emits type and targets.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define EXPORT __attribute__((visibility("default")))

static inline uint64_t mix64(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* stream(seed, a, b): the state of draw sequence b of kind a */
static inline uint64_t stream_seed(uint64_t seed, uint64_t a, uint64_t b)
{
    return mix64(mix64(mix64(seed) ^ (a * 0xD1B54A32D192ED03ull)) ^ (b * 0x8CB92BA72F3D8DD7ull));
}

typedef struct { uint64_t s; } rng_t;
static inline uint64_t rng_next(rng_t *r) { r->s += 0x9E3779B97F4A7C15ull; return mix64(r->s); }
/* uniform in [0, n), n < 2^32 (Lemire multiply-shift on the high 32 bits) */
static inline uint32_t rng_below(rng_t *r, uint32_t n)
{
    return (uint32_t)(((rng_next(r) >> 32) * (uint64_t)n) >> 32);
}
static inline double rng_unit(rng_t *r) { return (double)(rng_next(r) >> 11) * (1.0 / 9007199254740992.0); }

/* ------------------------------------------------------------------------ */
/* Alias table over Chung-Lu weights w_i = (i+1)^(-1/(gamma-1))              */
/* ------------------------------------------------------------------------ */
typedef struct { int64_t n; float *prob; int32_t *alias; } alias_t;

static int alias_build(alias_t *t, int64_t n, double gamma)
{
    t->n = n;
    t->prob = (float *)malloc(sizeof(float) * (size_t)n);
    t->alias = (int32_t *)malloc(sizeof(int32_t) * (size_t)n);
    double *w = (double *)malloc(sizeof(double) * (size_t)n);
    int32_t *small = (int32_t *)malloc(sizeof(int32_t) * (size_t)n);
    int32_t *large = (int32_t *)malloc(sizeof(int32_t) * (size_t)n);
    if (!t->prob || !t->alias || !w || !small || !large) { free(w); free(small); free(large); return -1; }
    double ex = -1.0 / (gamma - 1.0), sum = 0;
    for (int64_t i = 0; i < n; i++) { w[i] = pow((double)(i + 1), ex); sum += w[i]; }
    int64_t ns = 0, nl = 0;
    for (int64_t i = 0; i < n; i++) {
        w[i] = w[i] * (double)n / sum;
        if (w[i] < 1.0) small[ns++] = (int32_t)i; else large[nl++] = (int32_t)i;
    }
    while (ns && nl) {          /* Vose */
        int32_t s = small[--ns], l = large[--nl];
        t->prob[s] = (float)w[s];
        t->alias[s] = l;
        w[l] = (w[l] + w[s]) - 1.0;
        if (w[l] < 1.0) small[ns++] = l; else large[nl++] = l;
    }
    while (nl) { int32_t l = large[--nl]; t->prob[l] = 1.0f; t->alias[l] = l; }
    while (ns) { int32_t s = small[--ns]; t->prob[s] = 1.0f; t->alias[s] = s; }
    free(w); free(small); free(large);
    return 0;
}

static inline int32_t alias_sample(const alias_t *t, rng_t *r)
{
    uint64_t u = rng_next(r);
    int32_t i = (int32_t)(((u >> 32) * (uint64_t)t->n) >> 32);
    float f = (float)((u & 0xFFFFFFFFull) * (1.0 / 4294967296.0));
    return f < t->prob[i] ? i : t->alias[i];
}

/* ------------------------------------------------------------------------ */
/* Hypergraph: N nodes, M links, arity U{lo..hi}, distinct targets per link, */
/* drawn uniformly (gamma <= 0) or by Chung-Lu weights (gamma > 1).          */
/* ------------------------------------------------------------------------ */

/* pass 1: per-link arity -> tgt_off[M+1] (prefix) ; returns P */
EXPORT int64_t hgx_gen_hypergraph_offsets(int64_t M, int32_t lo, int32_t hi, uint64_t seed, int64_t *tgt_off)
{
    tgt_off[0] = 0;
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
    for (int64_t l = 0; l < M; l++) {
        rng_t r = { stream_seed(seed, 1, (uint64_t)l) };
        tgt_off[l + 1] = lo + (int64_t)rng_below(&r, (uint32_t)(hi - lo + 1));
    }
    for (int64_t l = 0; l < M; l++) tgt_off[l + 1] += tgt_off[l];
    return tgt_off[M];
}

/* pass 2: targets + link types (n_types <= 1: all type 0) */
EXPORT int hgx_gen_hypergraph_fill(int64_t N, int64_t M, int32_t lo, int32_t hi, double gamma,
                                   int32_t n_types, uint64_t seed, const int64_t *tgt_off,
                                   int32_t *tgt_idx, int32_t *link_type)
{
    (void)lo; (void)hi;
    alias_t at = { 0, NULL, NULL };
    int pl = gamma > 1.0;
    if (pl && alias_build(&at, N, gamma)) return -1;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 4096)
#endif
    for (int64_t l = 0; l < M; l++) {
        rng_t r = { stream_seed(seed, 1, (uint64_t)l) };
        (void)rng_next(&r);                        /* the arity draw of pass 1 */
        int64_t b = tgt_off[l], k = tgt_off[l + 1] - b;
        for (int64_t j = 0; j < k; j++) {
            int32_t t;
            int dup;
            do {
                t = pl ? alias_sample(&at, &r) : (int32_t)rng_below(&r, (uint32_t)N);
                dup = 0;
                for (int64_t q = 0; q < j; q++) if (tgt_idx[b + q] == t) { dup = 1; break; }
            } while (dup);
            tgt_idx[b + j] = t;
        }
        if (link_type) {
            rng_t rt = { stream_seed(seed, 2, (uint64_t)l) };
            link_type[l] = n_types > 1 ? (int32_t)rng_below(&rt, (uint32_t)n_types) : 0;
        }
    }
    free(at.prob); free(at.alias);
    return 0;
}

/* The first k entries of a Fisher-Yates permutation of 0..n-1 (config 1 sources). */
EXPORT int hgx_gen_permutation_prefix(int64_t n, int64_t k, uint64_t seed, int32_t *out)
{
    int32_t *p = (int32_t *)malloc(sizeof(int32_t) * (size_t)n);
    if (!p) return -1;
    for (int64_t i = 0; i < n; i++) p[i] = (int32_t)i;
    rng_t r = { stream_seed(seed, 3, 0) };
    for (int64_t i = 0; i < k && i < n; i++) {
        int64_t j = i + (int64_t)rng_below(&r, (uint32_t)(n - i));
        int32_t t = p[i]; p[i] = p[j]; p[j] = t;
        out[i] = p[i];
    }
    free(p);
    return 0;
}

/* k distinct nodes in [0, n) with deg >= 1 (deg computed from the target rows),
 * uniformly (config 2/4 sources). */
EXPORT int hgx_gen_sources(int64_t n, int64_t P, const int32_t *tgt_idx, int64_t k, uint64_t seed, int32_t *out)
{
    uint8_t *has = (uint8_t *)calloc((size_t)n, 1);
    uint8_t *taken = (uint8_t *)calloc((size_t)n, 1);
    if (!has || !taken) { free(has); free(taken); return -1; }
    for (int64_t p = 0; p < P; p++) if (tgt_idx[p] >= 0 && tgt_idx[p] < n) has[tgt_idx[p]] = 1;
    int64_t avail = 0;
    for (int64_t i = 0; i < n; i++) avail += has[i];
    if (avail < k) { free(has); free(taken); return -2; }
    rng_t r = { stream_seed(seed, 4, 0) };
    for (int64_t i = 0; i < k;) {
        int32_t c = (int32_t)rng_below(&r, (uint32_t)n);
        if (!has[c] || taken[c]) continue;
        taken[c] = 1;
        out[i++] = c;
    }
    free(has); free(taken);
    return 0;
}

/* Config 3 queries: hg.and(hg.type(T), hg.incident(a), hg.orderedLink(x, ANY, y)).
 * L* sampled by uniform pin (degree-biased anchors); T = type(L*); x = t0; y = t2;
 * a = a random target of L* at a position other than 0 and 2; with probability
 * neg_frac, a is replaced by a uniformly random node.  Link atom ids are N + row. */
EXPORT int hgx_gen_queries(int64_t N, int64_t M, const int64_t *tgt_off, const int32_t *tgt_idx,
                           const int32_t *link_type, int64_t Q, double neg_frac, uint64_t seed,
                           int32_t *q_type, int32_t *q_a, int32_t *q_x, int32_t *q_y, int32_t *q_row)
{
    int64_t P = tgt_off[M];
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
    for (int64_t q = 0; q < Q; q++) {
        rng_t r = { stream_seed(seed, 5, (uint64_t)q) };
        uint64_t pin = ((rng_next(&r) >> 11) % (uint64_t)P);
        int64_t lo = 0, hi = M;              /* row with tgt_off[row] <= pin < tgt_off[row+1] */
        while (hi - lo > 1) {
            int64_t mid = (lo + hi) >> 1;
            if ((uint64_t)tgt_off[mid] <= pin) lo = mid; else hi = mid;
        }
        int64_t b = tgt_off[lo], k = tgt_off[lo + 1] - b;
        q_row[q] = (int32_t)lo;
        q_type[q] = link_type ? link_type[lo] : 0;
        q_x[q] = tgt_idx[b];
        q_y[q] = k > 2 ? tgt_idx[b + 2] : tgt_idx[b + k - 1];
        int32_t pos;
        if (k <= 3) pos = 1;
        else { pos = (int32_t)rng_below(&r, (uint32_t)(k - 2)); pos = pos == 0 ? 1 : pos + 2; }
        q_a[q] = tgt_idx[b + (pos < k ? pos : 0)];
        if (rng_unit(&r) < neg_frac) q_a[q] = (int32_t)rng_below(&r, (uint32_t)N);
    }
    return 0;
}

/* Config 5 ontology.  Classes 0..C-1.  Class i>0 gets 1..3 HGSubsumes(parent, i) links
 * (general = target 0, specific = target 1; C/atom/HGSubsumes.java:27-45) with distinct
 * parents drawn preferentially among lower ids (parent = floor(i * u^2)), then n_noise
 * arity-2 links between random classes of another type.  Pass offsets == NULL to get
 * the link count; links are ordered: class 1's subsumes links, class 2's, ..., noise. */
EXPORT int64_t hgx_gen_ontology(int64_t C, int64_t n_noise, uint64_t seed, int32_t subsumes_type,
                                int32_t noise_type, int32_t *tgt_idx, int32_t *link_type)
{
    int64_t *cnt = (int64_t *)malloc(sizeof(int64_t) * (size_t)(C + 1));
    if (!cnt) return -1;
    cnt[0] = 0;
    for (int64_t i = 1; i < C; i++) {
        rng_t r = { stream_seed(seed, 6, (uint64_t)i) };
        int64_t k = 1 + rng_below(&r, 3);
        cnt[i] = k > i ? i : k;
    }
    int64_t total = 0;
    for (int64_t i = 0; i < C; i++) { int64_t c = cnt[i]; cnt[i] = total; total += c; }
    cnt[C] = total;
    if (!tgt_idx) { free(cnt); return total + n_noise; }
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
    for (int64_t i = 1; i < C; i++) {
        rng_t r = { stream_seed(seed, 6, (uint64_t)i) };
        (void)rng_next(&r);
        int64_t b = cnt[i], k = cnt[i + 1] - b;
        int32_t par[3];
        for (int64_t j = 0; j < k; j++) {
            int32_t p; int dup;
            do {
                double u = rng_unit(&r);
                p = (int32_t)((double)i * u * u);
                if (p >= i) p = (int32_t)i - 1;
                dup = 0;
                for (int64_t q = 0; q < j; q++) if (par[q] == p) dup = 1;
            } while (dup);
            par[j] = p;
            tgt_idx[2 * (b + j)] = p;
            tgt_idx[2 * (b + j) + 1] = (int32_t)i;
            link_type[b + j] = subsumes_type;
        }
    }
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
    for (int64_t j = 0; j < n_noise; j++) {
        rng_t r = { stream_seed(seed, 7, (uint64_t)j) };
        int32_t u = (int32_t)rng_below(&r, (uint32_t)C), v;
        do { v = (int32_t)rng_below(&r, (uint32_t)C); } while (v == u && C > 1);
        tgt_idx[2 * (total + j)] = u;
        tgt_idx[2 * (total + j) + 1] = v;
        link_type[total + j] = noise_type;
    }
    free(cnt);
    return total + n_noise;
}
