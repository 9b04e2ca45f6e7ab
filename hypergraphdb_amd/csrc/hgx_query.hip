// hgx_query.hip -- batched conjunctive pattern matching over typed hyperedges.
//
// Replaces, for And{type set?, IncidentCondition*, PositionedIncidentCondition*,
// OrderedLinkCondition*, ArityCondition?}:
//   ExpressionBasedQuery.expand (C/query/cond2qry/ExpressionBasedQuery.java:603-755: orderedLink and
//   LinkCondition add incident(x) for each non-ANY target, :730-746; TypePlusCondition becomes an
//   Or of its subtypes' AtomTypeConditions, :606-627) -> AndToQuery
//   (C/query/cond2qry/AndToQuery.java:102-306): nested ZigZagIntersectionResult
//   (C/query/impl/ZigZagIntersectionResult.java) over the sorted incidence sets, the type index and
//   the position-filtered incidence sets of PositionedIncidentToQuery, then PredicateBasedFilter for
//   OrderedLinkCondition (C/query/OrderedLinkCondition.java:92-124) and ArityCondition
//   (C/query/ArityCondition.java:49-67).
//
// GPU formulation: L is in inc(a) <=> a is a target of L.  So the intersection of the anchor
// incidence sets is the smallest anchor set filtered by "every other anchor is in targets(L)",
// which reads one short target row per candidate instead of zig-zag probes.  Candidates are
// visited in ascending order, so the result is ascending like the reference's.  A candidate
// failing the type filter (one 4-byte read) never touches its target row.
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>

#include "hgx_internal.h"

namespace hgx {

typedef unsigned long long u64;

constexpr int kMaxAnchors = 32;
constexpr int kMaxPattern = 64;     // targets of one OrderedLinkCondition
constexpr int kMaxPatterns = 16;    // OrderedLinkConditions in one And
constexpr int kMaxPositioned = 16;  // PositionedIncidentConditions in one And
constexpr int kMaxTypes = 1 << 16;  // types of one Or (TypePlusCondition)
constexpr int kQShards = 16, kQStride = 16;   // counter replicas of the match kernel

struct QPlan {
    int64_t beg;    // first incidence entry of the smallest anchor set
    int64_t n;      // its size (0: empty result)
    int32_t amin;   // index of that anchor inside the query's anchor list
    int32_t pad;
};

// Per-query descriptor on the device (offsets into the flat arrays of the batch).
struct QDesc {
    int64_t a_beg, a_end;   // anchors
    int64_t t_beg, t_end;   // types (ascending); empty = no type condition
    int64_t s_beg, s_end;   // positioned conditions (4 ints each: target, lb, ub, complement)
    int64_t r_beg, r_end;   // patterns (rows of p_off)
    int32_t arity;          // -1 = no ArityCondition
    int32_t pad;
};

enum QCtr { qCand = 0, qTyped, qArity, qHits, qInline, qNum = 5 };

__device__ __forceinline__ void wave_add_q(u64* ctr, u64 v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(ctr, v);
}

// type in the ascending list types[b, e)?  (one compare for AtomTypeCondition, a binary search for
// the subtype set of a TypePlusCondition)
__device__ __forceinline__ bool type_in(int32_t t, const int32_t* __restrict__ types, int64_t b, int64_t e) {
    if (e - b == 1) return types[b] == t;
    while (b < e) {
        const int64_t m = (b + e) >> 1;
        const int32_t v = types[m];
        if (v == t) return true;
        if (v < t) b = m + 1; else e = m;
    }
    return false;
}

// PositionedIncidentCondition.satisfies on one target row (C/query/PositionedIncidentCondition.java:123-177)
__device__ __forceinline__ bool positioned(const int32_t* __restrict__ row, int n, int32_t x, int32_t lb, int32_t ub,
                                           bool complement) {
    if (ub < 0) ub = n + ub;
    if (lb < 0) lb = n + lb;
    if (lb > ub || lb < 0 || ub < 0 || lb >= n || ub >= n) return false;
    if (complement) {
        for (int i = 0; i < lb; ++i)
            if (row[i] == x) return true;
        for (int i = ub + 1; i < n; ++i)
            if (row[i] == x) return true;
        return false;
    }
    for (int i = lb; i <= ub; ++i)
        if (row[i] == x) return true;
    return false;
}

// The same on a target row held in registers (n <= 8): unrolled, no indexed register access.
__device__ __forceinline__ bool positioned_regs(const int32_t (&tr)[8], int n, int32_t x, int32_t lb, int32_t ub,
                                                bool complement) {
    if (ub < 0) ub = n + ub;
    if (lb < 0) lb = n + lb;
    if (lb > ub || lb < 0 || ub < 0 || lb >= n || ub >= n) return false;
    bool f = false;
#pragma unroll
    for (int i = 0; i < 8; ++i) f |= (i < n) && ((i >= lb && i <= ub) != complement) && tr[i] == x;
    return f;
}

// Keys of the type-grouped incidence: (atom << 32 | type), value = link row; a stable radix sort
// keeps the rows of one (atom, type) ascending.  The owning atom of every entry comes from a max-scan
// over markers (atom + 1 at the first entry of each non-empty row), so the keys are written a thread
// per entry: the first version walked each row with one wavefront and a 1M-entry hub kept one wave
// busy for ~15 ms (36 ms for config 3).
__global__ void __launch_bounds__(256) k_ts_mark(int64_t A, const int64_t* __restrict__ inc_off,
                                                 int32_t* __restrict__ mark) {
    for (int64_t a = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; a < A; a += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = inc_off[a];
        if (inc_off[a + 1] > b) mark[b] = (int32_t)(a + 1);
    }
}

__global__ void __launch_bounds__(256) k_ts_keys(int64_t I, const int32_t* __restrict__ atom1,
                                                 const int32_t* __restrict__ inc_type, u64* __restrict__ keys) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < I; i += (int64_t)gridDim.x * blockDim.x)
        keys[i] = ((u64)(uint32_t)(atom1[i] - 1) << 32) | (uint32_t)inc_type[i];
}

__global__ void __launch_bounds__(256) k_low32(int64_t n, const u64* __restrict__ keys, int32_t* __restrict__ out) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = (int32_t)(uint32_t)keys[i];
}

// Inline target rows of the type-grouped incidence: one thread per entry writes the <= 8 targets of
// its link as two 16-byte stores (-1 padded; slot 0 = -2 marks arity > 8).
__global__ void __launch_bounds__(256) k_ts_inline(int64_t I, const int32_t* __restrict__ ts_row,
                                                   const int64_t* __restrict__ tgt_off,
                                                   const int32_t* __restrict__ tgt_idx, int4* __restrict__ out) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < I; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t L = ts_row[i];
        const int64_t b = tgt_off[L];
        const int n = (int)(tgt_off[L + 1] - b);
        int32_t t[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) t[k] = k < n ? tgt_idx[b + k] : -1;
        if (n > 8) t[0] = -2;
        out[2 * i] = make_int4(t[0], t[1], t[2], t[3]);
        out[2 * i + 1] = make_int4(t[4], t[5], t[6], t[7]);
    }
}

__device__ __forceinline__ int64_t lower_bound_i32(const int32_t* __restrict__ a, int64_t b, int64_t e, int32_t v) {
    // 8-ary steps while the range is long: 7 independent probes per step (log8 dependent loads
    // instead of log2), then one step of 8 independent probes
    while (e - b > 8) {
        const int64_t step = (e - b) >> 3;
        int c = 0;
#pragma unroll
        for (int j = 0; j < 7; ++j) c += a[b + (j + 1) * step] < v;
        const int64_t nb = c > 0 ? b + c * step + 1 : b;
        e = c < 7 ? b + (c + 1) * step : e;
        b = nb;
    }
    {   // <= 8 left: independent probes
        int c = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) c += (b + j < e) && a[b + j] < v;
        return b + c;
    }
}

// Plan per query (AndToQuery sorts the ORA inputs by size, :164-180): the anchor whose candidate
// range is smallest drives the scan.  With exactly one type the candidate range of an anchor is
// its type-T slice of the type-grouped incidence (the type index intersected for free); otherwise
// its whole incidence row with the streamed type filter.  pad = 1 marks a type-grouped plan.
// Plan of a query whose (distinct) anchors are in registers (na <= kRegAnchors).  The incidence
// bounds of every anchor are loaded together and the anchor with the fewest incident links drives
// the scan; with one type its type-T slice is found by an 8-ary search that brackets both bounds
// (`single`, `single + 1`) with probes issued together -- a chain of ~log8(deg) dependent loads per
// query.  (AndToQuery orders its ORA inputs by their size estimate; any anchor gives the same result
// set, the smallest untyped one only bounds the candidates.)
constexpr int kRegAnchors = 8;

__device__ __forceinline__ QPlan plan_regs(const int32_t (&av)[kRegAnchors], int na, int32_t single,
                                           const int64_t* __restrict__ inc_off, const int32_t* __restrict__ ts_type) {
    int64_t lo[kRegAnchors], hi[kRegAnchors];
#pragma unroll
    for (int k = 0; k < kRegAnchors; ++k) {
        lo[k] = k < na ? inc_off[av[k]] : 0;
        hi[k] = k < na ? inc_off[av[k] + 1] : 0;
    }
    QPlan p{0, 0, 0, 0};
    if (na == 0) return p;
    int best = 0;
#pragma unroll
    for (int k = 1; k < kRegAnchors; ++k)
        if (k < na && hi[k] - lo[k] < hi[best] - lo[best]) best = k;
    int64_t b = 0, e = 0;
#pragma unroll
    for (int k = 0; k < kRegAnchors; ++k)
        if (k == best) {
            b = lo[k];
            e = hi[k];
        }
    if (single >= 0) {
        int64_t b1 = b, e1 = e, b2 = b, e2 = e;   // brackets of lower_bound(single), lower_bound(single + 1)
        while (e1 - b1 > 8 || e2 - b2 > 8) {
            const int64_t s1 = (e1 - b1) >> 3, s2 = (e2 - b2) >> 3;
            int32_t p1[7], p2[7];
#pragma unroll
            for (int j = 0; j < 7; ++j) {
                p1[j] = ts_type[b1 + (j + 1) * s1];
                p2[j] = ts_type[b2 + (j + 1) * s2];
            }
            if (e1 - b1 > 8) {
                int c = 0;
#pragma unroll
                for (int j = 0; j < 7; ++j) c += p1[j] < single;
                const int64_t nb = c > 0 ? b1 + c * s1 + 1 : b1;
                e1 = c < 7 ? b1 + (c + 1) * s1 : e1;
                b1 = nb;
            }
            if (e2 - b2 > 8) {
                int c = 0;
#pragma unroll
                for (int j = 0; j < 7; ++j) c += p2[j] < single + 1;
                const int64_t nb = c > 0 ? b2 + c * s2 + 1 : b2;
                e2 = c < 7 ? b2 + (c + 1) * s2 : e2;
                b2 = nb;
            }
        }
        int32_t t1[8], t2[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            t1[j] = b1 + j < e1 ? ts_type[b1 + j] : INT32_MAX;
            t2[j] = b2 + j < e2 ? ts_type[b2 + j] : INT32_MAX;
        }
        int c1 = 0, c2 = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            c1 += t1[j] < single;
            c2 += t2[j] < single + 1;
        }
        b = b1 + c1;
        e = b2 + c2;
    }
    p.beg = b;
    p.n = e - b;
    p.amin = best;
    p.pad = single >= 0 ? 1 : 0;
    return p;
}

__device__ __forceinline__ QPlan plan_query(const QDesc& d, bool nop, const int32_t* __restrict__ anchors,
                                            const int32_t* __restrict__ types, const int64_t* __restrict__ inc_off,
                                            const int32_t* __restrict__ ts_type) {
    QPlan p{0, 0, 0, 0};
    if (nop) return p;
    const int32_t single = (d.t_end - d.t_beg == 1) ? types[d.t_beg] : -1;
    int64_t best = -1;
    for (int64_t k = d.a_beg; k < d.a_end; ++k) {
        const int32_t a = anchors[k];
        int64_t b = inc_off[a], e = inc_off[a + 1];
        if (single >= 0) {
            b = lower_bound_i32(ts_type, b, e, single);
            e = lower_bound_i32(ts_type, b, e, single + 1);
        }
        if (best < 0 || e - b < best) {
            best = e - b;
            p.beg = b;
            p.amin = (int32_t)(k - d.a_beg);
        }
    }
    p.n = best < 0 ? 0 : best;
    p.pad = single >= 0 ? 1 : 0;
    return p;
}

// Packed batch (hgx_pattern_batch_packed) normalised on the device, one thread per query:
// ExpressionBasedQuery.expand adds incident(x) for every non-ANY target of the orderedLink (:730-737),
// the toDNF HashSet drops duplicate anchors (:100).  The anchors of query q go to the fixed slot
// inc_off[q] + pat_off[q] (room for all of them), its type is type[q], its pattern row q of pat_off,
// so no scan is needed.  Bad queries are reported through err[0] (invalid) / err[1] (unsupported) as
// the smallest offending query index; the plan is computed in the same pass.
__device__ __forceinline__ QPlan norm_query(
    int32_t q, int64_t A, const int32_t* __restrict__ type, const int64_t* __restrict__ inc_off,
    const int32_t* __restrict__ inc, const int32_t* __restrict__ has_ordered, const int64_t* __restrict__ pat_off,
    const int32_t* __restrict__ pat, const int64_t* __restrict__ g_inc_off, const int32_t* __restrict__ ts_type,
    QDesc* __restrict__ desc, int32_t* __restrict__ anchors, int32_t* __restrict__ nop, int& status) {
    const int32_t tq = type[q];
    const int64_t b = inc_off[q], e = inc_off[q + 1];
    const bool ho = has_ordered[q] != 0;
    const int64_t pb = pat_off[q], pe = pat_off[q + 1];
    QDesc d;
    d.a_beg = b + pb;
    d.t_beg = q;
    d.t_end = q + (tq >= 0 ? 1 : 0);
    d.s_beg = d.s_end = 0;
    d.r_beg = q;
    d.r_end = q + (ho ? 1 : 0);
    d.arity = -1;
    d.pad = 0;
    bool bad = tq < -1 || e < b || pe < pb, unsup = false;
    int64_t na = 0;
    int32_t av[kRegAnchors];   // the first kRegAnchors distinct anchors also stay in registers
#pragma unroll
    for (int k = 0; k < kRegAnchors; ++k) av[k] = -1;
    auto add = [&](int32_t h) {
        if (h < 0 || h >= A) {
            bad = true;
            return;
        }
        bool dup = false;
#pragma unroll
        for (int k = 0; k < kRegAnchors; ++k) dup |= av[k] == h;
        for (int64_t k = kRegAnchors; k < na && !dup; ++k) dup = anchors[d.a_beg + k] == h;
        if (dup) return;
#pragma unroll
        for (int k = 0; k < kRegAnchors; ++k)
            if (k == na) av[k] = h;
        anchors[d.a_beg + na++] = h;
    };
    if (!bad) {
        for (int64_t i = b; i < e && !bad; ++i) add(inc[i]);
        if (ho) {
            if (pe - pb > kMaxPattern) unsup = true;
            for (int64_t i = pb; i < pe && !bad; ++i)
                if (pat[i] != HGX_ANY_HANDLE) add(pat[i]);
        }
    }
    d.a_end = d.a_beg + na;
    if (!bad && na == 0) unsup = true;
    if (na > kMaxAnchors) unsup = true;
    const bool isnop = ho && pe == pb;   // an empty OrderedLinkCondition compiles to HGQuery.NOP
    status = bad ? 1 : unsup ? 2 : 0;   // the caller reports the smallest offending query
    desc[q] = d;
    nop[q] = isnop ? 1 : 0;
    QPlan p{0, 0, 0, 0};
    if (!bad && !unsup && !isnop)
        p = na <= kRegAnchors ? plan_regs(av, (int)na, tq, g_inc_off, ts_type)
                              : plan_query(d, false, anchors, type, g_inc_off, ts_type);
    return p;
}

template <typename T>
__device__ __forceinline__ T block_exclusive_scan(T v, T* wsum, T& total) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
    T incl = v;
    for (int off = 1; off < 64; off <<= 1) {
        const T y = __shfl_up(incl, off);
        if (lane >= off) incl += y;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    T before = 0;
    total = 0;
    for (int k = 0; k < nw; ++k) {
        before += k < wv ? wsum[k] : (T)0;
        total += wsum[k];
    }
    __syncthreads();
    return before + incl - v;
}


// ---------------------------------------------------------------------------------------------
// Flat match (the only match since round 5; the per-query-chunk match of rounds 1-2 is gone).  The candidates of
// the batch form one flat space (query q owns [coff[q], coff[q+1])) cut into chunks of 64: a wave
// takes a chunk and each lane one candidate, whatever query it belongs to.  Half of the config-3
// queries have one candidate: with a wave per query chunk the batch was ~11K waves each running a
// chain of ~6 dependent loads for a handful of live lanes; flat it is ~4K full waves.  A lane finds
// its query in the chunk's window of coff (LDS), loads that query's plan / descriptor and checks
// its candidate on registers (inline record or target row).  Hits are compacted per chunk (flat
// order = query order, ascending candidates) and the chunk's hit mask gives every query its output
// offset: q_off[q] = outoff[coff[q] / 64] + popc(hitmask & bits below coff[q] % 64).
// ---------------------------------------------------------------------------------------------
constexpr int kFlatChunk = 64;

// Derived flat index (single-pass pipeline, at most kDerivedBlocks front blocks): the query offsets
// and the chunk owners come from the front kernel's block totals and in-block prefixes instead of a
// scan kernel.  Every workgroup of the match and of the placement sums the block totals itself into
// LDS (a few dozen values), so no launch sits between the front kernel and the match:
//   coff(q) = bp[q / 256] + lpre[q],  bp[b] = candidates of the front blocks before b.
// A chunk's owner (the last query whose candidates start at or before the chunk's first candidate)
// is found by a search over bp in LDS and one 256-entry window of lpre (a ballot per 64 entries).
constexpr int kDerivedBlocks = 256;

struct DIdx {
    const int64_t* bp;     // LDS [nb + 1]
    const int64_t* lpre;   // [n]
    int32_t nb, n;
    __device__ __forceinline__ int64_t coff(int64_t q) const { return q >= n ? bp[nb] : bp[q >> 8] + lpre[q]; }
};

// bp[0..nb] from blk (whole workgroup, 256 threads, nb <= 256); ends with a barrier.
__device__ __forceinline__ void didx_load(int64_t* bp, int64_t* ws, const int64_t* __restrict__ blk, int32_t nb) {
    const int64_t v = (int)threadIdx.x < nb ? blk[3 * threadIdx.x] : 0;
    int64_t tot;
    const int64_t ex = block_exclusive_scan<int64_t>(v, ws, tot);
    if ((int)threadIdx.x < nb) bp[threadIdx.x] = ex;
    if (threadIdx.x == 0) bp[nb] = tot;
    __syncthreads();
}

// Last query q with coff(q) <= x (strict: < x), -1 when there is none.  x is wave-uniform; the whole
// wave takes part and gets the same answer.
__device__ __forceinline__ int64_t didx_last(const DIdx& ix, int64_t x, bool strict) {
    int lo = 0, hi = ix.nb - 1, b = -1;   // last front block whose first query qualifies
    while (lo <= hi) {
        const int mid = (lo + hi) >> 1;
        const bool ok = strict ? ix.bp[mid] < x : ix.bp[mid] <= x;
        if (ok) {
            b = mid;
            lo = mid + 1;
        } else {
            hi = mid - 1;
        }
    }
    if (b < 0) return -1;
    const int lane = threadIdx.x & 63;
    const int64_t base = (int64_t)b * 256, t = x - ix.bp[b];
    int64_t v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int64_t q = base + i * 64 + lane;
        v[i] = q < ix.n ? ix.lpre[q] : INT64_MAX;
    }
    int c = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) c += __popcll(__ballot(strict ? v[i] < t : v[i] <= t));
    return base + c - 1;   // lpre is non-decreasing inside the block and lpre[base] = 0 qualifies
}

// One candidate against its query's conditions (the target row in registers, n <= 8).
__device__ __forceinline__ bool check_regs(const int32_t (&tr)[8], int n, const QDesc& d, int amin,
                                           const int32_t* __restrict__ anchors, const int32_t* __restrict__ pos,
                                           const int64_t* __restrict__ p_off, const int32_t* __restrict__ pattern) {
    bool hit = d.arity < 0 || n == d.arity;
    const int na = (int)(d.a_end - d.a_beg);
    for (int j = 0; j < na && hit; ++j) {   // IncidentCondition of every other anchor
        if (j == amin) continue;
        const int32_t a = anchors[d.a_beg + j];
        bool found = false;
#pragma unroll
        for (int i = 0; i < 8; ++i) found |= (i < n) && tr[i] == a;
        hit = found;
    }
    for (int64_t s = d.s_beg; s < d.s_end && hit; ++s)
        hit = positioned_regs(tr, n, pos[4 * s], pos[4 * s + 1], pos[4 * s + 2], pos[4 * s + 3] != 0);
    for (int64_t r = d.r_beg; r < d.r_end && hit; ++r) {   // OrderedLinkCondition: greedy subsequence
        const int64_t pb = p_off[r], np = p_off[r + 1] - pb;
        int64_t j = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i)
            if (i < n && j < np) {
                const int32_t pj = pattern[pb + j];
                if (pj < 0 || pj == tr[i]) ++j;
            }
        hit = (j == np);
    }
    return hit;
}

// The same on a target row in memory (links of arity > 8).
__device__ __forceinline__ bool check_mem(const int32_t* __restrict__ row, int n, const QDesc& d, int amin,
                                          const int32_t* __restrict__ anchors, const int32_t* __restrict__ pos,
                                          const int64_t* __restrict__ p_off, const int32_t* __restrict__ pattern) {
    bool hit = d.arity < 0 || n == d.arity;
    for (int64_t j = d.a_beg; j < d.a_end && hit; ++j) {
        if (j - d.a_beg == amin) continue;
        const int32_t a = anchors[j];
        bool found = false;
        for (int i = 0; i < n && !found; ++i) found = row[i] == a;
        hit = found;
    }
    for (int64_t s = d.s_beg; s < d.s_end && hit; ++s)
        hit = positioned(row, n, pos[4 * s], pos[4 * s + 1], pos[4 * s + 2], pos[4 * s + 3] != 0);
    for (int64_t r = d.r_beg; r < d.r_end && hit; ++r) {
        const int64_t pb = p_off[r], np = p_off[r + 1] - pb;
        int i = 0;
        int64_t j = 0;
        while (i < n && j < np) {
            const int32_t pj = pattern[pb + j];
            if (pj < 0 || pj == row[i]) ++j;
            ++i;
        }
        hit = (j == np);
    }
    return hit;
}

// D: the derived flat index (blk / lpre / nb; n_chunks_p, chq and coff unused), else the scanned one.
template <bool D>
__global__ void __launch_bounds__(256) hgx_pattern_match_flat(
    const int32_t* __restrict__ n_chunks_p, int32_t n, const int32_t* __restrict__ chq, const int64_t* __restrict__ coff,
    const QPlan* __restrict__ plan, const QDesc* __restrict__ desc, const int32_t* __restrict__ anchors,
    const int32_t* __restrict__ types, const int32_t* __restrict__ pos, const int64_t* __restrict__ p_off,
    const int32_t* __restrict__ pattern, const int32_t* __restrict__ inc_row, const int32_t* __restrict__ inc_type,
    const int32_t* __restrict__ inc_ts_row, const int64_t* __restrict__ tgt_off, const int32_t* __restrict__ tgt_idx,
    const int4* __restrict__ ts_tgt, int32_t* __restrict__ slots, int64_t* __restrict__ counts,
    u64* __restrict__ hitmask, u64* __restrict__ ctr, const int64_t* __restrict__ blk, const int64_t* __restrict__ lpre,
    int32_t nb, int64_t cap_chunks, int64_t cap_cand) {
    __shared__ int64_t win[4][kFlatChunk + 1];
    __shared__ int64_t bp[D ? kDerivedBlocks + 1 : 1], ws[4];
    int64_t* cw = win[threadIdx.x >> 6];
    DIdx ix{bp, lpre, nb, n};
    int64_t total;
    int32_t n_chunks;
    if (D) {
        didx_load(bp, ws, blk, nb);
        total = bp[nb];
        const int64_t tc = (total + kFlatChunk - 1) / kFlatChunk;
        n_chunks = (tc > cap_chunks || total > cap_cand) ? 0 : (int32_t)tc;
    } else {
        n_chunks = *n_chunks_p;
        total = coff[n];
    }
    auto qoff = [&](int64_t q) -> int64_t { return D ? ix.coff(q) : coff[q]; };
    const int lane = threadIdx.x & 63;
    const int64_t wave = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6));
    const int64_t nwave = ((int64_t)gridDim.x * blockDim.x) >> 6;
    const u64 lt = (1ull << lane) - 1ull;
    u64 n_cand = 0, n_typed = 0, n_ar = 0, n_hits = 0, n_inl = 0;
    for (int64_t k = wave; k < n_chunks; k += nwave) {
        const int32_t q0 = __builtin_amdgcn_readfirstlane(D ? (int32_t)didx_last(ix, k * kFlatChunk, false) : chq[k]);
        // the chunk's window of query offsets: queries q0 .. q0 + 64
        cw[lane] = q0 + lane <= n ? qoff(q0 + lane) : INT64_MAX;
        if (lane == 0) cw[kFlatChunk] = q0 + kFlatChunk <= n ? qoff(q0 + kFlatChunk) : INT64_MAX;
        __builtin_amdgcn_wave_barrier();
        const int64_t f = k * kFlatChunk + lane;
        const bool valid = f < total;
        int32_t q = q0;
        if (valid) {
            if (cw[kFlatChunk] <= f) {   // more than 64 queries in the chunk (empty ones): search coff
                int32_t lo = q0, hi = n - 1;
                while (lo < hi) {
                    const int32_t mid = (lo + hi + 1) >> 1;
                    if (qoff(mid) <= f) lo = mid; else hi = mid - 1;
                }
                q = lo;
            } else {
                int lo = 0, hi = kFlatChunk - 1;
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (cw[mid] <= f) lo = mid; else hi = mid - 1;
                }
                q = q0 + lo;
            }
        }
        bool hit = false;
        int32_t L = -1;
        if (valid) {
            const QPlan pl = plan[q];
            const QDesc d = desc[q];
            const int64_t ci = pl.beg + (f - qoff(q));
            const bool typed = d.t_end > d.t_beg && !pl.pad;
            hit = true;
            if (typed) {
                ++n_cand;
                hit = type_in(inc_type[ci], types, d.t_beg, d.t_end);
            }
            if (hit) {
                L = (pl.pad ? inc_ts_row : inc_row)[ci];
                ++n_typed;
                int32_t tr[8];
                bool have = false;
                if (pl.pad && ts_tgt) {
                    const int4 r0 = ts_tgt[2 * ci], r1 = ts_tgt[2 * ci + 1];
                    tr[0] = r0.x; tr[1] = r0.y; tr[2] = r0.z; tr[3] = r0.w;
                    tr[4] = r1.x; tr[5] = r1.y; tr[6] = r1.z; tr[7] = r1.w;
                    have = tr[0] != -2;
                }
                int nt = 0;
                if (have) {
#pragma unroll
                    for (int i = 0; i < 8; ++i) nt += tr[i] >= 0;
                    ++n_inl;
                    hit = check_regs(tr, nt, d, pl.amin, anchors, pos, p_off, pattern);
                } else {
                    const int64_t b = tgt_off[L];
                    nt = (int)(tgt_off[L + 1] - b);
                    n_ar += (u64)nt;
                    if (nt <= 8) {
#pragma unroll
                        for (int i = 0; i < 8; ++i) tr[i] = i < nt ? tgt_idx[b + i] : -1;
                        hit = check_regs(tr, nt, d, pl.amin, anchors, pos, p_off, pattern);
                    } else {
                        hit = check_mem(tgt_idx + b, nt, d, pl.amin, anchors, pos, p_off, pattern);
                    }
                }
            }
        }
        const u64 m = __ballot(hit);
        if (hit) slots[k * kFlatChunk + __popcll(m & lt)] = L;
        if (lane == 0) {
            counts[k] = __popcll(m);
            hitmask[k] = m;
        }
        n_hits += hit;
        __builtin_amdgcn_wave_barrier();
    }
    u64* c = ctr + (wave & (kQShards - 1)) * kQStride;
    wave_add_q(c + qCand, n_cand);
    wave_add_q(c + qTyped, n_typed);
    wave_add_q(c + qArity, n_ar);
    wave_add_q(c + qInline, n_inl);
    wave_add_q(c + qHits, n_hits);
}

// ---------------------------------------------------------------------------------------------
// Single-pass flat pipeline (HGX_OPT_QUERY_FLAT = 2, the default): four back-to-back kernels, no
// single-workgroup pass, no copy engine and no host round trip inside a batch.
//   hgx_q_norm_sp / hgx_q_plan_sp -- a thread per query: normalise + plan (packed batches, reading the
//        caller's arrays straight from the pinned staging area and keeping device copies of the
//        type and pattern columns the match reads) or plan (host-normalised batches); per block of 256
//        queries the candidate total and the smallest bad / unsupported query;
//   hgx_q_scan_sp   -- a block of 256 queries sums the candidate totals of the blocks before it (one
//        load per thread), scans its own queries, writes their candidate offsets, the chunk -> first
//        query map and the chunk -> first query at or past its start; the last block checks the
//        workspace and publishes the chunk count and statuses;
//   hgx_pattern_match_flat -- unchanged (a lane per candidate, per-chunk hit masks);
//   hgx_q_place     -- a block of 64 chunks sums the hit counts of the chunks before it (redundantly:
//        at most a few loads per thread), scans its own, and copies each chunk's hits as atom ids
//        into the mapped result area, then the result offsets of the queries starting in its chunks
//        (from its chunk offsets and their hit masks; a separate hgx_q_offsets_flat launch until
//        round 3 -- one launch and one dispatch gap fewer).
// Replaces norm + the one-workgroup scan (15 + 20 us on the config-3 batch), the one-workgroup finish
// + scatter (17 + 4 us) and the two copies (14 + 7 us, plus ~9 us of dispatch gap after each).
// Tried first: a decoupled look-back (blocks publishing prefixes through device-scope atomics) in
// the scan and in the match itself: 27 and 58 us -- each look-back step is a device-scope atomic
// round trip (the XCDs' L2 caches are not coherent with each other, so a plain store is not seen by
// a wave on another XCD, and a release store writes back the whole L2), so the redundant prefix sums
// that need no communication inside a kernel are faster.
constexpr int kSpBlock = 256;

template <typename T>
__device__ __forceinline__ T block_sum(T v, T* wsum) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = v;
    __syncthreads();
    T t = 0;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) t += wsum[k];
    __syncthreads();
    return t;
}

__device__ __forceinline__ int32_t block_min(int32_t v, int32_t* wmin) {
    for (int off = 32; off > 0; off >>= 1) v = min(v, __shfl_xor(v, off));
    if ((threadIdx.x & 63) == 0) wmin[threadIdx.x >> 6] = v;
    __syncthreads();
    int32_t t = INT32_MAX;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) t = min(t, wmin[k]);
    __syncthreads();
    return t;
}

// Packed batch: the inputs are the caller's arrays in the pinned staging area (read over the host
// link, no copy); the type, pattern-offset and pattern columns the match reads per candidate are
// copied to device memory.  blk[3b] = candidates of block b, blk[3b+1] / blk[3b+2] = its smallest
// bad / unsupported query (INT32_MAX: none).
__global__ void __launch_bounds__(kSpBlock) hgx_q_norm_sp(
    int32_t n, int64_t A, const int32_t* __restrict__ type, const int64_t* __restrict__ inc_off,
    const int32_t* __restrict__ inc, const int32_t* __restrict__ has_ordered, const int64_t* __restrict__ pat_off,
    const int32_t* __restrict__ pat, const int64_t* __restrict__ g_inc_off, const int32_t* __restrict__ ts_type,
    QDesc* __restrict__ desc, int32_t* __restrict__ anchors, int32_t* __restrict__ nop, QPlan* __restrict__ plan,
    int32_t* __restrict__ d_type, int64_t* __restrict__ d_poff, int32_t* __restrict__ d_pat, int64_t* __restrict__ ncand,
    int64_t* __restrict__ blk, int64_t* __restrict__ lpre, u64* __restrict__ ctr) {
    __shared__ int64_t ws[kSpBlock / 64];
    __shared__ int32_t wm[kSpBlock / 64];
    const int64_t q = (int64_t)blockIdx.x * kSpBlock + threadIdx.x;
    if (blockIdx.x == 0 && threadIdx.x < kQShards * kQStride) ctr[threadIdx.x] = 0ull;   // the match's counter shards
    QPlan p{0, 0, 0, 0};
    int32_t bad = INT32_MAX, uns = INT32_MAX;
    if (q < n) {
        int st = 0;
        p = norm_query((int32_t)q, A, type, inc_off, inc, has_ordered, pat_off, pat, g_inc_off, ts_type, desc, anchors,
                       nop, st);
        if (st == 1) bad = (int32_t)q;
        if (st == 2) uns = (int32_t)q;
        plan[q] = p;
        ncand[q] = p.n;
        d_type[q] = type[q];
        const int64_t pb = pat_off[q], pe = pat_off[q + 1];
        d_poff[q] = pb;
        if (q == n - 1) d_poff[n] = pe;
        for (int64_t i = pb; i < pe; ++i) d_pat[i] = pat[i];
    }
    int64_t tot;
    const int64_t lp = block_exclusive_scan<int64_t>(p.n, ws, tot);
    if (q < n) lpre[q] = lp;
    bad = block_min(bad, wm);
    uns = block_min(uns, wm);
    if (threadIdx.x == 0) {
        blk[3 * blockIdx.x] = tot;
        blk[3 * blockIdx.x + 1] = bad;
        blk[3 * blockIdx.x + 2] = uns;
    }
}

// Host-normalised batch (legacy / ext entry points): the plan of hgx_q_plan + the block totals.
__global__ void __launch_bounds__(kSpBlock) hgx_q_plan_sp(int32_t n, const QDesc* __restrict__ desc,
                                                         const int32_t* __restrict__ anchors,
                                                         const int32_t* __restrict__ types,
                                                         const int32_t* __restrict__ nop, const int64_t* __restrict__ inc_off,
                                                         const int32_t* __restrict__ ts_type, QPlan* __restrict__ plan,
                                                         int64_t* __restrict__ ncand, int64_t* __restrict__ blk,
                                                         int64_t* __restrict__ lpre, u64* __restrict__ ctr) {
    __shared__ int64_t ws[kSpBlock / 64];
    const int64_t q = (int64_t)blockIdx.x * kSpBlock + threadIdx.x;
    if (blockIdx.x == 0 && threadIdx.x < kQShards * kQStride) ctr[threadIdx.x] = 0ull;
    QPlan p{0, 0, 0, 0};
    if (q < n) {
        const QDesc d = desc[q];
        if (d.a_end - d.a_beg <= kRegAnchors && !nop[q]) {
            int32_t av[kRegAnchors];
            const int na = (int)(d.a_end - d.a_beg);
#pragma unroll
            for (int k = 0; k < kRegAnchors; ++k) av[k] = k < na ? anchors[d.a_beg + k] : 0;
            p = plan_regs(av, na, (d.t_end - d.t_beg == 1) ? types[d.t_beg] : -1, inc_off, ts_type);
        } else {
            p = plan_query(d, nop[q] != 0, anchors, types, inc_off, ts_type);
        }
        plan[q] = p;
        ncand[q] = p.n;
    }
    int64_t tot;
    const int64_t lp = block_exclusive_scan<int64_t>(p.n, ws, tot);
    if (q < n) lpre[q] = lp;
    if (threadIdx.x == 0) {
        blk[3 * blockIdx.x] = tot;
        blk[3 * blockIdx.x + 1] = INT32_MAX;
        blk[3 * blockIdx.x + 2] = INT32_MAX;
    }
}

// Candidate offsets: block b = queries [256 b, 256 b + 256).  stat (mapped result area): [0] chunks,
// [1] candidates, [2] workspace overflow (the match then sees no chunks), [4] / [5] smallest bad /
// unsupported query.
__global__ void __launch_bounds__(kSpBlock) hgx_q_scan_sp(int32_t n, const int64_t* __restrict__ ncand,
                                                         const int64_t* __restrict__ blk, int64_t* __restrict__ coff,
                                                         int32_t* __restrict__ chq, int32_t* __restrict__ n_chunks_out,
                                                         int64_t cap_chunks, int64_t cap_cand, int64_t* __restrict__ stat,
                                                         u64* __restrict__ ctr) {
    __shared__ int64_t ws[kSpBlock / 64];
    __shared__ int32_t wm[kSpBlock / 64];
    const int b = blockIdx.x, nb = gridDim.x;
    const bool last = b == nb - 1;
    const int64_t q = (int64_t)b * kSpBlock + threadIdx.x;
    const int64_t c = q < n ? ncand[q] : 0;   // issued before the block totals are summed
    // the candidates of the blocks before this one (the last block: of all blocks, + the statuses)
    int64_t before = 0;
    int32_t bad = INT32_MAX, uns = INT32_MAX;
    for (int j = threadIdx.x; j < (last ? nb : b); j += kSpBlock) {
        const int64_t t = blk[3 * j];
        if (j < b) before += t;
        if (last) {
            bad = min(bad, (int32_t)blk[3 * j + 1]);
            uns = min(uns, (int32_t)blk[3 * j + 2]);
        }
    }
    const int64_t pre = block_sum<int64_t>(before, ws);
    int64_t btot;
    const int64_t ex = pre + block_exclusive_scan<int64_t>(c, ws, btot);
    if (q < n) {
        coff[q] = ex;
        // the chunks whose first candidate is one of q's (beyond the workspace: overflow, re-run)
        for (int64_t k = (ex + kFlatChunk - 1) / kFlatChunk; k * kFlatChunk < ex + c && k < cap_chunks; ++k)
            chq[k] = (int32_t)q;
    }
    if (b == 0 && threadIdx.x < kQShards * kQStride) ctr[threadIdx.x] = 0ull;   // the match's counter shards
    if (last) {
        bad = block_min(bad, wm);
        uns = block_min(uns, wm);
        if (threadIdx.x == 0) {
            const int64_t tk = pre + btot, tc = (tk + kFlatChunk - 1) / kFlatChunk;
            const bool over = tc > cap_chunks || tk > cap_cand;
            coff[n] = tk;
            *n_chunks_out = over ? 0 : (int32_t)tc;
            stat[0] = tc;
            stat[1] = tk;
            stat[2] = over ? 1 : 0;
            stat[4] = bad;
            stat[5] = uns;
        }
    }
}

// Placement: block b = chunks [64 b, 64 b + 64): wave 0 scans their hit counts (after summing the
// counts of the chunks before the block), then each wave places the hits of 16 chunks with all 16 slot
// loads, then all 16 link-atom loads, in flight (two dependent rounds instead of one per chunk).
// outoff[n_chunks] = total hits; the block holding the last chunk (block 0 when there is none)
// publishes the hit total and the summed counter shards.
constexpr int kPlaceChunks = 64;
// Above this many placement blocks the prefix of the chunk hit counts before each block comes from
// a two-launch scan (hgx_q_place_bsum + hgx_q_place_bscan) instead of each block summing every chunk
// before it, which grows with the square of the chunk count.
constexpr int64_t kPlaceDirectBlocks = 256;

// bsum[b] = hit count of placement block b's chunks (one thread per block).
__global__ void __launch_bounds__(256) hgx_q_place_bsum(const int32_t* __restrict__ n_chunks_p,
                                                       const int64_t* __restrict__ counts, int64_t nbp,
                                                       int64_t* __restrict__ bsum) {
    const int32_t nc = *n_chunks_p;
    for (int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; b < nbp; b += (int64_t)gridDim.x * blockDim.x) {
        int64_t v = 0;
        const int64_t k0 = b * kPlaceChunks, k1 = min<int64_t>(nc, k0 + kPlaceChunks);
        for (int64_t k = k0; k < k1; ++k) v += counts[k];
        bsum[b] = v;
    }
}

// In-place exclusive scan of bsum[0, nbp) by one workgroup (1024 entries a round, carried).
__global__ void __launch_bounds__(1024) hgx_q_place_bscan(int64_t nbp, int64_t* __restrict__ bsum) {
    __shared__ int64_t wsum[16];
    __shared__ int64_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int64_t b0 = 0; b0 < nbp; b0 += 1024) {
        const int64_t b = b0 + threadIdx.x;
        const int64_t v = b < nbp ? bsum[b] : 0;
        int64_t x = v;
        for (int off = 1; off < 64; off <<= 1) {
            const int64_t y = __shfl_up(x, off);
            if (lane >= off) x += y;
        }
        if (lane == 63) wsum[w] = x;
        __syncthreads();
        int64_t base = carry, tot = 0;
        for (int k = 0; k < 16; ++k) {
            base += k < w ? wsum[k] : 0;
            tot += wsum[k];
        }
        if (b < nbp) bsum[b] = base + x - v;
        __syncthreads();
        if (threadIdx.x == 0) carry += tot;
        __syncthreads();
    }
}
// D: the derived flat index (blk / lpre / nb; n_chunks_p, chq and coff unused; the block holding the last
// chunk also publishes the chunk / candidate totals, the overflow flag and the bad / unsupported
// queries), else the scanned one.
template <bool D>
__global__ void __launch_bounds__(256) hgx_q_place(const int32_t* __restrict__ n_chunks_p,
                                                  const int64_t* __restrict__ counts, const int32_t* __restrict__ slots,
                                                  const int32_t* __restrict__ link_atom, int64_t* __restrict__ outoff,
                                                  int32_t* __restrict__ ids, int64_t* __restrict__ stat,
                                                  const u64* __restrict__ ctr, u64* __restrict__ ctr_out, int32_t n,
                                                  const int32_t* __restrict__ chq, const int64_t* __restrict__ coff,
                                                  const u64* __restrict__ hitmask, int64_t* __restrict__ q_off,
                                                  const int64_t* __restrict__ bpre, const int64_t* __restrict__ blk,
                                                  const int64_t* __restrict__ lpre, int32_t nb, int64_t cap_chunks,
                                                  int64_t cap_cand, u64* __restrict__ ticket, u64 seq) {
    __shared__ int64_t ws[4], c_off[kPlaceChunks], qb[2];
    __shared__ int32_t c_cnt[kPlaceChunks];
    __shared__ int64_t bp[D ? kDerivedBlocks + 1 : 1];
    __shared__ int32_t wm[4];
    DIdx ix{bp, lpre, nb, n};
    int32_t nc;
    bool over;
    if (D) {
        didx_load(bp, ws, blk, nb);
        const int64_t tk = bp[nb], tc = (tk + kFlatChunk - 1) / kFlatChunk;
        over = tc > cap_chunks || tk > cap_cand;
        nc = over ? 0 : (int32_t)tc;
    } else {
        nc = *n_chunks_p;
        over = stat[2] != 0;
    }
    auto qoff = [&](int64_t q) -> int64_t { return D ? ix.coff(q) : coff[q]; };
    const int64_t k0 = (int64_t)blockIdx.x * kPlaceChunks;
    if (k0 > 0 && k0 >= nc) return;   // beyond the chunks (block 0 always runs: it publishes an empty result)
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t k = k0 + lane;
    const int32_t cnt = wv == 0 && k < nc ? (int32_t)counts[k] : 0;   // issued before the prefix loads
    const bool holds_last = nc == 0 ? blockIdx.x == 0 : (nc - 1) / kPlaceChunks == (int32_t)blockIdx.x;
    // The queries whose first candidate lies in this block's chunks, [qb[0], qb[1]) (the block of the last
    // chunk: through n), whose result offsets the block writes below.  Boundary kb -> the first query
    // with a candidate offset >= kb * kFlatChunk: one past chunk kb's owner chq[kb] unless the owner's
    // candidates start exactly there, then at or before it (zero-candidate queries share that offset:
    // 64 at a time, one ballot).  Waves 2 and 3 find the two boundaries while wave 0 sums the counts.
    if (wv >= 2) {
        const int e = wv - 2;
        const int64_t kb = k0 + e * kPlaceChunks;
        int64_t res = 0;
        if (e == 1 && holds_last) {
            res = (int64_t)n + 1;
        } else if (kb > 0 && !over) {
            const int64_t target = kb * kFlatChunk;
            if (D) {
                res = didx_last(ix, target, true) + 1;
            } else {
                const int64_t q0 = chq[kb];
                if (coff[q0] < target) {
                    res = q0 + 1;
                } else {
                    for (int64_t hi = q0;; hi -= 64) {   // wave-uniform; coff[hi] >= target
                        const int64_t j = hi - 64 + lane;
                        const u64 m = __ballot(j < 0 || coff[j < 0 ? 0 : j] < target);
                        if (m) {
                            res = hi - 64 + (63 - __clzll((long long)m)) + 1;
                            break;
                        }
                    }
                }
            }
        }
        if (lane == 0) qb[e] = res;
    }
    int64_t before = 0;   // hit counts of the chunks before this block, eight loads in flight per thread
    if (!bpre) {          // (large batches: the scanned block sums instead)
        for (int64_t j = threadIdx.x; j < k0; j += 8 * 256) {
            int64_t v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = j + u * 256 < k0 ? counts[j + u * 256] : 0;
#pragma unroll
            for (int u = 0; u < 8; ++u) before += v[u];
        }
    } else if (threadIdx.x == 0) {
        before = bpre[blockIdx.x];
    }
    const int64_t pre = block_sum<int64_t>(before, ws);
    if (wv == 0) {
        int64_t incl = cnt;
        for (int off = 1; off < 64; off <<= 1) {
            const int64_t y = __shfl_up(incl, off);
            if (lane >= off) incl += y;
        }
        const int64_t ex = pre + incl - cnt;
        if (k < nc) outoff[k] = ex;
        c_off[lane] = ex;
        c_cnt[lane] = cnt;
        if (lane == 63) ws[0] = pre + incl;   // total through this block
    }
    __syncthreads();
    int32_t row[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
        const int cc = wv * 16 + u;
        row[u] = lane < c_cnt[cc] ? slots[(k0 + cc) * kFlatChunk + lane] : -1;
    }
    int32_t at[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) at[u] = row[u] >= 0 ? link_atom[row[u]] : 0;
#pragma unroll
    for (int u = 0; u < 16; ++u)
        if (row[u] >= 0) ids[c_off[wv * 16 + u] + lane] = at[u];
    // the result offsets of the queries starting in this block's chunks, from the chunk offsets in LDS
    // and the chunk's hit mask (the offsets launch folded in)
    if (!over) {
        for (int64_t q = qb[0] + threadIdx.x; q < qb[1]; q += 256) {
            const int64_t cf = qoff(q), kq = cf / kFlatChunk, lc = kq - k0;
            const u64 hm = kq < nc ? hitmask[kq] : 0ull;
            q_off[q] = (lc < kPlaceChunks ? c_off[lc] : ws[0]) + __popcll(hm & ((1ull << (cf % kFlatChunk)) - 1ull));
        }
    }
    if (holds_last) {
        if (D) {   // the scan kernel's statistics: totals, overflow, smallest bad / unsupported query
            int32_t bad = INT32_MAX, uns = INT32_MAX;
            for (int j = threadIdx.x; j < nb; j += 256) {
                bad = min(bad, (int32_t)blk[3 * j + 1]);
                uns = min(uns, (int32_t)blk[3 * j + 2]);
            }
            bad = block_min(bad, wm);
            uns = block_min(uns, wm);
            if (threadIdx.x == 0) {
                const int64_t tk = bp[nb];
                stat[0] = (tk + kFlatChunk - 1) / kFlatChunk;
                stat[1] = tk;
                stat[2] = over ? 1 : 0;
                stat[4] = bad;
                stat[5] = uns;
            }
        }
        if (threadIdx.x == 0) {
            const int64_t tot = ws[0];
            outoff[nc] = tot;
            stat[3] = over ? 0 : tot;
        }
        if (threadIdx.x < qNum) {
            u64 v = 0;
            for (int sh = 0; sh < kQShards; ++sh) v += ctr[sh * kQStride + threadIdx.x];
            ctr_out[threadIdx.x] = v;
        }
    }
    if (ticket) {   // completion flag: the last active block to finish publishes seq into stat[7]
        __shared__ bool last_block;
        __syncthreads();   // this block's result stores are issued
        if (threadIdx.x == 0) {
            __threadfence_system();
            const u64 n_active = nc == 0 ? 1ull : (u64)((nc + kPlaceChunks - 1) / kPlaceChunks);
            last_block = atomicAdd(ticket, 1ull) == n_active - 1ull;
            if (last_block) {
                *ticket = 0ull;
                __threadfence_system();
                __hip_atomic_store((u64*)(stat + 7), seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
}



// lower_bound(v1) and lower_bound(v2) (v1 < v2) in the ascending a[b, e), the bounds of a type slice.
// A range of <= 64 entries is read in one coalesced load; a longer one is narrowed 16x a round by 16
// strided probes (16 lines, one dependent load a round).  While both bounds share their range (the
// first round) one probe set serves both.
__device__ __forceinline__ void slice_bounds(const int32_t* __restrict__ a, int32_t v1, int32_t v2, int64_t b,
                                             int64_t e, int64_t& r1, int64_t& r2, u64& probes) {
    const int lane = threadIdx.x & 63;
    int64_t b1 = b, e1 = e, b2 = b, e2 = e;
    r1 = -1;
    r2 = -1;
    auto narrow = [&](int64_t& bb, int64_t& ee, int64_t st, int c, int64_t& r) {
        if (st == 1 || c == 0) {
            r = bb + (st == 1 ? c : 0);
            return;
        }
        const int64_t nb = bb + (int64_t)(c - 1) * st + 1;
        ee = bb + (int64_t)c * st < ee ? bb + (int64_t)c * st : ee;
        bb = nb;
    };
    while (r1 < 0 || r2 < 0) {   // wave-uniform
        if (r1 < 0 && r2 < 0 && b1 == b2 && e1 == e2) {   // shared range
            const int64_t span = e1 - b1;
            const int np = span <= 64 ? 64 : 16;
            const int64_t st = span <= 64 ? 1 : (span + 15) / 16;
            const int64_t p = b1 + (int64_t)lane * st;
            const bool in = lane < np && p < e1;
            const int32_t x = in ? a[p] : INT32_MAX;
            const int c1 = __popcll(__ballot(in && x < v1)), c2 = __popcll(__ballot(in && x < v2));
            probes += (u64)__popcll(__ballot(in));
            narrow(b1, e1, st, c1, r1);
            narrow(b2, e2, st, c2, r2);
            continue;
        }
        // separate ranges: lanes 0-31 serve bound 1, lanes 32-63 bound 2
        const bool hi = lane >= 32;
        const int l = lane & 31;
        const int64_t bb = hi ? b2 : b1, ee = hi ? e2 : e1;
        const bool live = hi ? r2 < 0 : r1 < 0;
        const int64_t span = ee - bb;
        const int np = span <= 32 ? 32 : 16;
        const int64_t st = span <= 32 ? 1 : (span + 15) / 16;
        const int64_t p = bb + (int64_t)l * st;
        const bool in = live && l < np && p < ee;
        const int32_t x = in ? a[p] : INT32_MAX;
        const u64 m = __ballot(in && x < (hi ? v2 : v1));
        probes += (u64)__popcll(__ballot(in));
        const int64_t st1 = __shfl(st, 0), st2 = __shfl(st, 32);
        if (r1 < 0) narrow(b1, e1, st1, __popcll(m & 0xffffffffull), r1);
        if (r2 < 0) narrow(b2, e2, st2, __popcll(m >> 32), r2);
    }
}

}  // namespace hgx

using namespace hgx;

struct hgx_query_result {
    int32_t n = 0;
    std::vector<int64_t> offsets;
    std::vector<int32_t> ids;
    double ms_total = 0, ms_match = 0, bytes_match = 0;
    // caller buffers (hgx_pattern_batch_set_into): the single-pass back end copies the offsets and,
    // when they fit, the ids straight from the mapped result area into them
    int64_t* ext_off = nullptr;
    int32_t* ext_ids = nullptr;
    int64_t ext_cap = 0, n_hits = 0;
};

// A packed batch resident in device memory (hgx_query_set_create), in the staging layout of the
// packed front end.
struct hgx_query_set {
    int device = 0;
    int32_t n = 0;
    size_t o_type = 0, o_ioff = 0, o_inc = 0, o_ho = 0, o_poff = 0, o_pat = 0, o_err = 0, bytes = 0;
    int64_t n_inc = 0, n_pat = 0;
    char* dev = nullptr;
};

namespace {

double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// One query as handed over by any of the entry points.
struct QueryIn {
    int32_t n_types = 0;
    const int32_t* types = nullptr;
    int32_t n_inc = 0;
    const int32_t* inc = nullptr;
    int32_t n_pos = 0;
    const int32_t* pos = nullptr;     // 4 ints each
    int32_t n_pat = 0;                // OrderedLinkConditions
    const int64_t* pat_off = nullptr; // [n_pat + 1] into pat
    const int32_t* pat = nullptr;
    int32_t arity = -1;
};

// Normalised batch: ExpressionBasedQuery.expand (orderedLink adds incident(x) for each non-ANY x,
// :730-737) + the toDNF HashSet dedupe (:100) -> per query: types, distinct anchors, positioned
// conditions, patterns, arity, nop.
struct NormBatch {
    std::vector<QDesc> desc;
    std::vector<int32_t> nop;
    std::vector<int32_t> anchors, types, pos, pattern;
    std::vector<int64_t> p_off{0};
};

template <class Get>
void normalise(hgx_graph* g, int32_t n, Get get, NormBatch& nb) {
    nb.desc.resize(n);
    nb.nop.assign(n, 0);
    nb.anchors.reserve((size_t)n * 3);
    nb.types.reserve((size_t)n);
    nb.pattern.reserve((size_t)n * 3);
    nb.p_off.reserve((size_t)n + 1);
    for (int32_t q = 0; q < n; ++q) {
        QueryIn in;
        get(q, in);
        auto qs = [q] { return std::to_string(q); };   // built only on the error paths
        if (in.n_types < 0 || in.n_inc < 0 || in.n_pos < 0 || in.n_pat < 0 || (in.n_types > 0 && !in.types) ||
            (in.n_inc > 0 && !in.inc) || (in.n_pos > 0 && !in.pos) || (in.n_pat > 0 && (!in.pat_off)) || in.arity < -1)
            fail(HGX_E_INVALID, "hgx_pattern_batch: bad query " + qs());
        if (in.n_types > kMaxTypes || in.n_pos > kMaxPositioned || in.n_pat > kMaxPatterns)
            fail(HGX_E_UNSUPPORTED, "hgx_pattern_batch: query " + qs() + " exceeds the condition limits");
        QDesc& d = nb.desc[q];
        d.arity = in.arity;
        // types: an Or of exact types (ascending, duplicates dropped)
        d.t_beg = (int64_t)nb.types.size();
        for (int32_t i = 0; i < in.n_types; ++i) {
            if (in.types[i] < 0) fail(HGX_E_INVALID, "hgx_pattern_batch: bad type in query " + qs());
            nb.types.push_back(in.types[i]);
        }
        if (in.n_types > 1) {
            std::sort(nb.types.begin() + d.t_beg, nb.types.end());
            nb.types.erase(std::unique(nb.types.begin() + d.t_beg, nb.types.end()), nb.types.end());
        }
        d.t_end = (int64_t)nb.types.size();
        // anchors
        d.a_beg = (int64_t)nb.anchors.size();
        auto add = [&](int32_t h) {
            if (h < 0 || h >= g->A) fail(HGX_E_INVALID, "hgx_pattern_batch: atom id out of range in query " + qs());
            for (size_t k = (size_t)d.a_beg; k < nb.anchors.size(); ++k)
                if (nb.anchors[k] == h) return;
            nb.anchors.push_back(h);
        };
        for (int32_t i = 0; i < in.n_inc; ++i) add(in.inc[i]);
        d.s_beg = (int64_t)nb.pos.size() / 4;
        for (int32_t i = 0; i < in.n_pos; ++i) {   // its ORA set is inc(target): the target anchors the scan
            add(in.pos[4 * i]);
            for (int k = 0; k < 4; ++k) nb.pos.push_back(in.pos[4 * i + k]);
        }
        d.s_end = (int64_t)nb.pos.size() / 4;
        d.r_beg = (int64_t)nb.p_off.size() - 1;
        for (int32_t r = 0; r < in.n_pat; ++r) {
            const int64_t b = in.pat_off[r], m = in.pat_off[r + 1] - b;
            if (m < 0 || (m > 0 && !in.pat)) fail(HGX_E_INVALID, "hgx_pattern_batch: bad pattern in query " + qs());
            if (m > kMaxPattern) fail(HGX_E_UNSUPPORTED, "hgx_pattern_batch: ordered pattern too long");
            // an empty OrderedLinkCondition gets QueryMetaData.EMPTY, lands in ORA and compiles to HGQuery.NOP
            if (m == 0) nb.nop[q] = 1;
            for (int64_t i = 0; i < m; ++i) {
                const int32_t p = in.pat[b + i];
                if (p != HGX_ANY_HANDLE) {
                    if (p < 0) fail(HGX_E_INVALID, "hgx_pattern_batch: bad pattern id");
                    add(p);
                }
                nb.pattern.push_back(p);
            }
            nb.p_off.push_back((int64_t)nb.pattern.size());
        }
        d.r_end = (int64_t)nb.p_off.size() - 1;
        d.a_end = (int64_t)nb.anchors.size();
        if (d.a_end == d.a_beg)
            fail(HGX_E_UNSUPPORTED, "hgx_pattern_batch: query " + qs() + " has no incidence anchor");
        if (d.a_end - d.a_beg > kMaxAnchors) fail(HGX_E_UNSUPPORTED, "hgx_pattern_batch: too many anchors");
    }
}

int run_batch(hgx_graph* g, int32_t n, NormBatch& nb, hgx_query_result** out);
int run_batch_packed(hgx_graph* g, int32_t n, const int32_t* type, const int64_t* inc_off, const int32_t* inc,
                     const int32_t* has_ordered, const int64_t* pat_off, const int32_t* pat, hgx_query_result** out);

}  // namespace

extern "C" int hgx_pattern_batch(hgx_graph* g, const hgx_and_query* qs, int32_t n, hgx_query_result** out) {
    HGX_API_BEGIN
    if (!g || !out || n < 0 || (n > 0 && !qs)) fail(HGX_E_INVALID, "hgx_pattern_batch: bad argument");
    *out = nullptr;
    NormBatch nb;
    std::vector<int64_t> one_off;
    normalise(g, n,
              [&](int32_t q, QueryIn& in) {
                  if (qs[q].type < HGX_NO_TYPE) fail(HGX_E_INVALID, "hgx_pattern_batch: bad type");
                  in.n_types = qs[q].type >= 0 ? 1 : 0;
                  in.types = &qs[q].type;
                  in.n_inc = qs[q].n_incident;
                  in.inc = qs[q].incident;
                  one_off.assign({0, (int64_t)std::max(qs[q].n_pattern, 0)});
                  in.n_pat = qs[q].has_ordered ? 1 : 0;
                  in.pat_off = one_off.data();
                  in.pat = qs[q].pattern;
              },
              nb);
    return run_batch(g, n, nb, out);
    HGX_API_END
}

extern "C" int hgx_pattern_batch_packed(hgx_graph* g, int32_t n, const int32_t* type, const int64_t* inc_off,
                                        const int32_t* inc, const int32_t* has_ordered, const int64_t* pat_off,
                                        const int32_t* pat, hgx_query_result** out) {
    HGX_API_BEGIN
    if (!g || !out || n < 0 || (n > 0 && (!type || !inc_off || !pat_off || !has_ordered)))
        fail(HGX_E_INVALID, "hgx_pattern_batch_packed: bad argument");
    *out = nullptr;
    return run_batch_packed(g, n, type, inc_off, inc, has_ordered, pat_off, pat, out);
    HGX_API_END
}

extern "C" int hgx_pattern_batch_ext(hgx_graph* g, int32_t n, const int64_t* type_off, const int32_t* types,
                                     const int64_t* inc_off, const int32_t* inc, const int64_t* pos_off,
                                     const int32_t* pos, const int64_t* pset_off, const int64_t* pat_off,
                                     const int32_t* pat, const int32_t* arity, hgx_query_result** out) {
    HGX_API_BEGIN
    if (!g || !out || n < 0 || (n > 0 && (!type_off || !inc_off || !pos_off || !pset_off || !arity)))
        fail(HGX_E_INVALID, "hgx_pattern_batch_ext: bad argument");
    *out = nullptr;
    NormBatch nb;
    normalise(g, n,
              [&](int32_t q, QueryIn& in) {
                  in.n_types = (int32_t)(type_off[q + 1] - type_off[q]);
                  in.types = types ? types + type_off[q] : nullptr;
                  in.n_inc = (int32_t)(inc_off[q + 1] - inc_off[q]);
                  in.inc = inc ? inc + inc_off[q] : nullptr;
                  in.n_pos = (int32_t)(pos_off[q + 1] - pos_off[q]);
                  in.pos = pos ? pos + 4 * pos_off[q] : nullptr;
                  in.n_pat = (int32_t)(pset_off[q + 1] - pset_off[q]);
                  if (in.n_pat > 0 && !pat_off) fail(HGX_E_INVALID, "hgx_pattern_batch_ext: null pat_off");
                  in.pat_off = pat_off ? pat_off + pset_off[q] : nullptr;
                  in.pat = pat;
                  in.arity = arity[q];
              },
              nb);
    return run_batch(g, n, nb, out);
    HGX_API_END
}

namespace {

// Type-grouped incidence index, once per snapshot (a stable radix sort of (atom, type) keys with
// the link row as value keeps each (atom, type) slice ascending).
void ensure_ts_inline(hgx_graph* g);

void ensure_type_grouped(hgx_graph* g) {
    if (g->inc_ts_row || g->I == 0) return;
    if (g->base) {   // an execution context: the snapshot builds the index once and every context borrows it
        hgx_graph* b = g->base;
        {
            std::lock_guard<std::mutex> lk(b->mu);   // lock order: context, then its snapshot (never the reverse)
            HGX_HIP(hipSetDevice(b->device));
            ensure_type_grouped(b);
            if (g->q_inline) ensure_ts_inline(b);
            HGX_HIP(hipStreamSynchronize(b->stream));
        }
        g->inc_ts_row = b->inc_ts_row;
        g->inc_ts_type = b->inc_ts_type;
        g->inc_ts_tgt = b->inc_ts_tgt;
        if (!b->inc_ts_tgt) g->q_inline = false;
        return;
    }
    hipStream_t s = g->stream;
    const int64_t I = g->I;
    u64* keys = (u64*)g->alloc(sizeof(u64) * I);
    u64* keys2 = (u64*)g->alloc(sizeof(u64) * I);
    int32_t* rows2 = (int32_t*)g->alloc(sizeof(int32_t) * I);
    {   // owning atom of every entry: markers, max-scan, keys
        int32_t* mark = (int32_t*)g->alloc(sizeof(int32_t) * I);
        int32_t* atom1 = (int32_t*)g->alloc(sizeof(int32_t) * I);
        HGX_HIP(hipMemsetAsync(mark, 0, sizeof(int32_t) * I, s));
        k_ts_mark<<<grid_for(g->A, 256, 65536), 256, 0, s>>>(g->A, g->inc_off, mark);
        HGX_CHECK_LAUNCH();
        size_t sb = 0;
        HGX_HIP(rocprim::inclusive_scan(nullptr, sb, mark, atom1, (size_t)I, rocprim::maximum<int32_t>(), s));
        void* st = g->alloc(sb);
        HGX_HIP(rocprim::inclusive_scan(st, sb, mark, atom1, (size_t)I, rocprim::maximum<int32_t>(), s));
        k_ts_keys<<<grid_for(I, 256, 65536), 256, 0, s>>>(I, atom1, g->inc_type, keys);
        HGX_CHECK_LAUNCH();
        HGX_HIP(hipStreamSynchronize(s));
        g->release(st, sb);
        g->release(mark, sizeof(int32_t) * I);
        g->release(atom1, sizeof(int32_t) * I);
    }
    int end_bit = 64;
    {
        int ab = 1;
        while (((int64_t)1 << ab) <= g->A) ab++;
        end_bit = std::min(64, 32 + ab);
    }
    size_t tb = 0;
    HGX_HIP(rocprim::radix_sort_pairs(nullptr, tb, keys, keys2, g->inc_row, rows2, (size_t)I, 0u, (unsigned)end_bit, s));
    void* tmp = g->alloc(tb);
    HGX_HIP(rocprim::radix_sort_pairs(tmp, tb, keys, keys2, g->inc_row, rows2, (size_t)I, 0u, (unsigned)end_bit, s));
    int32_t *ts_row = nullptr, *ts_type = nullptr;
    HGX_HIP(hipMalloc(&ts_row, sizeof(int32_t) * I));
    HGX_HIP(hipMalloc(&ts_type, sizeof(int32_t) * I));
    HGX_HIP(hipMemcpyAsync(ts_row, rows2, sizeof(int32_t) * I, hipMemcpyDeviceToDevice, s));
    k_low32<<<grid_for(I, 256), 256, 0, s>>>(I, keys2, ts_type);
    HGX_CHECK_LAUNCH();
    HGX_HIP(hipStreamSynchronize(s));
    g->release(tmp, tb);
    g->release(keys, sizeof(u64) * I);
    g->release(keys2, sizeof(u64) * I);
    g->release(rows2, sizeof(int32_t) * I);
    g->inc_ts_row = ts_row;
    g->inc_ts_type = ts_type;
}

// Inline target records of the type-grouped incidence (32 B per entry), built after the index when
// HGX_OPT_QUERY_INLINE is on and the device has room for them (a quarter of the free memory at most).
void ensure_ts_inline(hgx_graph* g) {
    if (!g->q_inline || g->inc_ts_tgt || !g->inc_ts_row || g->I == 0) return;
    const size_t bytes = (size_t)32 * (size_t)g->I;
    size_t free_b = 0, total_b = 0;
    HGX_HIP(hipMemGetInfo(&free_b, &total_b));
    if (bytes > free_b / 4) {
        g->q_inline = false;   // no room: the match reads target rows through tgt_off
        return;
    }
    int4* t = nullptr;
    HGX_HIP(hipMalloc(&t, bytes));
    k_ts_inline<<<grid_for(g->I, 256, 65536), 256, 0, g->stream>>>(g->I, g->inc_ts_row, g->tgt_off, g->tgt_idx, t);
    HGX_CHECK_LAUNCH();
    HGX_HIP(hipStreamSynchronize(g->stream));
    g->inc_ts_tgt = (int32_t*)t;
}

// Device arrays of one normalised batch (built by a front end) and the per-query plan.
struct Front {
    const QDesc* desc = nullptr;
    const int32_t* anch = nullptr;
    const int32_t* types = nullptr;
    const int32_t* pos = nullptr;
    const int64_t* poff = nullptr;
    const int32_t* pat = nullptr;
    QPlan* plan = nullptr;
    int32_t* nch = nullptr;      // [n + 1]
    int64_t* ncand = nullptr;    // [n + 1]
    int32_t* err = nullptr;      // [2] device-side normalisation errors (packed front end), or null
    double cond_bytes = 0;       // condition bytes read by the match (algorithmic accounting)
    int64_t* blk = nullptr;      // single-pass pipeline: [3 per block of 256 queries] candidates, bad, unsupported
    int64_t* lpre = nullptr;     //   [n] candidates of the queries before q in its block of 256
    u64* ctr = nullptr;          //   the match's counter shards, zeroed by the front kernel
};

// Buffers taken from the graph pool for one call, released on every exit path.
struct Scratch {
    hgx_graph* g;
    std::vector<std::pair<void*, size_t>> t;
    void* take(size_t bytes) {
        void* p = g->alloc(bytes);
        t.push_back({p, bytes});
        return p;
    }
    ~Scratch() { for (auto& x : t) g->release(x.first, x.second); }
};

// Timing events of one batch, taken from the graph's pool and given back (an event create + destroy
// per batch costs more host time than the batch's match kernel).  The caller holds g->mu.
struct Events {
    hgx_graph* g = nullptr;
    hipEvent_t e[4] = {nullptr, nullptr, nullptr, nullptr};
    bool on = false;
    void init(hgx_graph* gg) {
        g = gg;
        on = gg->timing;
        if (!on) return;
        for (int i = 0; i < 4; ++i) {
            if (!g->ev_pool.empty()) {
                e[i] = g->ev_pool.back();
                g->ev_pool.pop_back();
            } else {
                HGX_HIP(hipEventCreate(&e[i]));
            }
        }
    }
    void rec(int i, hipStream_t s) { if (on) HGX_HIP(hipEventRecord(e[i], s)); }
    ~Events() {
        for (int i = 0; i < 4; ++i)
            if (e[i]) g->ev_pool.push_back(e[i]);
    }
};

template <class T>
size_t bytes_of(const std::vector<T>& v) { return sizeof(T) * std::max<size_t>(v.size(), 1); }

// Pinned staging layout of one upload: put() reserves 16-byte aligned ranges.
struct Upload {
    size_t off = 0;
    size_t take(size_t bytes) {
        const size_t o = off;
        off = (off + std::max<size_t>(bytes, 1) + 15) & ~(size_t)15;
        return o;
    }
};

// Front end for host-normalised batches (legacy / ext entry points).
void front_host(hgx_graph* g, int32_t n, const NormBatch& nb, Scratch& sc, Events& ev, Front& f) {
    hipStream_t s = g->stream;
    Upload u;
    const size_t o_desc = u.take(sizeof(QDesc) * n), o_anch = u.take(bytes_of(nb.anchors)),
                 o_types = u.take(bytes_of(nb.types)), o_pos = u.take(bytes_of(nb.pos)),
                 o_poff = u.take(bytes_of(nb.p_off)), o_pat = u.take(bytes_of(nb.pattern)),
                 o_nop = u.take(bytes_of(nb.nop));
    char* h = (char*)g->pinned_buf(u.off);
    auto put = [&](size_t o, const auto& v) {
        if (!v.empty()) std::memcpy(h + o, v.data(), sizeof(v[0]) * v.size());
    };
    put(o_desc, nb.desc);
    put(o_anch, nb.anchors);
    put(o_types, nb.types);
    put(o_pos, nb.pos);
    put(o_poff, nb.p_off);
    put(o_pat, nb.pattern);
    put(o_nop, nb.nop);
    char* d = (char*)sc.take(u.off);
    f.plan = (QPlan*)sc.take(sizeof(QPlan) * n);
    f.nch = (int32_t*)sc.take(sizeof(int32_t) * (n + 1));
    f.ncand = (int64_t*)sc.take(sizeof(int64_t) * (n + 1));
    ev.rec(0, s);
    HGX_HIP(hipMemcpyAsync(d, h, u.off, hipMemcpyHostToDevice, s));
    f.desc = (const QDesc*)(d + o_desc);
    f.anch = (const int32_t*)(d + o_anch);
    f.types = (const int32_t*)(d + o_types);
    f.pos = (const int32_t*)(d + o_pos);
    f.poff = (const int64_t*)(d + o_poff);
    f.pat = (const int32_t*)(d + o_pat);
    f.cond_bytes = 20.0 * nb.anchors.size() + 4.0 * nb.types.size() + 4.0 * nb.pos.size() +
                   4.0 * nb.pattern.size() + (double)sizeof(QDesc) * n;
    // the single-pass pipeline: the plan + per-block candidate totals
    f.blk = (int64_t*)sc.take(sizeof(int64_t) * 3 * (size_t)ceil_div(n, kSpBlock));
    f.lpre = (int64_t*)sc.take(sizeof(int64_t) * (size_t)std::max(n, 1));
    f.ctr = (u64*)sc.take(sizeof(u64) * kQShards * kQStride);
    hgx_q_plan_sp<<<(unsigned)ceil_div(n, kSpBlock), kSpBlock, 0, s>>>(
        n, f.desc, f.anch, f.types, (const int32_t*)(d + o_nop), g->inc_off, g->inc_ts_type, f.plan, f.ncand, f.blk,
        f.lpre, f.ctr);
    HGX_CHECK_LAUNCH();
}

// Layout of a packed batch in one staging area (pinned, mapped or device): its columns at 16-byte
// aligned offsets, plus the 8-byte error slot of the legacy front kernel.
struct PackedLayout {
    size_t o_type = 0, o_ioff = 0, o_inc = 0, o_ho = 0, o_poff = 0, o_pat = 0, o_err = 0, bytes = 0;
    int64_t n_inc = 0, n_pat = 0;
};

PackedLayout packed_layout(int32_t n, const int32_t* inc, const int64_t* inc_off, const int32_t* pat,
                           const int64_t* pat_off, const char* who) {
    PackedLayout l;
    l.n_inc = inc_off[n] - inc_off[0];
    l.n_pat = pat_off[n] - pat_off[0];
    if (inc_off[0] != 0 || pat_off[0] != 0 || l.n_inc < 0 || l.n_pat < 0 || (l.n_inc > 0 && !inc) || (l.n_pat > 0 && !pat))
        fail(HGX_E_INVALID, std::string(who) + ": bad offsets");
    // every query's slices inside the columns: the device front end copies pat[pat_off[q] ..
    // pat_off[q+1]) and the anchors into fixed slots sized from these offsets
    for (int32_t q = 0; q < n; ++q)
        if (inc_off[q + 1] < inc_off[q] || pat_off[q + 1] < pat_off[q])
            fail(HGX_E_INVALID, std::string(who) + ": offsets decrease at query " + std::to_string(q));
    Upload u;
    l.o_type = u.take(4 * (size_t)n);
    l.o_ioff = u.take(8 * (size_t)(n + 1));
    l.o_inc = u.take(4 * (size_t)l.n_inc);
    l.o_ho = u.take(4 * (size_t)n);
    l.o_poff = u.take(8 * (size_t)(n + 1));
    l.o_pat = u.take(4 * (size_t)l.n_pat);
    l.o_err = u.take(8);
    l.bytes = u.off;
    return l;
}

void packed_fill(char* h, const PackedLayout& l, int32_t n, const int32_t* type, const int64_t* inc_off,
                 const int32_t* inc, const int32_t* has_ordered, const int64_t* pat_off, const int32_t* pat) {
    const int32_t none[2] = {INT32_MAX, INT32_MAX};   // smallest bad query index, none yet
    std::memcpy(h + l.o_err, none, 8);
    std::memcpy(h + l.o_type, type, 4 * (size_t)n);
    std::memcpy(h + l.o_ioff, inc_off, 8 * (size_t)(n + 1));
    if (l.n_inc) std::memcpy(h + l.o_inc, inc, 4 * (size_t)l.n_inc);
    std::memcpy(h + l.o_ho, has_ordered, 4 * (size_t)n);
    std::memcpy(h + l.o_poff, pat_off, 8 * (size_t)(n + 1));
    if (l.n_pat) std::memcpy(h + l.o_pat, pat, 4 * (size_t)l.n_pat);
}

// Normalise + plan a packed batch the device can read at d (the mapped staging area, a device copy of
// the pinned staging, or a query set resident in HBM).  sp: the single-pass front kernel.
void front_device(hgx_graph* g, int32_t n, const PackedLayout& l, const char* d, Scratch& sc, Events& ev,
                  Front& f) {
    hipStream_t s = g->stream;
    QDesc* desc = (QDesc*)sc.take(sizeof(QDesc) * n);
    int32_t* anch = (int32_t*)sc.take(4 * (size_t)std::max<int64_t>(l.n_inc + l.n_pat, 1));
    int32_t* nop = (int32_t*)sc.take(4 * (size_t)n);
    f.plan = (QPlan*)sc.take(sizeof(QPlan) * n);
    f.nch = (int32_t*)sc.take(sizeof(int32_t) * (n + 1));
    f.ncand = (int64_t*)sc.take(sizeof(int64_t) * (n + 1));
    f.err = (int32_t*)(d + l.o_err);
    f.cond_bytes = 20.0 * (double)(l.n_inc + l.n_pat) + 4.0 * n + 4.0 * (double)l.n_pat + (double)sizeof(QDesc) * n;
    {   // normalise + plan straight from d; device copies of the match's columns
        int32_t* dty = (int32_t*)sc.take(4 * (size_t)n);
        int64_t* dpo = (int64_t*)sc.take(8 * (size_t)(n + 1));
        int32_t* dpa = (int32_t*)sc.take(4 * (size_t)std::max<int64_t>(l.n_pat, 1));
        f.blk = (int64_t*)sc.take(sizeof(int64_t) * 3 * (size_t)ceil_div(n, kSpBlock));
        f.lpre = (int64_t*)sc.take(sizeof(int64_t) * (size_t)std::max(n, 1));
        f.ctr = (u64*)sc.take(sizeof(u64) * kQShards * kQStride);
        hgx_q_norm_sp<<<(unsigned)ceil_div(n, kSpBlock), kSpBlock, 0, s>>>(
            n, g->A, (const int32_t*)(d + l.o_type), (const int64_t*)(d + l.o_ioff), (const int32_t*)(d + l.o_inc),
            (const int32_t*)(d + l.o_ho), (const int64_t*)(d + l.o_poff), (const int32_t*)(d + l.o_pat), g->inc_off,
            g->inc_ts_type, desc, anch, nop, f.plan, dty, dpo, dpa, f.ncand, f.blk, f.lpre, f.ctr);
        HGX_CHECK_LAUNCH();
        f.desc = desc;
        f.anch = anch;
        f.types = dty;
        f.pos = nullptr;
        f.poff = dpo;
        f.pat = dpa;
        return;
    }
}

// Front end for the packed batch: the raw arrays go into one staging area (the single-pass kernel reads
// it in place through the mapping; otherwise one copy up) and are normalised + planned on the device.
void front_packed(hgx_graph* g, int32_t n, const int32_t* type, const int64_t* inc_off, const int32_t* inc,
                  const int32_t* has_ordered, const int64_t* pat_off, const int32_t* pat, Scratch& sc, Events& ev,
                  Front& f) {
    hipStream_t s = g->stream;
    const PackedLayout l = packed_layout(n, inc, inc_off, pat, pat_off, "hgx_pattern_batch_packed");
    char* h = (char*)g->zc_in_buf(l.bytes);   // the front kernel reads the staging area in place
    packed_fill(h, l, n, type, inc_off, inc, has_ordered, pat_off, pat);
    ev.rec(0, s);
    front_device(g, n, l, (char*)g->zc_in_dev, sc, ev, f);
}

// Single-pass back end (HGX_OPT_QUERY_FLAT = 2, default): scan + match + placement + offsets after the
// front kernel, results written by the kernels into mapped host memory, one synchronisation.
void back_end_sp(hgx_graph* g, int32_t n, Front& f, Scratch& sc, Events& ev, hgx_query_result* r, bool prof,
                 double t0) {
    (void)sc;
    hipStream_t s = g->stream;
    if (g->q_cap_chunks < (int64_t)n / 4 + 64) g->q_cap_chunks = (int64_t)n / 4 + 64;
    if (g->q_cap_cand < 16 * (int64_t)n + 4096) g->q_cap_cand = 16 * (int64_t)n + 4096;
    const int nblk = (int)ceil_div(n, kSpBlock);
    for (int attempt = 0;; ++attempt) {
        const int64_t capC = std::max<int64_t>(g->q_cap_chunks, ceil_div(g->q_cap_cand, kFlatChunk)), capK = g->q_cap_cand;
        if (capC > (int64_t)INT32_MAX - 1) fail(HGX_E_UNSUPPORTED, "hgx_pattern_batch: candidate volume overflow");
        Scratch w{g, {}};
        int64_t* coff = (int64_t*)w.take(sizeof(int64_t) * (n + 1));
        int32_t* chq = (int32_t*)w.take(sizeof(int32_t) * capC);
        int32_t* nch = (int32_t*)w.take(sizeof(int32_t) * 4);
        int32_t* slots = (int32_t*)w.take(sizeof(int32_t) * capC * kFlatChunk);
        int64_t* cnt = (int64_t*)w.take(sizeof(int64_t) * (capC + 1));
        u64* hmask = (u64*)w.take(sizeof(u64) * (capC + 1));
        int64_t* outoff = (int64_t*)w.take(sizeof(int64_t) * (capC + 1));
        u64* ctr = (u64*)w.take(sizeof(u64) * kQShards * kQStride);
        // result area in mapped host memory, written by the kernels (no copy back):
        // stat[8] | ctr[4] | q_off[n+1] | ids[capK]
        const size_t m_stat = 0, m_ctr = 64, m_qoff = 128;
        const size_t m_ids = m_qoff + ((8 * (size_t)(n + 1) + 15) & ~(size_t)15);
        char* hm = (char*)g->mapped_buf(m_ids + 4 * (size_t)capK);
        void* hmd = nullptr;
        HGX_HIP(hipHostGetDevicePointer(&hmd, hm, 0));
        char* rd = (char*)hmd;
        int64_t* stat_d = (int64_t*)(rd + m_stat);
        u64* ctr_d = (u64*)(rd + m_ctr);
        int64_t* qoff_d = (int64_t*)(rd + m_qoff);
        int32_t* ids_d = (int32_t*)(rd + m_ids);
        const int64_t nbp = std::max<int64_t>(1, ceil_div(capC, kPlaceChunks));
        // derived flat index: no scan launch between the front kernel and the match (its counter shards
        // were zeroed by the front kernel; a re-run after a workspace overflow zeroes them here)
        const bool derived = f.lpre && nblk <= kDerivedBlocks && nbp <= kPlaceDirectBlocks;
        const int4* tt = g->q_inline ? (const int4*)g->inc_ts_tgt : nullptr;
        // without timing events the host waits on a completion flag the placement writes into the result
        // area (stat[7]) instead of asking the stream (each hipStreamQuery costs a few microseconds)
        static const bool stream_wait = ab_env("HGX_Q_STREAM_WAIT") != nullptr;   // A/B
        const bool flag = derived && !ev.on && !stream_wait;
        u64 flag_seq = 0;
        if (flag) {
            if (!g->q_ticket) {
                HGX_HIP(hipMalloc(&g->q_ticket, sizeof(u64)));
                HGX_HIP(hipMemsetAsync(g->q_ticket, 0, sizeof(u64), s));
            }
            flag_seq = ++g->q_seq;
            __atomic_store_n((u64*)(hm + m_stat) + 7, (u64)0, __ATOMIC_RELEASE);
        }
        if (derived) {
            ctr = f.ctr;
            if (attempt > 0) HGX_HIP(hipMemsetAsync(ctr, 0, sizeof(u64) * kQShards * kQStride, s));
            ev.rec(1, s);
            hgx_pattern_match_flat<true><<<grid_for(capC * 64, 256, 4096), 256, 0, s>>>(
                nullptr, n, nullptr, nullptr, f.plan, f.desc, f.anch, f.types, f.pos, f.poff, f.pat, g->inc_row,
                g->inc_type, g->inc_ts_row, g->tgt_off, g->tgt_idx, tt, slots, cnt, hmask, ctr, f.blk, f.lpre, nblk, capC,
                capK);
            HGX_CHECK_LAUNCH();
            ev.rec(2, s);
            hgx_q_place<true><<<(unsigned)nbp, 256, 0, s>>>(nullptr, cnt, slots, g->link_atom, outoff, ids_d, stat_d, ctr,
                                                            ctr_d, n, nullptr, nullptr, hmask, qoff_d, nullptr, f.blk,
                                                            f.lpre, nblk, capC, capK, flag ? g->q_ticket : nullptr,
                                                            flag_seq);
            HGX_CHECK_LAUNCH();
        }
        if (!derived) {
            hgx_q_scan_sp<<<nblk, kSpBlock, 0, s>>>(n, f.ncand, f.blk, coff, chq, nch, capC, capK, stat_d, ctr);
            HGX_CHECK_LAUNCH();
            ev.rec(1, s);
            hgx_pattern_match_flat<false><<<grid_for(capC * 64, 256, 4096), 256, 0, s>>>(
                nch, n, chq, coff, f.plan, f.desc, f.anch, f.types, f.pos, f.poff, f.pat, g->inc_row, g->inc_type,
                g->inc_ts_row, g->tgt_off, g->tgt_idx, tt, slots, cnt, hmask, ctr, nullptr, nullptr, 0, 0, 0);
            HGX_CHECK_LAUNCH();
            ev.rec(2, s);
            int64_t* bpre = nullptr;
            if (nbp > kPlaceDirectBlocks) {
                bpre = (int64_t*)w.take(sizeof(int64_t) * (nbp + 1));
                hgx_q_place_bsum<<<grid_for(nbp, 256, 4096), 256, 0, s>>>(nch, cnt, nbp, bpre);
                HGX_CHECK_LAUNCH();
                hgx_q_place_bscan<<<1, 1024, 0, s>>>(nbp, bpre);
                HGX_CHECK_LAUNCH();
            }
            hgx_q_place<false><<<(unsigned)nbp, 256, 0, s>>>(nch, cnt, slots, g->link_atom, outoff, ids_d, stat_d, ctr,
                                                             ctr_d, n, chq, coff, hmask, qoff_d, bpre, nullptr, nullptr,
                                                             0, 0, 0, nullptr, 0);
            HGX_CHECK_LAUNCH();
        }
        ev.rec(3, s);
        if (flag) {
            const u64* fl = (const u64*)(hm + m_stat) + 7;
            for (unsigned spin = 0; __atomic_load_n(fl, __ATOMIC_ACQUIRE) != flag_seq; ++spin) {
                if ((spin & 1023u) != 1023u) continue;   // the stream is asked every 1024 polls
                const hipError_t e = hipStreamQuery(s);
                if (e == hipErrorNotReady) continue;
                if (e != hipSuccess) HGX_HIP(e);
                if (__atomic_load_n(fl, __ATOMIC_ACQUIRE) != flag_seq)
                    fail(HGX_E_DEVICE, "hgx_pattern_batch: the completion flag never arrived");
            }
        } else {
            spin_sync(s);
        }
        const int64_t* stat = (const int64_t*)(hm + m_stat);
        const u64* ctr_h = (const u64*)(hm + m_ctr);
        const int64_t* qoff_h = (const int64_t*)(hm + m_qoff);
        const int32_t* ids_h = (const int32_t*)(hm + m_ids);
        if (stat[4] < n) fail(HGX_E_INVALID, "hgx_pattern_batch: bad query " + std::to_string(stat[4]));
        if (stat[5] < n)
            fail(HGX_E_UNSUPPORTED, "hgx_pattern_batch: query " + std::to_string(stat[5]) +
                                        " is not accelerated (no incidence anchor or condition limits)");
        if (stat[2]) {   // workspace too small: grow to the reported totals and match again
            if (attempt > 0) fail(HGX_E_DEVICE, "hgx_pattern_batch: workspace sizing failed");
            g->q_cap_chunks = std::max<int64_t>(capC, stat[0] + stat[0] / 4 + 64);
            g->q_cap_cand = std::max<int64_t>(capK, stat[1] + stat[1] / 4 + 4096);
            continue;
        }
        const int64_t total = stat[3];
        r->n_hits = total;
        if (r->ext_off) {   // caller buffers: no result vectors
            std::memcpy(r->ext_off, qoff_h, sizeof(int64_t) * (n + 1));
            if (total <= r->ext_cap && total > 0) std::memcpy(r->ext_ids, ids_h, sizeof(int32_t) * total);
        } else {
            std::memcpy(r->offsets.data(), qoff_h, sizeof(int64_t) * (n + 1));
            r->ids.assign(ids_h, ids_h + total);
        }
        if (prof)
            std::fprintf(stderr, "[hgx query] single-pass n=%d host+device %.3f ms (chunks %lld, candidates %lld, hits %lld)\n",
                         n, now_ms() - t0, (long long)stat[0], (long long)stat[1], (long long)total);
        if (ev.on) {
            float a = 0, b = 0;
            HGX_HIP(hipEventElapsedTime(&a, ev.e[0], ev.e[3]));
            HGX_HIP(hipEventElapsedTime(&b, ev.e[1], ev.e[2]));
            r->ms_total = a;
            r->ms_match = b;
        }
        // algorithmic bytes of hgx_pattern_match_flat (as back_end_flat)
        r->bytes_match = (4.0 + 8.0 * (kFlatChunk + 1) + 16.0) * (double)stat[0] +
                         (double)(sizeof(QPlan) + sizeof(QDesc)) * n + 4.0 * (double)ctr_h[qCand] +
                         4.0 * (double)ctr_h[qTyped] + 32.0 * (double)ctr_h[qInline] +
                         16.0 * ((double)ctr_h[qTyped] - (double)ctr_h[qInline]) + 4.0 * (double)ctr_h[qArity] +
                         4.0 * (double)ctr_h[qHits] + f.cond_bytes;
        return;
    }
}

// The back end of every batch: the single-pass pipeline (round 5: the per-query-chunk (HGX_OPT_QUERY_FLAT 0)
// and separate-scan flat (1) back ends are gone; both measured slower).
void back_end(hgx_graph* g, int32_t n, Front& f, Scratch& sc, Events& ev, hgx_query_result* r, bool prof,
              double t0) {
    back_end_sp(g, n, f, sc, ev, r, prof, t0);
}



template <class FrontFn>
int run_batch_with(hgx_graph* g, int32_t n, hgx_query_result** out, FrontFn front, hgx_query_result* into = nullptr) {
    HGX_API_BEGIN
    const bool prof = trace_env("HGX_QUERY_PROFILE");
    const double t0 = now_ms();
    if (g->shard) fail(HGX_E_UNSUPPORTED, "hgx_pattern_batch: not available on a partition shard");
    std::unique_ptr<hgx_query_result> own;
    hgx_query_result* r = into;
    if (!r) {
        own.reset(new hgx_query_result());
        r = own.get();
    }
    r->n = n;
    // the single-pass back end writes caller buffers directly; the other back ends fill the vectors
    if (!r->ext_off) r->offsets.assign(n + 1, 0);
    if (n > 0) {
        std::lock_guard<std::mutex> lk(g->mu);
        HGX_HIP(hipSetDevice(g->device));
        ensure_type_grouped(g);
        ensure_ts_inline(g);
        Scratch sc{g, {}};
        Events ev;
        ev.init(g);
        Front f;
        front(sc, ev, f);
        back_end(g, n, f, sc, ev, r, prof, t0);
    }
    if (out) *out = own.release();
    HGX_API_END
}

int run_batch(hgx_graph* g, int32_t n, NormBatch& nb, hgx_query_result** out) {
    return run_batch_with(g, n, out, [&](Scratch& sc, Events& ev, Front& f) { front_host(g, n, nb, sc, ev, f); });
}

int run_batch_packed_direct(hgx_graph* g, int32_t n, const int32_t* type, const int64_t* inc_off, const int32_t* inc,
                            const int32_t* has_ordered, const int64_t* pat_off, const int32_t* pat,
                            hgx_query_result** out);

// One caller batch of the combiner run on its own: the result, or the status and this thread's
// error message handed to the waiting caller.
void serve_one(hgx_graph* g, PackedReq* q) {
    hgx_query_result* r = nullptr;
    q->rc = run_batch_packed_direct(g, q->n, q->type, q->inc_off, q->inc, q->has_ordered, q->pat_off, q->pat, &r);
    if (q->rc == HGX_OK) q->r = r;
    else q->err = hgx_last_error();
}

// The offsets of a caller batch are what the merge relies on (the device checks everything else).
bool mergeable(const PackedReq* q) {
    if (q->n <= 0 || q->inc_off[0] != 0 || q->pat_off[0] != 0) return false;
    const int64_t ni = q->inc_off[q->n], np = q->pat_off[q->n];
    return ni >= 0 && np >= 0 && (ni == 0 || q->inc) && (np == 0 || q->pat);
}

// Serve a group of queued caller batches: those that can merge run as ONE device batch (their
// arrays concatenated, offsets rebased) whose result is split back per caller; a merged run that
// reports a bad or unsupported query is re-run caller by caller, so every caller gets exactly the
// result or error of a separate call.  Never throws (statuses go to the requests).
void serve_group(hgx_graph* g, const std::vector<PackedReq*>& grp) {
    std::vector<PackedReq*> m;
    for (PackedReq* q : grp) {
        if (grp.size() > 1 && mergeable(q)) m.push_back(q);
        else serve_one(g, q);
    }
    if (m.empty()) return;
    if (m.size() == 1) {
        serve_one(g, m[0]);
        return;
    }
    int rc = HGX_OK;
    std::string err;
    try {
        int64_t N = 0, NI = 0, NP = 0;
        for (PackedReq* q : m) {
            N += q->n;
            NI += q->inc_off[q->n];
            NP += q->pat_off[q->n];
        }
        std::vector<int32_t> type((size_t)N), ho((size_t)N), inc((size_t)std::max<int64_t>(NI, 1)),
            pat((size_t)std::max<int64_t>(NP, 1));
        std::vector<int64_t> io((size_t)N + 1), po((size_t)N + 1);
        int64_t b = 0, bi = 0, bp = 0;
        for (PackedReq* q : m) {
            std::memcpy(&type[b], q->type, 4 * (size_t)q->n);
            std::memcpy(&ho[b], q->has_ordered, 4 * (size_t)q->n);
            for (int32_t k = 0; k < q->n; ++k) {
                io[b + k] = bi + q->inc_off[k];
                po[b + k] = bp + q->pat_off[k];
            }
            if (q->inc_off[q->n]) std::memcpy(&inc[bi], q->inc, 4 * (size_t)q->inc_off[q->n]);
            if (q->pat_off[q->n]) std::memcpy(&pat[bp], q->pat, 4 * (size_t)q->pat_off[q->n]);
            b += q->n;
            bi += q->inc_off[q->n];
            bp += q->pat_off[q->n];
        }
        io[N] = bi;
        po[N] = bp;
        hgx_query_result* all = nullptr;
        rc = run_batch_packed_direct(g, (int32_t)N, type.data(), io.data(), inc.data(), ho.data(), po.data(), pat.data(),
                                     &all);
        if (rc == HGX_OK) {
            std::unique_ptr<hgx_query_result> keep(all);
            int64_t q0 = 0;
            for (PackedReq* q : m) {
                std::unique_ptr<hgx_query_result> r(new hgx_query_result());
                r->n = q->n;
                r->offsets.resize((size_t)q->n + 1);
                const int64_t base = all->offsets[(size_t)q0];
                for (int32_t k = 0; k <= q->n; ++k) r->offsets[(size_t)k] = all->offsets[(size_t)(q0 + k)] - base;
                r->ids.assign(all->ids.begin() + base, all->ids.begin() + all->offsets[(size_t)(q0 + q->n)]);
                r->ms_total = all->ms_total;
                r->ms_match = all->ms_match;
                r->bytes_match = all->bytes_match;
                q->r = r.release();
                q->rc = HGX_OK;
                q0 += q->n;
            }
            return;
        }
        err = hgx_last_error();
    } catch (const std::bad_alloc&) {
        rc = HGX_E_NOMEM;
        err = "host allocation failed";
    } catch (const std::exception& e) {
        rc = HGX_E_DEVICE;
        err = e.what();
    }
    if (rc == HGX_E_INVALID || rc == HGX_E_UNSUPPORTED) {   // a query-specific status: whose query?
        for (PackedReq* q : m) serve_one(g, q);
        return;
    }
    for (PackedReq* q : m) {
        q->rc = rc;
        q->err = err;
    }
}

int run_batch_packed(hgx_graph* g, int32_t n, const int32_t* type, const int64_t* inc_off, const int32_t* inc,
                     const int32_t* has_ordered, const int64_t* pat_off, const int32_t* pat, hgx_query_result** out) {
    if (n <= 0 || !g->q_coalesce || g->shard)
        return run_batch_packed_direct(g, n, type, inc_off, inc, has_ordered, pat_off, pat, out);
    PackedReq me;
    me.n = n;
    me.type = type;
    me.inc_off = inc_off;
    me.inc = inc;
    me.has_ordered = has_ordered;
    me.pat_off = pat_off;
    me.pat = pat;
    QueryCombiner& c = g->qcomb;
    std::unique_lock<std::mutex> lk(c.mu);
    c.pending.push_back(&me);
    // an exception below (allocation) must not leave this stack request queued for another caller
    struct Unqueue {
        QueryCombiner& c;
        PackedReq* me;
        std::unique_lock<std::mutex>& lk;
        ~Unqueue() {
            if (!lk.owns_lock()) lk.lock();
            auto it = std::find(c.pending.begin(), c.pending.end(), me);
            if (it != c.pending.end()) c.pending.erase(it);
        }
    } unqueue{c, &me, lk};
    while (!me.done) {
        if (c.busy) {
            c.cv.wait(lk);
            continue;
        }
        // run the queue's head group: FIFO, up to the query cap (a batch above the cap runs alone)
        std::vector<PackedReq*> grp;
        grp.reserve(c.pending.size());   // the only allocation: before the combiner is marked busy
        c.busy = true;
        // whatever happens while the group runs, its members end done (an unserved one with an error),
        // the combiner is released and the waiting callers are woken
        struct Release {
            QueryCombiner& c;
            std::vector<PackedReq*>& grp;
            std::unique_lock<std::mutex>& lk;
            bool served = false;
            ~Release() {
                if (!lk.owns_lock()) lk.lock();
                for (PackedReq* q : grp) {
                    if (!served && q->rc == HGX_OK && !q->r) {
                        q->rc = HGX_E_DEVICE;
                        q->err = "hgx_pattern_batch_packed: the coalesced batch failed";
                    }
                    q->done = true;
                }
                c.busy = false;
                c.cv.notify_all();
            }
        } release{c, grp, lk};
        int64_t tot = 0;
        while (!c.pending.empty() && (grp.empty() || tot + c.pending.front()->n <= g->q_coalesce_max)) {
            grp.push_back(c.pending.front());
            tot += c.pending.front()->n;
            c.pending.pop_front();
        }
        lk.unlock();
        serve_group(g, grp);
        lk.lock();
        c.batches += 1;
        c.requests += (int64_t)grp.size();
        release.served = true;
    }
    lk.unlock();
    if (me.rc != HGX_OK) {
        set_last_error(me.err);
        return me.rc;
    }
    *out = me.r;
    return HGX_OK;
}

int run_batch_packed_direct(hgx_graph* g, int32_t n, const int32_t* type, const int64_t* inc_off, const int32_t* inc,
                            const int32_t* has_ordered, const int64_t* pat_off, const int32_t* pat,
                            hgx_query_result** out) {
    return run_batch_with(g, n, out, [&](Scratch& sc, Events& ev, Front& f) {
        front_packed(g, n, type, inc_off, inc, has_ordered, pat_off, pat, sc, ev, f);
    });
}

}  // namespace

extern "C" {

int hgx_query_result_count(const hgx_query_result* r, int64_t* n_queries) {
    HGX_API_BEGIN
    if (!r || !n_queries) fail(HGX_E_INVALID, "hgx_query_result_count: bad argument");
    *n_queries = (int64_t)r->offsets.size() - 1;
    HGX_API_END
}

int hgx_query_result_offsets(const hgx_query_result* r, int64_t* offsets) {
    HGX_API_BEGIN
    if (!r || !offsets) fail(HGX_E_INVALID, "hgx_query_result_offsets: bad argument");
    std::memcpy(offsets, r->offsets.data(), sizeof(int64_t) * r->offsets.size());
    HGX_API_END
}

int hgx_query_result_ids(const hgx_query_result* r, int32_t* ids) {
    HGX_API_BEGIN
    if (!r || (!ids && !r->ids.empty())) fail(HGX_E_INVALID, "hgx_query_result_ids: bad argument");
    if (!r->ids.empty()) std::memcpy(ids, r->ids.data(), sizeof(int32_t) * r->ids.size());
    HGX_API_END
}

int hgx_query_result_ms(const hgx_query_result* r, double* ms_total, double* ms_match, double* bytes_match) {
    HGX_API_BEGIN
    if (!r) fail(HGX_E_INVALID, "null result");
    if (ms_total) *ms_total = r->ms_total;
    if (ms_match) *ms_match = r->ms_match;
    if (bytes_match) *bytes_match = r->bytes_match;
    HGX_API_END
}

void hgx_query_result_free(hgx_query_result* r) { delete r; }

int hgx_query_coalesce_stats(hgx_graph* g, int64_t* device_batches, int64_t* caller_batches) {
    HGX_API_BEGIN
    if (!g) fail(HGX_E_INVALID, "null graph");
    std::lock_guard<std::mutex> lk(g->qcomb.mu);
    if (device_batches) *device_batches = g->qcomb.batches;
    if (caller_batches) *caller_batches = g->qcomb.requests;
    HGX_API_END
}

}  // extern "C"

// ---------------------------------------------------------------------------------------------
// Query sets: a packed batch uploaded once and run many times with its arrays resident in HBM (a
// fixed set of compiled queries re-executed by the application's threads, QueryCompilation.java:
// 76-122; the bench's config-3 step with its inputs in HBM).  The run is the packed path's front
// kernel reading the set instead of the pinned staging area, then the same back end.
// ---------------------------------------------------------------------------------------------
extern "C" {

int hgx_query_set_create(hgx_graph* g, int32_t n, const int32_t* type, const int64_t* inc_off, const int32_t* inc,
                         const int32_t* has_ordered, const int64_t* pat_off, const int32_t* pat, hgx_query_set** out) {
    HGX_API_BEGIN
    if (!g || !out || n <= 0 || !type || !inc_off || !pat_off || !has_ordered)
        fail(HGX_E_INVALID, "hgx_query_set_create: bad argument");
    *out = nullptr;
    const PackedLayout l = packed_layout(n, inc, inc_off, pat, pat_off, "hgx_query_set_create");
    std::vector<char> h(l.bytes);
    packed_fill(h.data(), l, n, type, inc_off, inc, has_ordered, pat_off, pat);
    std::unique_ptr<hgx_query_set> qs(new hgx_query_set());
    qs->device = g->device;
    qs->n = n;
    qs->o_type = l.o_type; qs->o_ioff = l.o_ioff; qs->o_inc = l.o_inc; qs->o_ho = l.o_ho;
    qs->o_poff = l.o_poff; qs->o_pat = l.o_pat; qs->o_err = l.o_err; qs->bytes = l.bytes;
    qs->n_inc = l.n_inc; qs->n_pat = l.n_pat;
    HGX_HIP(hipSetDevice(g->device));
    HGX_HIP(hipMalloc(&qs->dev, l.bytes));
    if (hipMemcpy(qs->dev, h.data(), l.bytes, hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(qs->dev);
        fail(HGX_E_DEVICE, "hgx_query_set_create: upload failed");
    }
    *out = qs.release();
    HGX_API_END
}

int hgx_pattern_batch_set(hgx_graph* g, const hgx_query_set* qs, hgx_query_result** out) {
    HGX_API_BEGIN
    if (!g || !qs || !out) fail(HGX_E_INVALID, "hgx_pattern_batch_set: bad argument");
    if (qs->device != g->device) fail(HGX_E_INVALID, "hgx_pattern_batch_set: the set lives on another device");
    *out = nullptr;
    PackedLayout l;
    l.o_type = qs->o_type; l.o_ioff = qs->o_ioff; l.o_inc = qs->o_inc; l.o_ho = qs->o_ho;
    l.o_poff = qs->o_poff; l.o_pat = qs->o_pat; l.o_err = qs->o_err; l.bytes = qs->bytes;
    l.n_inc = qs->n_inc; l.n_pat = qs->n_pat;
    return run_batch_with(g, qs->n, out, [&](Scratch& sc, Events& ev, Front& f) {
        ev.rec(0, g->stream);
        front_device(g, qs->n, l, qs->dev, sc, ev, f);
    });
    HGX_API_END
}

int hgx_pattern_batch_set_into(hgx_graph* g, const hgx_query_set* qs, int64_t* offsets, int32_t* ids, int64_t ids_cap,
                                int64_t* n_ids, double* timing) {
    HGX_API_BEGIN
    if (!g || !qs || !offsets || !n_ids || ids_cap < 0 || (ids_cap > 0 && !ids))
        fail(HGX_E_INVALID, "hgx_pattern_batch_set_into: bad argument");
    if (qs->device != g->device) fail(HGX_E_INVALID, "hgx_pattern_batch_set_into: the set lives on another device");
    if (qs->n == 0) {
        offsets[0] = 0;
        *n_ids = 0;
        if (timing) timing[0] = timing[1] = timing[2] = 0.0;
        return HGX_OK;
    }
    PackedLayout l;
    l.o_type = qs->o_type; l.o_ioff = qs->o_ioff; l.o_inc = qs->o_inc; l.o_ho = qs->o_ho;
    l.o_poff = qs->o_poff; l.o_pat = qs->o_pat; l.o_err = qs->o_err; l.bytes = qs->bytes;
    l.n_inc = qs->n_inc; l.n_pat = qs->n_pat;
    hgx_query_result r;
    r.ext_off = offsets;
    r.ext_ids = ids;
    r.ext_cap = ids_cap;
    const int rc = run_batch_with(
        g, qs->n, nullptr,
        [&](Scratch& sc, Events& ev, Front& f) {
            ev.rec(0, g->stream);
            front_device(g, qs->n, l, qs->dev, sc, ev, f);
        },
        &r);
    if (rc != HGX_OK) return rc;
    *n_ids = r.n_hits;
    if (timing) {
        timing[0] = r.ms_total;
        timing[1] = r.ms_match;
        timing[2] = r.bytes_match;
    }
    HGX_API_END
}

int hgx_query_set_info(const hgx_query_set* qs, int32_t* n_queries) {
    HGX_API_BEGIN
    if (!qs || !n_queries) fail(HGX_E_INVALID, "hgx_query_set_info: null argument");
    *n_queries = qs->n;
    HGX_API_END
}

void hgx_query_set_free(hgx_query_set* qs) {
    if (!qs) return;
    (void)hipSetDevice(qs->device);
    if (qs->dev) (void)hipFree(qs->dev);
    delete qs;
}

}  // extern "C"
