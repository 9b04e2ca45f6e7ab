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
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "hgx_internal.h"

namespace hgx {

typedef unsigned long long u64;

constexpr int kQChunk = 1024;       // candidates per wave-chunk (16 per lane)
constexpr int kMaxAnchors = 32;
constexpr int kMaxPattern = 64;     // targets of one OrderedLinkCondition
constexpr int kMaxPatterns = 16;    // OrderedLinkConditions in one And
constexpr int kMaxPositioned = 16;  // PositionedIncidentConditions in one And
constexpr int kMaxTypes = 1 << 16;  // types of one Or (TypePlusCondition)

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

enum QCtr { qCand = 0, qTyped, qArity, qHits, qNum = 4 };

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

// Keys of the type-grouped incidence: (atom << 32 | type), value = link row; a stable radix sort
// keeps the rows of one (atom, type) ascending.
__global__ void __launch_bounds__(256) k_ts_keys(int64_t A, const int64_t* __restrict__ inc_off,
                                                 const int32_t* __restrict__ inc_type, u64* __restrict__ keys) {
    const int lane = threadIdx.x & 63;   // a wave per atom: hub rows are written 64 entries at a time
    const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    const int64_t nwave = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t a = wave; a < A; a += nwave)
        for (int64_t i = inc_off[a] + lane; i < inc_off[a + 1]; i += 64) keys[i] = ((u64)a << 32) | (uint32_t)inc_type[i];
}

__global__ void __launch_bounds__(256) k_low32(int64_t n, const u64* __restrict__ keys, int32_t* __restrict__ out) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = (int32_t)(uint32_t)keys[i];
}

__device__ __forceinline__ int64_t lower_bound_i32(const int32_t* __restrict__ a, int64_t b, int64_t e, int32_t v) {
    while (b < e) {
        const int64_t m = (b + e) >> 1;
        if (a[m] < v) b = m + 1; else e = m;
    }
    return b;
}

// Plan per query (AndToQuery sorts the ORA inputs by size, :164-180): the anchor whose candidate
// range is smallest drives the scan.  With exactly one type the candidate range of an anchor is
// its type-T slice of the type-grouped incidence (the type index intersected for free); otherwise
// its whole incidence row with the streamed type filter.  pad = 1 marks a type-grouped plan.
__global__ void __launch_bounds__(256) hgx_q_plan(int32_t n, const QDesc* __restrict__ desc,
                                                  const int32_t* __restrict__ anchors, const int32_t* __restrict__ types,
                                                  const int32_t* __restrict__ nop, const int64_t* __restrict__ inc_off,
                                                  const int32_t* __restrict__ ts_type, QPlan* __restrict__ plan,
                                                  int32_t* __restrict__ nchunks) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n) return;
    const QDesc d = desc[q];
    QPlan p{0, 0, 0, 0};
    if (!nop[q]) {
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
    }
    plan[q] = p;
    nchunks[q] = (int32_t)((p.n + kQChunk - 1) / kQChunk);
}

__global__ void hgx_q_chunk_map(int32_t n, const int32_t* __restrict__ chunk_off, int32_t* __restrict__ chunk_q) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n) return;
    for (int32_t c = chunk_off[q]; c < chunk_off[q + 1]; ++c) chunk_q[c] = q;
}

// A wave per chunk of kQChunk candidates of one query (grid-stride over chunks; the counters are
// summed in registers and added once per wave into sharded replicas).
//   stage 1: every lane streams kPerLane consecutive entries of the type column (16-byte loads) and
//            keeps a bit per type-passing candidate;
//   stage 2: the passing candidates go to an LDS list in ascending order (wave prefix sum);
//   stage 3: the list is processed 64 at a time, one candidate per lane: link row, target offsets,
//            target row, anchor / positioned / ordered / arity checks; hits are compacted in order.
// The type filter passes ~1/T of the candidates, so stage 3 runs on full waves instead of lanes
// idling behind failed type checks.  Hits of a chunk land in its own candidate range of slots.
constexpr int kQShards = 16, kQStride = 16;
constexpr int kPerLane = kQChunk / 64;

__global__ void __launch_bounds__(256) hgx_pattern_match(
    const int32_t* __restrict__ n_chunks_p, const int32_t* __restrict__ chunk_q, const int32_t* __restrict__ chunk_off,
    const int64_t* __restrict__ cand_off, const QPlan* __restrict__ plan, const QDesc* __restrict__ desc,
    const int32_t* __restrict__ anchors, const int32_t* __restrict__ types, const int32_t* __restrict__ pos,
    const int64_t* __restrict__ p_off, const int32_t* __restrict__ pattern, const int32_t* __restrict__ inc_row,
    const int32_t* __restrict__ inc_type, const int32_t* __restrict__ inc_ts_row, const int64_t* __restrict__ tgt_off,
    const int32_t* __restrict__ tgt_idx, int32_t* __restrict__ slots, int64_t* __restrict__ counts,
    u64* __restrict__ ctr) {
    __shared__ int32_t lds[4][kQChunk];
    const int32_t n_chunks = *n_chunks_p;
    int32_t* list = lds[threadIdx.x >> 6];
    const int lane = threadIdx.x & 63;
    const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    const int64_t nwave = ((int64_t)gridDim.x * blockDim.x) >> 6;
    const u64 lt = (1ull << lane) - 1ull;
    u64 n_cand = 0, n_typed = 0, n_ar = 0, n_hits = 0;
    for (int64_t chunk = wave; chunk < n_chunks; chunk += nwave) {
        const int32_t q = chunk_q[chunk];
        const QPlan pl = plan[q];
        const QDesc d = desc[q];
        const int64_t c0 = (int64_t)(chunk - chunk_off[q]) * kQChunk;
        const int64_t nc = pl.n - c0 < kQChunk ? pl.n - c0 : kQChunk;   // candidates of this chunk
        const bool typed = d.t_end > d.t_beg && !pl.pad;   // a type-grouped range is all of type T
        const int32_t* rows = pl.pad ? inc_ts_row : inc_row;
        // stage 1: lane l owns candidates [l*kPerLane, (l+1)*kPerLane) of the chunk
        unsigned passm = 0;
        const int64_t cb = c0 + lane * kPerLane;
        if (!typed) {
            for (int k = 0; k < kPerLane; ++k) passm |= (unsigned)(lane * kPerLane + k < nc) << k;
        } else {
            const int32_t* col = inc_type + pl.beg + cb;
            if (lane * kPerLane + kPerLane <= nc && ((pl.beg + cb) & 3) == 0) {
                int32_t t[kPerLane];
#pragma unroll
                for (int k = 0; k < kPerLane; k += 4) {
                    const int4 v = *reinterpret_cast<const int4*>(col + k);
                    t[k] = v.x; t[k + 1] = v.y; t[k + 2] = v.z; t[k + 3] = v.w;
                }
#pragma unroll
                for (int k = 0; k < kPerLane; ++k) passm |= (unsigned)type_in(t[k], types, d.t_beg, d.t_end) << k;
            } else {
                for (int k = 0; k < kPerLane; ++k)
                    if (lane * kPerLane + k < nc) passm |= (unsigned)type_in(col[k], types, d.t_beg, d.t_end) << k;
            }
        }
        if (typed)   // streamed type column entries (a type-grouped range streams none)
            n_cand += (u64)(lane * kPerLane < nc ? (nc - lane * kPerLane < kPerLane ? nc - lane * kPerLane : kPerLane)
                                                 : 0);
        // stage 2: ascending list of passing candidate indices (relative to the chunk)
        const int cnt = __popc(passm);
        int pre = cnt;
        for (int off = 1; off < 64; off <<= 1) {
            const int y = __shfl_up(pre, off);
            if (lane >= off) pre += y;
        }
        const int total = __shfl(pre, 63);
        pre -= cnt;
        for (unsigned m = passm; m; m &= m - 1u) list[pre++] = lane * kPerLane + __ffs(m) - 1;
        __builtin_amdgcn_wave_barrier();
        // stage 3
        int32_t written = 0;
        int32_t* out = slots + cand_off[q] + c0;
        for (int base = 0; base < total; base += 64) {   // wave-uniform
            const int idx = base + lane;
            bool hit = idx < total;
            int32_t L = -1;
            if (hit) {
                L = rows[pl.beg + c0 + list[idx]];
                ++n_typed;
                const int64_t b = tgt_off[L];
                const int n = (int)(tgt_off[L + 1] - b);
                n_ar += (u64)n;
                const int32_t* row = tgt_idx + b;
                // ArityCondition: layout.length == arity + 2
                if (d.arity >= 0) hit = n == d.arity;
                // IncidentCondition for every other anchor (L in inc(a) <=> a in targets(L))
                for (int64_t j = d.a_beg; j < d.a_end && hit; ++j) {
                    if (j - d.a_beg == pl.amin) continue;
                    const int32_t a = anchors[j];
                    bool found = false;
                    for (int i = 0; i < n; ++i) found |= (row[i] == a);
                    hit = found;
                }
                // PositionedIncidentCondition (its ORA set: inc(target) filtered by the predicate)
                for (int64_t s = d.s_beg; s < d.s_end && hit; ++s)
                    hit = positioned(row, n, pos[4 * s], pos[4 * s + 1], pos[4 * s + 2], pos[4 * s + 3] != 0);
                // OrderedLinkCondition.satisfies: greedy subsequence with hg.anyHandle()
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
            }
            const u64 m = __ballot(hit);
            if (hit) out[written + __popcll(m & lt)] = L;
            written += __popcll(m);
        }
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) counts[chunk] = written;
        n_hits += (u64)written;
    }
    u64* c = ctr + (wave & (kQShards - 1)) * kQStride;
    wave_add_q(c + qCand, n_cand);
    wave_add_q(c + qTyped, n_typed);
    wave_add_q(c + qArity, n_ar);
    if (lane == 0 && n_hits) atomicAdd(c + qHits, n_hits);
}

// Copy each chunk's hits to its output position, mapping link rows to atom ids.
__global__ void __launch_bounds__(256) hgx_q_scatter(const int32_t* __restrict__ n_chunks_p,
                                                     const int32_t* __restrict__ chunk_q,
                                                     const int32_t* __restrict__ chunk_off,
                                                     const int64_t* __restrict__ cand_off,
                                                     const int64_t* __restrict__ counts,
                                                     const int64_t* __restrict__ out_off,
                                                     const int32_t* __restrict__ slots,
                                                     const int32_t* __restrict__ link_atom, int32_t* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t chunk = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    if (chunk >= *n_chunks_p) return;
    const int64_t c = counts[chunk];
    const int64_t o = out_off[chunk];
    const int32_t q = chunk_q[chunk];
    const int32_t* src = slots + cand_off[q] + (int64_t)(chunk - chunk_off[q]) * kQChunk;
    for (int64_t i = lane; i < c; i += 64) out[o + i] = link_atom[src[i]];
}

__global__ void hgx_q_offsets(int32_t n, const int32_t* __restrict__ chunk_off, const int64_t* __restrict__ out_off,
                              int64_t* __restrict__ q_off) {
    int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q <= n) q_off[q] = out_off[chunk_off[q]];
}

}  // namespace hgx

using namespace hgx;

struct hgx_query_result {
    int32_t n = 0;
    std::vector<int64_t> offsets;
    std::vector<int32_t> ids;
    double ms_total = 0, ms_match = 0, bytes_match = 0;
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
    NormBatch nb;
    std::vector<int64_t> one_off;
    const double t0 = now_ms();
    normalise(g, n,
              [&](int32_t q, QueryIn& in) {
                  if (type[q] < HGX_NO_TYPE) fail(HGX_E_INVALID, "hgx_pattern_batch: bad type");
                  in.n_types = type[q] >= 0 ? 1 : 0;
                  in.types = type + q;
                  in.n_inc = (int32_t)(inc_off[q + 1] - inc_off[q]);
                  in.inc = inc ? inc + inc_off[q] : nullptr;
                  one_off.assign({0, pat_off[q + 1] - pat_off[q]});
                  in.n_pat = has_ordered[q] ? 1 : 0;
                  in.pat_off = one_off.data();
                  in.pat = pat ? pat + pat_off[q] : nullptr;
              },
              nb);
    if (std::getenv("HGX_QUERY_PROFILE")) std::fprintf(stderr, "[hgx query] normalise %.3f ms\n", now_ms() - t0);
    return run_batch(g, n, nb, out);
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
void ensure_type_grouped(hgx_graph* g) {
    if (g->inc_ts_row || g->I == 0) return;
    hipStream_t s = g->stream;
    const int64_t I = g->I;
    if (I > (int64_t)INT32_MAX) fail(HGX_E_UNSUPPORTED, "type-grouped incidence: more than 2^31-1 entries");
    u64* keys = (u64*)g->alloc(sizeof(u64) * I);
    u64* keys2 = (u64*)g->alloc(sizeof(u64) * I);
    int32_t* rows2 = (int32_t*)g->alloc(sizeof(int32_t) * I);
    k_ts_keys<<<grid_for(g->A * 64, 256, 16384), 256, 0, s>>>(g->A, g->inc_off, g->inc_type, keys);
    HGX_CHECK_LAUNCH();
    int end_bit = 64;
    {
        int ab = 1;
        while (((int64_t)1 << ab) <= g->A) ab++;
        end_bit = std::min(64, 32 + ab);
    }
    size_t tb = 0;
    HGX_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, keys, keys2, g->inc_row, rows2, (int)I, 0, end_bit, s));
    void* tmp = g->alloc(tb);
    HGX_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, tb, keys, keys2, g->inc_row, rows2, (int)I, 0, end_bit, s));
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

int run_batch(hgx_graph* g, int32_t n, NormBatch& nb, hgx_query_result** out) {
    HGX_API_BEGIN
    const bool prof = std::getenv("HGX_QUERY_PROFILE") != nullptr;
    double t0 = now_ms();
    if (g->shard) fail(HGX_E_UNSUPPORTED, "hgx_pattern_batch: not available on a partition shard");
    const std::vector<int32_t>& anchors = nb.anchors;
    hgx_query_result* r = new hgx_query_result();
    struct Guard {
        hgx_query_result* r;
        ~Guard() { delete r; }
    } guard{r};
    r->n = n;
    r->offsets.assign(n + 1, 0);
    if (n == 0) {
        guard.r = nullptr;
        *out = r;
        return HGX_OK;
    }
    std::lock_guard<std::mutex> lk(g->mu);
    HGX_HIP(hipSetDevice(g->device));
    hipStream_t s = g->stream;
    if (g->inc_off_host.empty()) {   // host copy of the incidence offsets: buffer sizing needs no round trip
        g->inc_off_host.resize((size_t)g->A + 1);
        HGX_HIP(hipMemcpyAsync(g->inc_off_host.data(), g->inc_off, sizeof(int64_t) * (g->A + 1), hipMemcpyDeviceToHost,
                               s));
        HGX_HIP(hipStreamSynchronize(s));
    }
    ensure_type_grouped(g);
    // Upper bounds from the untyped plan (the device plan can only shrink a query's range): the
    // chunk count and each query's slot base in the flat candidate space.
    std::vector<int64_t> cand_off(n + 1, 0);
    const int64_t* io = g->inc_off_host.data();
    int64_t nc_ub = 0;
    for (int32_t q = 0; q < n; ++q) {
        int64_t best = 0;
        if (!nb.nop[q]) {
            best = -1;
            for (int64_t k = nb.desc[q].a_beg; k < nb.desc[q].a_end; ++k) {
                const int32_t a = anchors[k];
                const int64_t d = io[a + 1] - io[a];
                if (best < 0 || d < best) best = d;
            }
        }
        cand_off[q + 1] = cand_off[q] + best;
        nc_ub += (best + kQChunk - 1) / kQChunk;
    }
    if (nc_ub > (int64_t)INT32_MAX - 1) fail(HGX_E_UNSUPPORTED, "hgx_pattern_batch: candidate volume overflow");
    const double t_plan = now_ms();
    const int64_t total_ub = cand_off[n];
    const int32_t nc = (int32_t)std::max<int64_t>(nc_ub, 1);

    // one pinned staging buffer, one upload
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t o = off;
        off = (off + bytes + 15) & ~(size_t)15;
        return o;
    };
    auto bytes_of = [](const auto& v) { return sizeof(v[0]) * std::max<size_t>(v.size(), 1); };
    const size_t o_desc = take(sizeof(QDesc) * n), o_anch = take(bytes_of(anchors)), o_types = take(bytes_of(nb.types)),
                 o_pos = take(bytes_of(nb.pos)), o_poff = take(bytes_of(nb.p_off)),
                 o_pat = take(bytes_of(nb.pattern)), o_nop = take(bytes_of(nb.nop)), o_coff = take(bytes_of(cand_off));
    const size_t up_bytes = off;
    char* h = (char*)g->pinned_buf(up_bytes);
    auto put = [&](size_t o, const auto& v) {
        if (!v.empty()) std::memcpy(h + o, v.data(), sizeof(v[0]) * v.size());
    };
    put(o_desc, nb.desc);
    put(o_anch, anchors);
    put(o_types, nb.types);
    put(o_pos, nb.pos);
    put(o_poff, nb.p_off);
    put(o_pat, nb.pattern);
    put(o_nop, nb.nop);
    put(o_coff, cand_off);
    const double t_pack = now_ms();

    std::vector<std::pair<void*, size_t>> tmp;
    auto dalloc = [&](size_t bytes) {
        void* p = g->alloc(bytes);
        tmp.push_back({p, bytes});
        return p;
    };
    struct TmpGuard {
        hgx_graph* g;
        std::vector<std::pair<void*, size_t>>* t;
        ~TmpGuard() { for (auto& x : *t) g->release(x.first, x.second); }
    } tg{g, &tmp};
    char* d = (char*)dalloc(up_bytes);
    QPlan* d_plan = (QPlan*)dalloc(sizeof(QPlan) * n);
    int32_t* d_nch = (int32_t*)dalloc(sizeof(int32_t) * (n + 1));
    int32_t* d_choff = (int32_t*)dalloc(sizeof(int32_t) * (n + 1));
    int32_t* d_chq = (int32_t*)dalloc(sizeof(int32_t) * nc);
    int32_t* d_slots = (int32_t*)dalloc(sizeof(int32_t) * (size_t)std::max<int64_t>(total_ub, 1));
    int64_t* d_cnt = (int64_t*)dalloc(sizeof(int64_t) * (nc + 1));
    int64_t* d_outoff = (int64_t*)dalloc(sizeof(int64_t) * (nc + 1));
    int64_t* d_qoff = (int64_t*)dalloc(sizeof(int64_t) * (n + 1));
    u64* d_ctr = (u64*)dalloc(sizeof(u64) * kQShards * kQStride);
    int32_t* d_out = (int32_t*)dalloc(sizeof(int32_t) * (size_t)std::max<int64_t>(total_ub, 1));
    size_t scan1 = 0, scan2 = 0;
    HGX_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, scan1, d_nch, d_choff, n + 1, s));
    HGX_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, scan2, d_cnt, d_outoff, nc + 1, s));
    void* d_scan = dalloc(std::max(scan1, scan2));
    size_t scan_bytes = std::max(scan1, scan2);

    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    struct EvGuard {
        hipEvent_t* e;
        ~EvGuard() { for (int i = 0; i < 4; ++i) if (e[i]) (void)hipEventDestroy(e[i]); }
    } evg{ev};
    if (g->timing)
        for (int i = 0; i < 4; ++i) HGX_HIP(hipEventCreate(&ev[i]));
    if (g->timing) HGX_HIP(hipEventRecord(ev[0], s));
    HGX_HIP(hipMemcpyAsync(d, h, up_bytes, hipMemcpyHostToDevice, s));
    HGX_HIP(hipMemsetAsync(d_ctr, 0, sizeof(u64) * kQShards * kQStride, s));
    HGX_HIP(hipMemsetAsync(d_cnt, 0, sizeof(int64_t) * (nc + 1), s));
    HGX_HIP(hipMemsetAsync(d_nch + n, 0, sizeof(int32_t), s));
    const QDesc* d_desc = (const QDesc*)(d + o_desc);
    const int32_t* d_anch = (const int32_t*)(d + o_anch);
    const int32_t* d_types = (const int32_t*)(d + o_types);
    const int64_t* d_coff = (const int64_t*)(d + o_coff);
    // plan, chunk offsets and the chunk -> query map on the device: no host round trip before the match
    hgx_q_plan<<<grid_for(n, 256, 1 << 20), 256, 0, s>>>(n, d_desc, d_anch, d_types, (const int32_t*)(d + o_nop),
                                                         g->inc_off, g->inc_ts_type, d_plan, d_nch);
    HGX_CHECK_LAUNCH();
    HGX_HIP(hipcub::DeviceScan::ExclusiveSum(d_scan, scan_bytes, d_nch, d_choff, n + 1, s));
    hgx_q_chunk_map<<<grid_for(n, 256, 1 << 20), 256, 0, s>>>(n, d_choff, d_chq);
    HGX_CHECK_LAUNCH();
    const int32_t* d_nchunks = d_choff + n;
    if (g->timing) HGX_HIP(hipEventRecord(ev[1], s));
    hgx_pattern_match<<<grid_for((int64_t)nc * 64, 256, 4096), 256, 0, s>>>(
        d_nchunks, d_chq, d_choff, d_coff, d_plan, d_desc, d_anch, d_types, (const int32_t*)(d + o_pos),
        (const int64_t*)(d + o_poff), (const int32_t*)(d + o_pat), g->inc_row, g->inc_type, g->inc_ts_row, g->tgt_off,
        g->tgt_idx, d_slots, d_cnt, d_ctr);
    HGX_CHECK_LAUNCH();
    if (g->timing) HGX_HIP(hipEventRecord(ev[2], s));
    // per-chunk hit counts -> exclusive output offsets -> per-query offsets; compaction into d_out
    HGX_HIP(hipcub::DeviceScan::ExclusiveSum(d_scan, scan_bytes, d_cnt, d_outoff, nc + 1, s));
    hgx_q_offsets<<<grid_for(n + 1, 256, 1 << 20), 256, 0, s>>>(n, d_choff, d_outoff, d_qoff);
    HGX_CHECK_LAUNCH();
    hgx_q_scatter<<<(unsigned)ceil_div((int64_t)nc * 64, 256), 256, 0, s>>>(d_nchunks, d_chq, d_choff, d_coff, d_cnt,
                                                                            d_outoff, d_slots, g->link_atom, d_out);
    HGX_CHECK_LAUNCH();
    u64 hsh[kQShards * kQStride], hctr[qNum] = {0, 0, 0, 0};
    int32_t n_chunks = 0;
    HGX_HIP(hipMemcpyAsync(r->offsets.data(), d_qoff, sizeof(int64_t) * (n + 1), hipMemcpyDeviceToHost, s));
    HGX_HIP(hipMemcpyAsync(hsh, d_ctr, sizeof(hsh), hipMemcpyDeviceToHost, s));
    HGX_HIP(hipMemcpyAsync(&n_chunks, d_nchunks, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HGX_HIP(hipStreamSynchronize(s));
    const double t_sync1 = now_ms();
    const int64_t total = r->offsets[n];
    r->ids.resize((size_t)std::max<int64_t>(total, 0));
    if (total > 0) HGX_HIP(hipMemcpyAsync(r->ids.data(), d_out, sizeof(int32_t) * total, hipMemcpyDeviceToHost, s));
    if (g->timing) HGX_HIP(hipEventRecord(ev[3], s));
    HGX_HIP(hipStreamSynchronize(s));
    if (prof)
        std::fprintf(stderr, "[hgx query] n=%d plan %.3f pack %.3f device+sync %.3f ids %.3f ms\n", n, t_plan - t0,
                     t_pack - t_plan, t_sync1 - t_pack, now_ms() - t_sync1);
    for (int k = 0; k < qNum; ++k)
        for (int sh = 0; sh < kQShards; ++sh) hctr[k] += hsh[sh * kQStride + k];
    if (g->timing) {
        float a = 0, b = 0;
        HGX_HIP(hipEventElapsedTime(&a, ev[0], ev[3]));
        HGX_HIP(hipEventElapsedTime(&b, ev[1], ev[2]));
        r->ms_total = a;
        r->ms_match = b;
    }
    // algorithmic bytes of hgx_pattern_match: per streamed candidate its type (4 B; none in a
    // type-grouped range), per examined candidate its link row, tgt_off pair and target row, 4 B per
    // hit, per chunk its plan / descriptor, plus the conditions
    {
        double cond_bytes = 20.0 * anchors.size() + 4.0 * nb.types.size() + 4.0 * nb.pos.size() +
                            4.0 * nb.pattern.size() + (double)sizeof(QDesc) * n;
        r->bytes_match = 4.0 * (double)hctr[qCand] + 20.0 * (double)hctr[qTyped] + 4.0 * (double)hctr[qArity] +
                         4.0 * (double)hctr[qHits] + (8.0 + sizeof(QPlan) + sizeof(QDesc)) * (double)n_chunks +
                         cond_bytes;
    }
    guard.r = nullptr;
    *out = r;
    HGX_API_END
}

}  // namespace

extern "C" {

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

}  // extern "C"
