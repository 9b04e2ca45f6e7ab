// hgx_query.hip -- batched conjunctive pattern matching over typed hyperedges.
//
// Replaces, for And{AtomTypeCondition?, IncidentCondition*, OrderedLinkCondition?}:
//   ExpressionBasedQuery.expand (C/query/cond2qry/ExpressionBasedQuery.java:730-737; orderedLink
//   adds incident(x) for each non-ANY target) -> AndToQuery (C/query/cond2qry/AndToQuery.java:102-306):
//   nested ZigZagIntersectionResult (C/query/impl/ZigZagIntersectionResult.java) over sorted
//   incidence sets and the type index, then PredicateBasedFilter(OrderedLinkCondition)
//   (C/query/impl/PredicateBasedFilter.java:67-86, C/query/OrderedLinkCondition.java:92-124).
//
// GPU formulation: L is in inc(a) <=> a is a target of L.  So the intersection of the anchor
// incidence sets is the smallest anchor set filtered by "every other anchor is in targets(L)",
// which reads one short target row per candidate instead of zig-zag probes.  Candidates are
// visited in ascending order, so the result is ascending like the reference's.  A candidate
// failing the type filter (one 4-byte read) never touches its target row.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstring>

#include "hgx_internal.h"

namespace hgx {

typedef unsigned long long u64;

constexpr int kQChunk = 256;        // candidates per wave-chunk (4 per lane)
constexpr int kMaxAnchors = 32;
constexpr int kMaxPattern = 64;

struct QPlan {
    int64_t beg;    // first incidence entry of the smallest anchor set
    int64_t n;      // its size (0: empty result)
    int32_t amin;   // index of that anchor inside the query's anchor list
    int32_t pad;
};

enum QCtr { qCand = 0, qTyped, qArity, qHits, qNum = 4 };

__device__ __forceinline__ void wave_add_q(u64* ctr, u64 v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(ctr, v);
}

// A wave per chunk of kQChunk candidates of one query (grid-stride over chunks; the counters are
// summed in registers and added once per wave into sharded replicas).
constexpr int kQShards = 16, kQStride = 16;

__global__ void __launch_bounds__(256) hgx_pattern_match(
    int32_t n_chunks, const int32_t* __restrict__ chunk_q, const int32_t* __restrict__ chunk_off,
    const QPlan* __restrict__ plan, const int32_t* __restrict__ q_type, const int64_t* __restrict__ a_off,
    const int32_t* __restrict__ anchors, const int64_t* __restrict__ p_off, const int32_t* __restrict__ pattern,
    const int32_t* __restrict__ q_has_ordered, const int32_t* __restrict__ inc_row,
    const int32_t* __restrict__ inc_type, const int64_t* __restrict__ tgt_off, const int32_t* __restrict__ tgt_idx,
    int32_t* __restrict__ slots, int64_t* __restrict__ counts, u64* __restrict__ ctr) {
    constexpr int K = kQChunk / 64;   // candidates per lane, loaded stage by stage (K loads in flight)
    const int lane = threadIdx.x & 63;
    const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    const int64_t nwave = ((int64_t)gridDim.x * blockDim.x) >> 6;
    u64 n_cand = 0, n_typed = 0, n_ar = 0, n_hits = 0;
    for (int64_t chunk = wave; chunk < n_chunks; chunk += nwave) {
        const int32_t q = chunk_q[chunk];
        const QPlan pl = plan[q];
        const int64_t c0 = (int64_t)(chunk - chunk_off[q]) * kQChunk;
        const int32_t T = q_type[q];
        const int64_t ab = a_off[q], na = a_off[q + 1] - ab;
        const int64_t pb = p_off[q], np = p_off[q + 1] - pb;
        const bool ordered = q_has_ordered[q] != 0;
        // stage 1: the streamed type column (inc_type = link_type of the incidence entry)
        bool pass[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int64_t ci = c0 + k * 64 + lane;
            pass[k] = ci < pl.n && (T < 0 || inc_type[pl.beg + ci] == T);
            n_cand += ci < pl.n;
        }
        // stage 2: link rows of the type-passing candidates; stage 3: their target offsets
        int32_t L[K];
#pragma unroll
        for (int k = 0; k < K; ++k) L[k] = pass[k] ? inc_row[pl.beg + c0 + k * 64 + lane] : -1;
        int64_t b[K], e[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            b[k] = L[k] >= 0 ? tgt_off[L[k]] : 0;
            e[k] = L[k] >= 0 ? tgt_off[L[k] + 1] : 0;
        }
        int32_t written = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            bool hit = L[k] >= 0;
            if (hit) {
                ++n_typed;
                n_ar += (u64)(e[k] - b[k]);
                // IncidentCondition for every other anchor (L in inc(a) <=> a in targets(L))
                for (int64_t j = 0; j < na && hit; ++j) {
                    if (j == pl.amin) continue;
                    const int32_t a = anchors[ab + j];
                    bool found = false;
                    for (int64_t i = b[k]; i < e[k]; ++i) found |= (tgt_idx[i] == a);
                    hit = found;
                }
                // OrderedLinkCondition.satisfies: greedy subsequence with hg.anyHandle()
                if (hit && ordered) {
                    int64_t i = b[k], j = 0;
                    while (i < e[k] && j < np) {
                        const int32_t pj = pattern[pb + j];
                        if (pj < 0 || pj == tgt_idx[i]) ++j;
                        ++i;
                    }
                    hit = (j == np);
                }
            }
            const u64 m = __ballot(hit);
            if (hit) slots[chunk * kQChunk + written + __popcll(m & ((1ull << lane) - 1ull))] = L[k];
            written += __popcll(m);
        }
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
__global__ void __launch_bounds__(256) hgx_q_scatter(int32_t n_chunks, const int64_t* __restrict__ counts,
                                                     const int64_t* __restrict__ out_off,
                                                     const int32_t* __restrict__ slots,
                                                     const int32_t* __restrict__ link_atom, int32_t* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t chunk = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    if (chunk >= n_chunks) return;
    const int64_t c = counts[chunk];
    const int64_t o = out_off[chunk];
    for (int64_t i = lane; i < c; i += 64) out[o + i] = link_atom[slots[chunk * kQChunk + i]];
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

// Normalised batch: ExpressionBasedQuery.expand (orderedLink adds incident(x) for each non-ANY x,
// :730-737) + the toDNF HashSet dedupe (:100) -> per query: type, distinct anchors, pattern, nop.
struct NormBatch {
    std::vector<int32_t> q_type, q_nop, q_ord;
    std::vector<int64_t> a_off, p_off;
    std::vector<int32_t> anchors, pattern;
};

template <class Get>
void normalise(hgx_graph* g, int32_t n, Get get, NormBatch& nb) {
    nb.q_type.resize(n);
    nb.q_nop.resize(n);
    nb.q_ord.resize(n);
    nb.a_off.assign(n + 1, 0);
    nb.p_off.assign(n + 1, 0);
    for (int32_t q = 0; q < n; ++q) {
        int32_t type, n_inc, has_ord, n_pat;
        const int32_t *inc, *pat;
        get(q, type, n_inc, inc, has_ord, n_pat, pat);
        if (n_inc < 0 || n_pat < 0 || (n_inc > 0 && !inc) || (n_pat > 0 && !pat))
            fail(HGX_E_INVALID, "hgx_pattern_batch: bad query " + std::to_string(q));
        if (type < HGX_NO_TYPE) fail(HGX_E_INVALID, "hgx_pattern_batch: bad type in query " + std::to_string(q));
        nb.q_type[q] = type;
        nb.q_ord[q] = has_ord ? 1 : 0;
        const int32_t m = has_ord ? n_pat : 0;
        if (m > kMaxPattern) fail(HGX_E_UNSUPPORTED, "hgx_pattern_batch: ordered pattern too long");
        const size_t a0 = nb.anchors.size();
        auto add = [&](int32_t h) {
            if (h < 0 || h >= g->A)
                fail(HGX_E_INVALID, "hgx_pattern_batch: atom id out of range in query " + std::to_string(q));
            for (size_t k = a0; k < nb.anchors.size(); ++k)
                if (nb.anchors[k] == h) return;
            nb.anchors.push_back(h);
        };
        for (int32_t i = 0; i < n_inc; ++i) add(inc[i]);
        for (int32_t i = 0; i < m; ++i) {
            if (pat[i] == HGX_ANY_HANDLE) continue;
            if (pat[i] < 0) fail(HGX_E_INVALID, "hgx_pattern_batch: bad pattern id");
            add(pat[i]);
        }
        if (nb.anchors.size() == a0)
            fail(HGX_E_UNSUPPORTED, "hgx_pattern_batch: query " + std::to_string(q) + " has no incidence anchor");
        if ((int64_t)(nb.anchors.size() - a0) > kMaxAnchors)
            fail(HGX_E_UNSUPPORTED, "hgx_pattern_batch: too many anchors");
        // an empty OrderedLinkCondition gets QueryMetaData.EMPTY, lands in ORA and compiles to HGQuery.NOP
        nb.q_nop[q] = (has_ord && m == 0) ? 1 : 0;
        for (int32_t i = 0; i < m; ++i) nb.pattern.push_back(pat[i]);
        nb.a_off[q + 1] = (int64_t)nb.anchors.size();
        nb.p_off[q + 1] = (int64_t)nb.pattern.size();
    }
}

int run_batch(hgx_graph* g, int32_t n, NormBatch& nb, hgx_query_result** out);

}  // namespace

extern "C" int hgx_pattern_batch(hgx_graph* g, const hgx_and_query* qs, int32_t n, hgx_query_result** out) {
    HGX_API_BEGIN
    if (!g || !out || n < 0 || (n > 0 && !qs)) fail(HGX_E_INVALID, "hgx_pattern_batch: bad argument");
    *out = nullptr;
    NormBatch nb;
    normalise(g, n,
              [&](int32_t q, int32_t& t, int32_t& ni, const int32_t*& inc, int32_t& ho, int32_t& np,
                  const int32_t*& pat) {
                  t = qs[q].type;
                  ni = qs[q].n_incident;
                  inc = qs[q].incident;
                  ho = qs[q].has_ordered;
                  np = qs[q].n_pattern;
                  pat = qs[q].pattern;
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
    normalise(g, n,
              [&](int32_t q, int32_t& t, int32_t& ni, const int32_t*& ii, int32_t& ho, int32_t& np,
                  const int32_t*& pp) {
                  t = type[q];
                  ni = (int32_t)(inc_off[q + 1] - inc_off[q]);
                  ii = inc ? inc + inc_off[q] : nullptr;
                  ho = has_ordered[q];
                  np = (int32_t)(pat_off[q + 1] - pat_off[q]);
                  pp = pat ? pat + pat_off[q] : nullptr;
              },
              nb);
    return run_batch(g, n, nb, out);
    HGX_API_END
}

namespace {

int run_batch(hgx_graph* g, int32_t n, NormBatch& nb, hgx_query_result** out) {
    HGX_API_BEGIN
    if (g->shard) fail(HGX_E_UNSUPPORTED, "hgx_pattern_batch: not available on a partition shard");
    const std::vector<int64_t>& a_off = nb.a_off;
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
    if (g->inc_off_host.empty()) {   // host copy of the incidence offsets: planning needs no device round trip
        g->inc_off_host.resize((size_t)g->A + 1);
        HGX_HIP(hipMemcpyAsync(g->inc_off_host.data(), g->inc_off, sizeof(int64_t) * (g->A + 1), hipMemcpyDeviceToHost,
                               s));
        HGX_HIP(hipStreamSynchronize(s));
    }
    // plan (AndToQuery orders the ORA inputs by size: the first smallest anchor set drives the scan)
    std::vector<QPlan> plan(n);
    std::vector<int32_t> choff(n + 1, 0);
    const int64_t* io = g->inc_off_host.data();
    int64_t total_ub = 0;
    for (int32_t q = 0; q < n; ++q) {
        QPlan p{0, 0, 0, 0};
        if (!nb.q_nop[q]) {
            int64_t best = -1;
            for (int64_t k = a_off[q]; k < a_off[q + 1]; ++k) {
                const int32_t a = anchors[k];
                const int64_t d = io[a + 1] - io[a];
                if (best < 0 || d < best) {
                    best = d;
                    p.beg = io[a];
                    p.amin = (int32_t)(k - a_off[q]);
                }
            }
            p.n = best < 0 ? 0 : best;
        }
        plan[q] = p;
        total_ub += p.n;
        const int64_t c = choff[q] + (p.n + kQChunk - 1) / kQChunk;
        if (c > INT32_MAX / kQChunk) fail(HGX_E_UNSUPPORTED, "hgx_pattern_batch: candidate volume overflow");
        choff[q + 1] = (int32_t)c;
    }
    const int32_t n_chunks = choff[n], nc = std::max(n_chunks, 1);
    std::vector<int32_t> chq((size_t)nc, 0);
    for (int32_t q = 0; q < n; ++q)
        for (int32_t c = choff[q]; c < choff[q + 1]; ++c) chq[c] = q;

    // one pinned staging buffer, one upload
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t o = off;
        off = (off + bytes + 15) & ~(size_t)15;
        return o;
    };
    const size_t o_type = take(4 * (size_t)n), o_ord = take(4 * (size_t)n), o_aoff = take(8 * (size_t)(n + 1)),
                 o_poff = take(8 * (size_t)(n + 1)), o_anch = take(4 * std::max<size_t>(anchors.size(), 1)),
                 o_pat = take(4 * std::max<size_t>(nb.pattern.size(), 1)), o_plan = take(sizeof(QPlan) * n),
                 o_choff = take(4 * (size_t)(n + 1)), o_chq = take(4 * (size_t)nc);
    const size_t up_bytes = off;
    char* h = (char*)g->pinned_buf(up_bytes);
    std::memcpy(h + o_type, nb.q_type.data(), 4 * (size_t)n);
    std::memcpy(h + o_ord, nb.q_ord.data(), 4 * (size_t)n);
    std::memcpy(h + o_aoff, a_off.data(), 8 * (size_t)(n + 1));
    std::memcpy(h + o_poff, nb.p_off.data(), 8 * (size_t)(n + 1));
    if (!anchors.empty()) std::memcpy(h + o_anch, anchors.data(), 4 * anchors.size());
    if (!nb.pattern.empty()) std::memcpy(h + o_pat, nb.pattern.data(), 4 * nb.pattern.size());
    std::memcpy(h + o_plan, plan.data(), sizeof(QPlan) * n);
    std::memcpy(h + o_choff, choff.data(), 4 * (size_t)(n + 1));
    std::memcpy(h + o_chq, chq.data(), 4 * (size_t)nc);

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
    int32_t* d_slots = (int32_t*)dalloc(sizeof(int32_t) * (size_t)nc * kQChunk);
    int64_t* d_cnt = (int64_t*)dalloc(sizeof(int64_t) * (nc + 1));
    int64_t* d_outoff = (int64_t*)dalloc(sizeof(int64_t) * (nc + 1));
    int64_t* d_qoff = (int64_t*)dalloc(sizeof(int64_t) * (n + 1));
    u64* d_ctr = (u64*)dalloc(sizeof(u64) * kQShards * kQStride);
    int32_t* d_out = (int32_t*)dalloc(sizeof(int32_t) * (size_t)std::max<int64_t>(total_ub, 1));
    size_t scan_bytes = 0;
    HGX_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, d_cnt, d_outoff, nc + 1, s));
    void* d_scan = dalloc(scan_bytes);

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
    const int32_t* d_type = (const int32_t*)(d + o_type);
    const int32_t* d_ord = (const int32_t*)(d + o_ord);
    const int64_t* d_aoff = (const int64_t*)(d + o_aoff);
    const int64_t* d_poff = (const int64_t*)(d + o_poff);
    const int32_t* d_anch = (const int32_t*)(d + o_anch);
    const int32_t* d_pat = (const int32_t*)(d + o_pat);
    const QPlan* d_plan = (const QPlan*)(d + o_plan);
    const int32_t* d_choff = (const int32_t*)(d + o_choff);
    const int32_t* d_chq = (const int32_t*)(d + o_chq);
    if (g->timing) HGX_HIP(hipEventRecord(ev[1], s));
    if (n_chunks > 0) {
        hgx_pattern_match<<<grid_for((int64_t)n_chunks * 64, 256, 4096), 256, 0, s>>>(
            n_chunks, d_chq, d_choff, d_plan, d_type, d_aoff, d_anch, d_poff, d_pat, d_ord, g->inc_row, g->inc_type,
            g->tgt_off, g->tgt_idx, d_slots, d_cnt, d_ctr);
        HGX_CHECK_LAUNCH();
    }
    if (g->timing) HGX_HIP(hipEventRecord(ev[2], s));
    // per-chunk hit counts -> exclusive output offsets -> per-query offsets; compaction into d_out
    HGX_HIP(hipcub::DeviceScan::ExclusiveSum(d_scan, scan_bytes, d_cnt, d_outoff, nc + 1, s));
    hgx_q_offsets<<<grid_for(n + 1, 256, 1 << 20), 256, 0, s>>>(n, d_choff, d_outoff, d_qoff);
    HGX_CHECK_LAUNCH();
    if (n_chunks > 0) {
        hgx_q_scatter<<<(unsigned)ceil_div((int64_t)n_chunks * 64, 256), 256, 0, s>>>(n_chunks, d_cnt, d_outoff,
                                                                                       d_slots, g->link_atom, d_out);
        HGX_CHECK_LAUNCH();
    }
    u64 hsh[kQShards * kQStride], hctr[qNum] = {0, 0, 0, 0};
    HGX_HIP(hipMemcpyAsync(r->offsets.data(), d_qoff, sizeof(int64_t) * (n + 1), hipMemcpyDeviceToHost, s));
    HGX_HIP(hipMemcpyAsync(hsh, d_ctr, sizeof(hsh), hipMemcpyDeviceToHost, s));
    HGX_HIP(hipStreamSynchronize(s));
    const int64_t total = r->offsets[n];
    r->ids.resize((size_t)std::max<int64_t>(total, 0));
    if (total > 0) HGX_HIP(hipMemcpyAsync(r->ids.data(), d_out, sizeof(int32_t) * total, hipMemcpyDeviceToHost, s));
    if (g->timing) HGX_HIP(hipEventRecord(ev[3], s));
    HGX_HIP(hipStreamSynchronize(s));
    for (int k = 0; k < qNum; ++k)
        for (int sh = 0; sh < kQShards; ++sh) hctr[k] += hsh[sh * kQStride + k];
    if (g->timing) {
        float a = 0, b = 0;
        HGX_HIP(hipEventElapsedTime(&a, ev[0], ev[3]));
        HGX_HIP(hipEventElapsedTime(&b, ev[1], ev[2]));
        r->ms_total = a;
        r->ms_match = b;
    }
    // algorithmic bytes of hgx_pattern_match: per candidate inc_type (+ inc_row when the type
    // passes), per type-passing candidate its tgt_off pair and target row, 4 B per hit, 8 B per chunk
    {
        double anchors_bytes = 4.0 * anchors.size() + 16.0 * anchors.size() + 4.0 * nb.pattern.size();
        r->bytes_match = 4.0 * (double)hctr[qCand] + 20.0 * (double)hctr[qTyped] + 4.0 * (double)hctr[qArity] +
                         4.0 * (double)hctr[qHits] + 8.0 * (double)n_chunks + anchors_bytes;
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
