// hgx_seq.hip -- order-exact breadth-first traversal: the (link, atom) sequence that
// HGBreadthFirstTraversal.next() returns (C/algorithms/HGBreadthFirstTraversal.java:49-66,143-156),
// for a batch of start atoms.
//
// The reference's FIFO order is reproduced level-synchronously: an atom t
// first discovered at distance d+1 is enqueued by the FIRST yield, in generator stream order, that
// reaches it while the atoms of distance d are expanded in their own FIFO order.  Stream order is
// the lexicographic order of
//     (FIFO rank e of the expanded atom, index j of the link in inc(parent), yield rank k in the link)
// (DefaultALGenerator.getNextLink walks inc(src) ascending, :287-315; FTargetSetIterator yields
// positions ascending, BTargetSetIterator descending, :121-285).  The triple is packed into one
// 64-bit key and every candidate does an atomicMin on key[seed][t]; the winning key names the
// discovering link, and sorting the level's discoveries by key gives the next FIFO segment.
//
// e counts frontier entries across all levels of the batch (seed-major inside a level), so a key
// from an earlier level is always smaller than any key of the current one: key[] doubles as the
// 'examined' map, and a plain load filters the candidates that are already visited before any
// atomic is issued.
//
// Data-parallel structure per level:  flat incidence items (entry, j) of the frontier
// -> hgx_seq_expand (one item per lane, block-local entry search) -> gather final keys ->
// rocPRIM radix sort by key -> hgx_seq_decode (next frontier + (link, atom) pairs).
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <cstring>
#include <vector>

#include "hgx_internal.h"

namespace hgx {
namespace {

typedef unsigned long long u64;
constexpr u64 kNoKey = ~0ull;

enum SeqMode { sSym = 0, sAfterFirst = 1, sBeforeFirst = 2, sBeforeLast = 3, sAfterLast = 4 };

// Same closed-form rule as the bitset engine (hgx_bfs.hip mode_of; pyref.mode_of).
int seq_mode(const hgx_algen_opts& o) {
    bool P = o.return_preceding, S = o.return_succeeding, R = o.reverse_order, RS = o.return_source;
    if (!R) {
        if (!P) return sAfterFirst;
        if (!S && !RS) return sBeforeFirst;
        return sSym;
    }
    if (!P) return sBeforeLast;
    if (!S && !RS) return sAfterLast;
    return sSym;
}

int bitlen(u64 x) { return x ? 64 - __builtin_clzll(x) : 0; }

__global__ void __launch_bounds__(256) k_seq_maxes(int64_t M, const int64_t* __restrict__ tgt_off, int64_t A,
                                                   const int64_t* __restrict__ inc_off, u64* out) {
    u64 ma = 0, md = 0;
    const int64_t n = M > A ? M : A;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        if (i < M) ma = max(ma, (u64)(tgt_off[i + 1] - tgt_off[i]));
        if (i < A) md = max(md, (u64)(inc_off[i + 1] - inc_off[i]));
    }
    for (int off = 32; off > 0; off >>= 1) {
        ma = max(ma, (u64)__shfl_xor(ma, off));
        md = max(md, (u64)__shfl_xor(md, off));
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMax(&out[0], ma);
        atomicMax(&out[1], md);
    }
}

// deg[i] = |inc(fr_atom[i])| (0 at i == F so the exclusive scan yields the total)
__global__ void __launch_bounds__(256) k_seq_degree(int64_t F, const int32_t* __restrict__ fr_atom,
                                                    const int64_t* __restrict__ inc_off, int64_t* __restrict__ deg) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i <= F; i += (int64_t)gridDim.x * blockDim.x)
        deg[i] = i < F ? inc_off[fr_atom[i] + 1] - inc_off[fr_atom[i]] : 0;
}

// last index i in [lo, hi] with pre[i] <= x  (pre non-decreasing, pre[lo] <= x)
__device__ __forceinline__ int64_t seg_search(const int64_t* __restrict__ pre, int64_t lo, int64_t hi, int64_t x) {
    while (lo < hi) {
        int64_t mid = (lo + hi + 1) >> 1;
        if (pre[mid] <= x) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

struct ExpandArgs {
    int64_t T, F;                  // incidence items, frontier entries
    const int64_t* pre;            // [F+1] exclusive degree prefix
    const int32_t* fr_atom;        // [F]
    const int32_t* fr_seed;        // [F] seed slot within the chunk
    u64 e_base;                    // global FIFO rank of entry 0
    int64_t A;
    const int64_t* inc_off;
    const int32_t* inc_row;
    const int32_t* inc_type;
    const int64_t* tgt_off;
    const int32_t* tgt_idx;
    int32_t want_type;             // HGX_NO_TYPE = no link predicate
    int32_t min_arity;             // 2, or 1 with returnSource (DefaultALGenerator.java:94,326-327)
    int32_t mode, rev;
    int32_t sh_e, sh_j;            // key = e << sh_e | j << sh_j | k
    u64* key;                      // [chunk * A]
    int64_t* list;                 // first discoveries of the level: seed * A + atom
    u64* list_n;
    int64_t cap;
};

// One incidence item (frontier entry i, link index j) per lane.  A block covers 256 consecutive
// items; their entries are found by one pair of global searches plus a short per-lane search.
__global__ void __launch_bounds__(256) hgx_seq_expand(ExpandArgs a) {
    __shared__ int64_t s_lo, s_hi;
    const int64_t tiles = (a.T + 255) / 256;
    for (int64_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
        const int64_t t0 = tile * 256, t1 = min(a.T, t0 + 256) - 1;
        __syncthreads();
        if (threadIdx.x == 0) {
            int64_t lo = seg_search(a.pre, 0, a.F - 1, t0);
            s_lo = lo;
            s_hi = seg_search(a.pre, lo, a.F - 1, t1);
        }
        __syncthreads();
        const int64_t it = t0 + threadIdx.x;
        int32_t p = -1, lo = 0, cnt = 0, n = 0;
        int64_t i = 0, j = 0, b = 0;
        if (it <= t1) {
            i = seg_search(a.pre, s_lo, s_hi, it);
            j = it - a.pre[i];
            p = a.fr_atom[i];
            const int64_t ii = a.inc_off[p] + j;
            if (a.want_type < 0 || a.inc_type[ii] == a.want_type) {              // linkPredicate (:300)
                const int32_t L = a.inc_row[ii];
                b = a.tgt_off[L];
                n = (int32_t)(a.tgt_off[L + 1] - b);
                if (n >= a.min_arity) {                                           // minArity (:309)
                    int32_t hi = n;                                               // yielded positions [lo, hi)
                    if (a.mode != sSym) {
                        int32_t fv = -1, lv = -1;
                        for (int32_t q = 0; q < n; ++q)
                            if (a.tgt_idx[b + q] == p) {
                                if (fv < 0) fv = q;
                                lv = q;
                            }
                        if (a.mode == sAfterFirst) lo = fv + 1;
                        else if (a.mode == sBeforeFirst) hi = fv;
                        else if (a.mode == sBeforeLast) hi = lv;
                        else lo = lv + 1;
                    }
                    cnt = hi > lo ? hi - lo : 0;
                }
            }
        }
        int32_t rounds = cnt;
        for (int off = 32; off > 0; off >>= 1) rounds = max(rounds, __shfl_xor(rounds, off));
        const int64_t sA = p >= 0 ? (int64_t)a.fr_seed[i] * a.A : 0;
        const u64 kb = ((a.e_base + (u64)i) << a.sh_e) | ((u64)j << a.sh_j);
        // wave-uniform rounds so first discoveries are appended with one atomic per wave and round
        for (int32_t r = 0; r < rounds; ++r) {
            bool isnew = false;
            int32_t t = 0;
            if (r < cnt) {
                const int32_t q = lo + r;
                t = a.tgt_idx[b + q];
                if (t != p) {                          // the expanded atom is examined already
                    const u64 k = kb | (u64)(a.rev ? n - 1 - q : q);
                    u64* slot = a.key + sA + t;
                    if (*slot > k)                     // else: examined, or an earlier yield won
                        isnew = atomicMin(slot, k) == kNoKey;
                }
            }
            const u64 m = __ballot(isnew);
            if (m) {
                const int lane = threadIdx.x & 63;
                const int leader = __ffsll((long long)m) - 1;
                u64 base = 0;
                if (lane == leader) base = atomicAdd(a.list_n, (u64)__popcll(m));
                base = __shfl(base, leader);
                if (isnew) {
                    const u64 w = base + (u64)__popcll(m & ((1ull << lane) - 1ull));
                    if ((int64_t)w < a.cap) a.list[w] = sA + t;
                }
            }
        }
    }
}

__global__ void __launch_bounds__(256) k_seq_gather_keys(int64_t n, const int64_t* __restrict__ list,
                                                         const u64* __restrict__ key, u64* __restrict__ out) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = key[list[i]];
}

// Sorted discoveries -> next frontier (seed-major FIFO) and the returned (link, atom) pairs.
__global__ void __launch_bounds__(256) hgx_seq_decode(int64_t n, const u64* __restrict__ skey,
                                                      const int64_t* __restrict__ sflat, u64 e_base, int32_t sh_e,
                                                      int32_t sh_j, u64 jmask, int64_t A,
                                                      const int32_t* __restrict__ fr_atom,
                                                      const int32_t* __restrict__ fr_seed,
                                                      const int64_t* __restrict__ inc_off,
                                                      const int32_t* __restrict__ inc_row,
                                                      const int32_t* __restrict__ link_atom,
                                                      int32_t* __restrict__ nx_atom, int32_t* __restrict__ nx_seed,
                                                      int32_t* __restrict__ out_link) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const u64 k = skey[i];
        const int64_t fi = (int64_t)((k >> sh_e) - e_base);
        const int64_t j = (int64_t)((k >> sh_j) & jmask);
        const int32_t p = fr_atom[fi], s = fr_seed[fi];
        out_link[i] = link_atom[inc_row[inc_off[p] + j]];
        nx_atom[i] = (int32_t)(sflat[i] - (int64_t)s * A);
        nx_seed[i] = s;
    }
}

__global__ void k_seq_seed_keys(int32_t B, const int32_t* __restrict__ seeds, int64_t A, u64* key,
                                int32_t* fr_atom, int32_t* fr_seed) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < B) {
        key[(int64_t)i * A + seeds[i]] = 0ull;   // examined.put(start, TRUE) (:42-46)
        fr_atom[i] = seeds[i];
        fr_seed[i] = i;
    }
}

template <class T> struct DevBuf {
    hgx_graph* g;
    T* p = nullptr;
    size_t n = 0;
    explicit DevBuf(hgx_graph* gg) : g(gg) {}
    ~DevBuf() { reset(); }
    void reset() {
        if (p) g->release(p, n * sizeof(T));
        p = nullptr;
        n = 0;
    }
    T* get(size_t want) {
        if (want > n) {
            reset();
            n = std::max<size_t>(want, 1);
            p = (T*)g->alloc(n * sizeof(T));
        }
        return p;
    }
};

}  // namespace
}  // namespace hgx

using namespace hgx;

struct hgx_seq_result {
    int32_t n_seeds = 0;
    int32_t n_levels = 0;           // 1 + deepest distance returned by any seed
    std::vector<int64_t> off;       // [n_seeds + 1]
    std::vector<int32_t> link, atom, dist;
    double ms_total = 0, traversed = 0;
};

extern "C" {

int hgx_bfs_sequence(hgx_graph* g, const int32_t* seeds, int32_t n_seeds, int32_t max_depth,
                     const hgx_algen_opts* opts, hgx_seq_result** out) {
    HGX_API_BEGIN
    if (!g || !out || n_seeds < 0 || (n_seeds > 0 && !seeds)) fail(HGX_E_INVALID, "hgx_bfs_sequence: bad argument");
    *out = nullptr;
    if (g->shard) fail(HGX_E_UNSUPPORTED, "hgx_bfs_sequence: not available on a partition shard");
    // FIFO order and the discovering link follow the incidence order, i.e. rank order; after an
    // update appended ranks whose handles may sort before existing ones that is not handle order
    // (ADVICE r01), and no re-sort of the output can repair it.
    if (!g->ranks_ordered)
        fail(HGX_E_UNSUPPORTED, "hgx_bfs_sequence: ranks were appended by hgx_graph_update and may not follow "
                                "handle order (re-assert with HGX_OPT_RANKS_ORDERED or rebuild the snapshot)");
    hgx_algen_opts o = opts ? *opts : hgx_algen_opts{HGX_NO_TYPE, 1, 1, 0, 0};
    for (int32_t i = 0; i < n_seeds; ++i)
        if (seeds[i] < 0 || seeds[i] >= g->A) fail(HGX_E_INVALID, "hgx_bfs_sequence: seed out of range");
    if (max_depth < -1) fail(HGX_E_INVALID, "hgx_bfs_sequence: bad max_depth");
    std::lock_guard<std::mutex> lk(g->mu);
    HGX_HIP(hipSetDevice(g->device));
    hipStream_t st = g->stream;
    const int64_t A = g->A;
    const int32_t maxd = max_depth < 0 ? INT32_MAX : max_depth;

    if (g->max_deg < 0) {                       // key widths, once per snapshot
        u64* d = (u64*)g->alloc(16);
        HGX_HIP(hipMemsetAsync(d, 0, 16, st));
        k_seq_maxes<<<grid_for(std::max(g->M, A), 256), 256, 0, st>>>(g->M, g->tgt_off, A, g->inc_off, d);
        HGX_CHECK_LAUNCH();
        u64 h[2];
        HGX_HIP(hipMemcpyAsync(h, d, 16, hipMemcpyDeviceToHost, st));
        HGX_HIP(hipStreamSynchronize(st));
        g->release(d, 16);
        g->max_arity = (int64_t)h[0];
        g->max_deg = (int64_t)h[1];
    }
    const int sh_j = bitlen(g->max_arity > 0 ? (u64)(g->max_arity - 1) : 0);
    const int bits_j = bitlen(g->max_deg > 0 ? (u64)(g->max_deg - 1) : 0);
    const int sh_e = sh_j + bits_j;
    const u64 jmask = bits_j ? (bits_j == 64 ? ~0ull : ((1ull << bits_j) - 1ull)) : 0ull;
    // chunk of seeds: e < B * (A + 1) must fit the key, key[B*A] within the memory budget
    int64_t B = std::max<int64_t>(1, std::min<int64_t>(n_seeds, 1024));
    const int64_t budget = g->seq_budget_bytes;
    while (B > 1 && (bitlen((u64)B * (u64)(A + 1)) + sh_e > 64 || B * A * 40 > budget)) B = (B + 1) / 2;
    if (bitlen((u64)B * (u64)(A + 1)) + sh_e > 64)
        fail(HGX_E_UNSUPPORTED, "hgx_bfs_sequence: stream keys exceed 64 bits for this graph");

    hgx_seq_result* r = new hgx_seq_result();
    struct Guard {
        hgx_seq_result* r;
        ~Guard() { delete r; }
    } guard{r};
    r->n_seeds = n_seeds;
    r->off.assign((size_t)n_seeds + 1, 0);
    // per level: (seed slot, link, atom) host copies, assembled seed-major at the end
    struct Level {
        int64_t chunk0;
        int32_t depth;
        std::vector<int32_t> seed, link, atom;
    };
    std::vector<Level> levels;

    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    if (g->timing) {
        HGX_HIP(hipEventCreate(&ev0));
        HGX_HIP(hipEventCreate(&ev1));
        HGX_HIP(hipEventRecord(ev0, st));
    }
    DevBuf<u64> key(g), knew(g), ksort(g);
    DevBuf<int32_t> fa(g), fs(g), na(g), ns(g), olink(g), dseeds(g);
    DevBuf<int64_t> pre(g), pre_in(g), list(g), lsort(g);
    DevBuf<u64> cnt(g);
    DevBuf<char> tmp(g);
    u64* h_cnt = (u64*)g->pinned_buf(64);
    int32_t deepest = 0;
    for (int64_t c0 = 0; c0 < n_seeds; c0 += B) {
        const int64_t nb = std::min<int64_t>(B, n_seeds - c0);
        u64* dkey = key.get((size_t)(nb * A));
        HGX_HIP(hipMemsetAsync(dkey, 0xFF, sizeof(u64) * nb * A, st));
        int32_t* dsd = dseeds.get(nb);
        HGX_HIP(hipMemcpyAsync(dsd, seeds + c0, sizeof(int32_t) * nb, hipMemcpyHostToDevice, st));
        int32_t* cur_a = fa.get(nb);
        int32_t* cur_s = fs.get(nb);
        k_seq_seed_keys<<<grid_for(nb, 256), 256, 0, st>>>((int32_t)nb, dsd, A, dkey, cur_a, cur_s);
        HGX_CHECK_LAUNCH();
        int64_t F = nb;
        u64 e_base = 0;
        u64* dcnt = cnt.get(1);
        for (int32_t d = 0; F > 0 && d < maxd; ++d) {
            // degree prefix over the frontier entries
            int64_t* dpre = pre.get(F + 1);
            int64_t* ddeg = pre_in.get(F + 1);
            k_seq_degree<<<grid_for(F + 1, 256), 256, 0, st>>>(F, cur_a, g->inc_off, ddeg);
            HGX_CHECK_LAUNCH();
            size_t tb = 0;
            HGX_HIP(rocprim::exclusive_scan(nullptr, tb, ddeg, dpre, (int64_t)0, (size_t)F + 1, rocprim::plus<int64_t>(), st));
            HGX_HIP(rocprim::exclusive_scan(tmp.get(tb), tb, ddeg, dpre, (int64_t)0, (size_t)F + 1, rocprim::plus<int64_t>(),
                                            st));
            HGX_HIP(hipMemcpyAsync(&h_cnt[0], dpre + F, sizeof(int64_t), hipMemcpyDeviceToHost, st));
            HGX_HIP(hipStreamSynchronize(st));
            const int64_t T = (int64_t)h_cnt[0];
            r->traversed += (double)T;
            if (T == 0) break;
            const int64_t cap = std::min<int64_t>(nb * A, T * std::max<int64_t>(g->max_arity, 1));
            int64_t* dlist = list.get(cap);
            HGX_HIP(hipMemsetAsync(dcnt, 0, sizeof(u64), st));
            ExpandArgs ea{T, F, dpre, cur_a, cur_s, e_base, A, g->inc_off, g->inc_row, g->inc_type, g->tgt_off,
                          g->tgt_idx, o.link_type, o.return_source ? 1 : 2, seq_mode(o), o.reverse_order ? 1 : 0,
                          sh_e, sh_j, dkey, dlist, dcnt, cap};
            hgx_seq_expand<<<grid_for(ceil_div(T, 256) * 256, 256, 16384), 256, 0, st>>>(ea);
            HGX_CHECK_LAUNCH();
            HGX_HIP(hipMemcpyAsync(&h_cnt[1], dcnt, sizeof(u64), hipMemcpyDeviceToHost, st));
            HGX_HIP(hipStreamSynchronize(st));
            const int64_t nn = (int64_t)h_cnt[1];
            if (nn > cap) fail(HGX_E_DEVICE, "hgx_bfs_sequence: discovery list overflow");
            e_base += (u64)F;
            if (nn == 0) break;
            // order the discoveries by stream key
            u64* dk = knew.get(nn);
            u64* dks = ksort.get(nn);
            int64_t* dls = lsort.get(nn);
            k_seq_gather_keys<<<grid_for(nn, 256), 256, 0, st>>>(nn, dlist, dkey, dk);
            HGX_CHECK_LAUNCH();
            const int end_bit = std::min(64, sh_e + bitlen(e_base));
            tb = 0;
            HGX_HIP(rocprim::radix_sort_pairs(nullptr, tb, dk, dks, dlist, dls, (size_t)nn, 0u, (unsigned)end_bit, st));
            HGX_HIP(rocprim::radix_sort_pairs(tmp.get(tb), tb, dk, dks, dlist, dls, (size_t)nn, 0u, (unsigned)end_bit, st));
            int32_t* nxa = na.get(nn);
            int32_t* nxs = ns.get(nn);
            int32_t* ol = olink.get(nn);
            hgx_seq_decode<<<grid_for(nn, 256), 256, 0, st>>>(nn, dks, dls, e_base - (u64)F, sh_e, sh_j, jmask, A,
                                                              cur_a, cur_s, g->inc_off, g->inc_row, g->link_atom,
                                                              nxa, nxs, ol);
            HGX_CHECK_LAUNCH();
            Level lv;
            lv.chunk0 = c0;
            lv.depth = d + 1;
            lv.seed.resize(nn);
            lv.link.resize(nn);
            lv.atom.resize(nn);
            HGX_HIP(hipMemcpyAsync(lv.seed.data(), nxs, sizeof(int32_t) * nn, hipMemcpyDeviceToHost, st));
            HGX_HIP(hipMemcpyAsync(lv.link.data(), ol, sizeof(int32_t) * nn, hipMemcpyDeviceToHost, st));
            HGX_HIP(hipMemcpyAsync(lv.atom.data(), nxa, sizeof(int32_t) * nn, hipMemcpyDeviceToHost, st));
            levels.push_back(std::move(lv));
            deepest = std::max(deepest, d + 1);
            // the new level becomes the frontier (swap buffers)
            std::swap(fa.p, na.p);
            std::swap(fa.n, na.n);
            std::swap(fs.p, ns.p);
            std::swap(fs.n, ns.n);
            cur_a = fa.p;
            cur_s = fs.p;
            F = nn;
        }
    }
    if (g->timing) HGX_HIP(hipEventRecord(ev1, st));
    HGX_HIP(hipStreamSynchronize(st));
    if (g->timing) {
        float ms = 0;
        HGX_HIP(hipEventElapsedTime(&ms, ev0, ev1));
        r->ms_total = ms;
        (void)hipEventDestroy(ev0);
        (void)hipEventDestroy(ev1);
    }
    // assemble: seed-major, then distance, then FIFO order
    std::vector<int64_t>& off = r->off;
    for (auto& lv : levels)
        for (int32_t s : lv.seed) off[(size_t)(lv.chunk0 + s) + 1]++;
    for (int32_t i = 0; i < n_seeds; ++i) off[i + 1] += off[i];
    const int64_t total = off[n_seeds];
    r->link.resize(total);
    r->atom.resize(total);
    r->dist.resize(total);
    std::vector<int64_t> pos(off.begin(), off.end() - 1);
    for (auto& lv : levels)
        for (size_t i = 0; i < lv.seed.size(); ++i) {
            const int64_t q = pos[(size_t)(lv.chunk0 + lv.seed[i])]++;
            r->link[q] = lv.link[i];
            r->atom[q] = lv.atom[i];
            r->dist[q] = lv.depth;
        }
    r->n_levels = deepest + 1;
    guard.r = nullptr;
    *out = r;
    HGX_API_END
}

int hgx_seq_result_info(const hgx_seq_result* r, int32_t* n_seeds, int64_t* n_pairs, int32_t* n_levels) {
    HGX_API_BEGIN
    if (!r) fail(HGX_E_INVALID, "null result");
    if (n_seeds) *n_seeds = r->n_seeds;
    if (n_pairs) *n_pairs = r->off.back();
    if (n_levels) *n_levels = r->n_levels;
    HGX_API_END
}

int hgx_seq_result_offsets(const hgx_seq_result* r, int64_t* offsets) {
    HGX_API_BEGIN
    if (!r || !offsets) fail(HGX_E_INVALID, "null argument");
    std::memcpy(offsets, r->off.data(), sizeof(int64_t) * r->off.size());
    HGX_API_END
}

int hgx_seq_result_pairs(const hgx_seq_result* r, int32_t* links, int32_t* atoms, int32_t* dists) {
    HGX_API_BEGIN
    if (!r) fail(HGX_E_INVALID, "null result");
    const size_t n = r->link.size();
    if (links && n) std::memcpy(links, r->link.data(), sizeof(int32_t) * n);
    if (atoms && n) std::memcpy(atoms, r->atom.data(), sizeof(int32_t) * n);
    if (dists && n) std::memcpy(dists, r->dist.data(), sizeof(int32_t) * n);
    HGX_API_END
}

int hgx_seq_result_stats(const hgx_seq_result* r, double* ms_total, double* traversed_edges) {
    HGX_API_BEGIN
    if (!r) fail(HGX_E_INVALID, "null result");
    if (ms_total) *ms_total = r->ms_total;
    if (traversed_edges) *traversed_edges = r->traversed;
    HGX_API_END
}

void hgx_seq_result_free(hgx_seq_result* r) { delete r; }

}  // extern "C"
