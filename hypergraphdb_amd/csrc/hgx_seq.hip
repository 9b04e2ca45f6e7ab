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
// integer key and every candidate lowers the key of its target with an atomicMin; the winning key
// names the discovering link, and ordering the level's discoveries by key gives the next FIFO segment.
//
// Two engines share that rule:
//   * workgroup per seed (default, hgx_seq_block): the whole traversal of one start atom inside one
//     workgroup, examined set / frontier / ranks in LDS, no host round trip per level -- the shape of
//     the drop-in's calls (one HGGpuTraversal or one hg.subsumed closure at a time);
//   * level-synchronous (fallback for traversals larger than a workgroup holds, HGX_OPT_SEQ_ENGINE 1):
//     flat incidence items (entry, j) of the frontier -> hgx_seq_expand (one item per lane,
//     block-local entry search, atomicMin on key[seed][atom]) -> gather final keys -> rocPRIM radix
//     sort by key -> hgx_seq_decode (next frontier + (link, atom) pairs).
//
// Level-synchronous keys: e counts frontier entries across all levels of the batch (seed-major
// inside a level), so a key from an earlier level is always smaller than any key of the current one:
// key[] doubles as the 'examined' map, and a plain load filters the candidates that are already
// visited before any atomic is issued.
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include <sys/mman.h>

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

// Host-side phase trace of hgx_bfs_sequence (HGX_SEQ_TRACE=1): microseconds since the call began.
struct SeqTrace {
    bool on = trace_env("HGX_SEQ_TRACE");
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    void operator()(const char* what) const {
        if (on)
            std::fprintf(stderr, "[hgx seq trace] %-28s %8.1f us\n", what,
                         std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
};
thread_local SeqTrace* g_seq_trace = nullptr;
inline void seq_mark(const char* what) {
    if (g_seq_trace) (*g_seq_trace)(what);
}

// fn(0 .. n-1) on up to 16 host threads (the job's CPU share; HGX_COPY_THREADS overrides), or on the
// calling thread when `wide` is false.
template <class F>
void host_parallel(int64_t n, bool wide, F&& fn) {
    static const int env = ab_int("HGX_COPY_THREADS", 0);
    const int hw = (int)std::max(1u, std::thread::hardware_concurrency());
    const int nt = !wide ? 1 : (int)std::min<int64_t>(n, env > 0 ? env : std::min(hw, 16));
    if (nt <= 1) {
        for (int64_t k = 0; k < n; ++k) fn(k);
        return;
    }
    std::atomic<int64_t> next{0};
    auto work = [&]() {
        for (int64_t k; (k = next.fetch_add(1)) < n;) fn(k);
    };
    std::vector<std::thread> th;
    th.reserve((size_t)nt - 1);
    try {
        for (int t = 1; t < nt; ++t) th.emplace_back(work);
    } catch (const std::exception&) {
        // no more threads (a process or memory limit): the ones started and this thread finish the jobs
    }
    work();
    for (auto& t : th) t.join();
}

// ---------------------------------------------------------------------------------------------
// Yield adjacency (hgx::yield_adj): incidence entry i of atom p -> the targets it yields (link type,
// yield flag, minimum arity, the mode's position rule, t != p -- DefaultALGenerator.getNextLink
// :287-315 and F/BTargetSetIterator :121-285 as bb_process / sb_process apply them), counted per atom,
// then written per atom in stream order (entry order; inside a link by yield rank: descending
// positions in reverse order).  One wave per atom, a lane per entry.
struct YaArgs {
    int64_t A;
    const int64_t* inc_off;
    const int32_t* inc_row;
    const int32_t* inc_type;
    const uint8_t* yf;
    const int64_t* tgt_off;
    const int32_t* tgt_idx;
    const int32_t* link_atom;
    int32_t mode, rev, type, min_arity;
    int64_t* cnt;          // count pass: [A + 1]
    const int64_t* off;    // fill pass
    int32_t* tgt;
    int32_t* lnk;
};

__device__ __forceinline__ int32_t ya_entry(const YaArgs& a, int32_t p, int64_t i, int32_t& L, int64_t& b,
                                            int32_t& lo, int32_t& hi) {
    lo = hi = 0;
    if (a.type >= 0 && a.inc_type[i] != a.type) return 0;   // linkPredicate (:300)
    if (a.yf && !((a.yf[i] >> a.mode) & 1)) return 0;      // no target this mode can yield
    L = a.inc_row[i];
    b = a.tgt_off[L];
    const int32_t n = (int32_t)(a.tgt_off[L + 1] - b);
    if (n < a.min_arity) return 0;                           // minArity (:309)
    hi = n;
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
    int32_t c = 0;
    for (int32_t q = lo; q < hi; ++q) c += a.tgt_idx[b + q] != p;
    return c;
}

__global__ void __launch_bounds__(256) hgx_ya_count(YaArgs a) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t v = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; v < a.A; v += nw) {
        const int64_t b = a.inc_off[v], e = a.inc_off[v + 1];
        int64_t c = 0;
        for (int64_t i = b + lane; i < e; i += 64) {
            int32_t L, lo, hi;
            int64_t tb;
            c += ya_entry(a, (int32_t)v, i, L, tb, lo, hi);
        }
        for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
        if (lane == 0) a.cnt[v] = c;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) a.cnt[a.A] = 0;
}

__global__ void __launch_bounds__(256) hgx_ya_fill(YaArgs a) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t v = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; v < a.A; v += nw) {
        const int64_t b = a.inc_off[v], e = a.inc_off[v + 1];
        int64_t o = a.off[v];
        for (int64_t i0 = b; i0 < e; i0 += 64) {   // wave-uniform trip count
            const int64_t i = i0 + lane;
            int32_t L = 0, lo = 0, hi = 0, c = 0;
            int64_t tb = 0;
            if (i < e) c = ya_entry(a, (int32_t)v, i, L, tb, lo, hi);
            int32_t x = c;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const int32_t y = __shfl_up(x, off);
                if (lane >= off) x += y;
            }
            const int32_t tot = __shfl(x, 63);
            int64_t w = o + x - c;
            if (c) {
                const int32_t la = a.link_atom[L];
                for (int32_t j = 0; j < hi - lo; ++j) {
                    const int32_t q = a.rev ? hi - 1 - j : lo + j;   // yield rank order
                    const int32_t t = a.tgt_idx[tb + q];
                    if (t == (int32_t)v) continue;
                    a.tgt[w] = t;
                    a.lnk[w] = la;
                    ++w;
                }
            }
            o += tot;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Yield lists (hgx::yield_list): per atom, the links of its incidence entries that pass a fixed link
// type and can yield in a fixed generator mode (yield-flag bit `mode`; every entry in the symmetric
// mode), in entry order.  One wave per atom: count, then (after the offsets' scan) a ballot-compacted
// fill.  A traversal over them reads only the entries that can yield: a class hub whose incidence is
// its subclasses' links costs nothing in hg.subsumes, where none of them yields.
__device__ __forceinline__ bool yl_pass(int64_t i, const int32_t* __restrict__ inc_type, const uint8_t* __restrict__ yf,
                                        int mode, int32_t type) {
    return (!yf || ((yf[i] >> mode) & 1)) && (type < 0 || inc_type[i] == type);
}

__global__ void __launch_bounds__(256) hgx_yl_count(int64_t A, const int64_t* __restrict__ inc_off,
                                                    const int32_t* __restrict__ inc_type, const uint8_t* __restrict__ yf,
                                                    int mode, int32_t type, int64_t* __restrict__ cnt) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t v = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; v < A; v += nw) {
        const int64_t b = inc_off[v], e = inc_off[v + 1];
        int64_t c = 0;
        for (int64_t i = b + lane; i < e; i += 64) c += yl_pass(i, inc_type, yf, mode, type) ? 1 : 0;
        for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
        if (lane == 0) cnt[v] = c;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) cnt[A] = 0;
}

__global__ void __launch_bounds__(256) hgx_yl_fill(int64_t A, const int64_t* __restrict__ inc_off,
                                                   const int32_t* __restrict__ inc_row,
                                                   const int32_t* __restrict__ inc_type, const uint8_t* __restrict__ yf,
                                                   int mode, int32_t type, const int64_t* __restrict__ off,
                                                   int32_t* __restrict__ row) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t v = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; v < A; v += nw) {
        const int64_t b = inc_off[v], e = inc_off[v + 1];
        int64_t o = off[v];
        for (int64_t i0 = b; i0 < e; i0 += 64) {   // wave-uniform trip count
            const int64_t i = i0 + lane;
            const bool ok = i < e && yl_pass(i, inc_type, yf, mode, type);
            const u64 m = __ballot(ok);
            if (ok) row[o + __popcll(m & ((1ull << lane) - 1ull))] = inc_row[i];
            o += __popcll(m);
        }
    }
}


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

// Sorted discoveries -> next frontier (seed-major FIFO) and the returned (link, atom) pairs, the
// pairs written straight into mapped host memory (out_link / out_atom), plus each chunk seed's range
// of the level: [first[s], last[s]) (the level is seed-major: the key's entry rank e is).
__global__ void __launch_bounds__(256) hgx_seq_decode(int64_t n, const u64* __restrict__ skey,
                                                      const int64_t* __restrict__ sflat, u64 e_base, int32_t sh_e,
                                                      int32_t sh_j, u64 jmask, int64_t A,
                                                      const int32_t* __restrict__ fr_atom,
                                                      const int32_t* __restrict__ fr_seed,
                                                      const int64_t* __restrict__ inc_off,
                                                      const int32_t* __restrict__ inc_row,
                                                      const int32_t* __restrict__ link_atom,
                                                      int32_t* __restrict__ nx_atom, int32_t* __restrict__ nx_seed,
                                                      int32_t* __restrict__ out_link, int32_t* __restrict__ out_atom,
                                                      int64_t* __restrict__ first, int64_t* __restrict__ last) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const u64 k = skey[i];
        const int64_t fi = (int64_t)((k >> sh_e) - e_base);
        const int64_t j = (int64_t)((k >> sh_j) & jmask);
        const int32_t p = fr_atom[fi], s = fr_seed[fi];
        const int32_t t = (int32_t)(sflat[i] - (int64_t)s * A);
        out_link[i] = link_atom[inc_row[inc_off[p] + j]];
        out_atom[i] = t;
        nx_atom[i] = t;
        nx_seed[i] = s;
        if (i == 0 || (int32_t)(sflat[i - 1] / A) != s) first[s] = i;
        if (i == n - 1 || (int32_t)(sflat[i + 1] / A) != s) last[s] = i + 1;
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

// ---------------------------------------------------------------------------------------------
// Workgroup-per-seed engine (HGX_OPT_SEQ_ENGINE 0, the default).
//
// The drop-in (HGGpuTraversal.next(), hg.subsumed / hg.subsumes through TraversalBasedQuery) asks for
// one traversal at a time, and the closures it asks for are small: config 5's hg.subsumes closures
// hold <= 1265 atoms over ~15 levels, hg.subsumed ones a median of 1.  The level-synchronous engine
// below pays ~8 launches and 2 host round trips per level for those.  Here one workgroup runs one
// seed's whole traversal with its state in LDS:
//   - an open-addressing hash (kSbHash slots) of the examined atoms: atom id + a 64-bit value
//     ((key + 1) << 32 | discovering link atom id) lowered with atomicMin by every yield of the
//     level; 0 marks an atom examined at an earlier level, so the min never displaces it;
//   - the frontier table: atom, incidence start, degree prefix and 16-byte segment prefix;
//   - a staging area of candidate incidence items (their flat item index), re-used as the rank
//     bitmap or the sort buffer at the end of a level.
// Stream order is the reference's: key = (flat item index it, yield rank k), it = (FIFO entry,
// index of the link in inc(entry)) flattened in order, k = position rank in the link (descending in
// reverse mode) -- the same lexicographic triple as the level-synchronous engine's
// (DefaultALGenerator.getNextLink :287-315; F/BTargetSetIterator :121-285).
// A level: (1) the frontier's incidence is streamed 16 entries per lane (one 16-byte load of the
// ordered-mode yield flags, hgx_inc_yield; the symmetric mode stages every entry) and the entries
// that can yield are staged; (2) each staged entry reads its link's type, targets and atom id, and
// every yielded target not examined yet takes part in the atomicMin; (3) the new atoms are ranked by
// their keys (a bitmap over the level's key space + a popcount prefix, or a bitonic sort when the key
// space is wider than the staging area); rank r is the r-th pair of the level and the r-th entry of
// the next frontier.  Pairs go straight into mapped host memory.  A seed whose traversal needs more
// than kSbPairs pairs (or a level wider than a 32-bit key) reports -1 and reruns on the
// level-synchronous engine.
constexpr int kSbThreads = 512;
constexpr int kSbWaves = kSbThreads / 64;
constexpr int kSbHash = 4096;                       // hash slots (power of two)
constexpr int kSbDisc = kSbHash / 2 - 1;            // examined atoms incl. the seed (load <= 1/2)
constexpr int kSbPairs = kSbDisc - 1;               // pairs one seed may return
constexpr int kSbFront = 2048;                      // frontier entries (>= kSbPairs)
constexpr int kSbCand = 16384;                      // staged candidate items
constexpr int kSbRound = kSbThreads * 16;           // items one staging step may add
constexpr int kSbU = 4;                             // 16-byte segments a lane loads at once
constexpr int kSbInline = 32;                       // seeds passed in the kernel arguments
constexpr int kSbChunk = 1024;                      // seeds per launch (mapped output per launch)
constexpr int kSbSmallRank = 128;                    // levels of at most this many new atoms: ranked by comparisons

struct SbArgs {
    int32_t n;                                      // seeds of this launch
    const int32_t* seeds;                           // device seeds (n > kSbInline)
    int32_t seed_inline[kSbInline];
    const int64_t* inc_off;
    const int32_t* inc_row;
    const int32_t* inc_type;
    const uint8_t* yf;                              // ordered-mode yield flags; null in the symmetric mode
    const int64_t* tgt_off;
    const int32_t* tgt_idx;
    const int32_t* link_atom;
    int32_t want_type, min_arity, mode, rev, kbits, maxd;
    int64_t t_limit;                                // largest item count of a level with 32-bit keys
    int32_t* out_link;                              // [n * kSbPairs] (mapped host memory)
    int32_t* out_atom;
    int32_t* out_dist;
    int64_t* meta;                                  // [3 n]: pairs (-1 = fall back), traversed items, bytes
    // the generator's yield list (yield_list; null: stream the incidence and its yield flags).  Its
    // item numbering keeps the stream order (a subsequence of the entries, in entry order), so the
    // keys rank the same.
    const int64_t* y_off;
    const int32_t* y_row;
    // or the yield adjacency (yield_adj): y_off its offsets, an item is one (target, link atom) pair
    // (kbits 0: the pair's index is its stream position)
    const int32_t* a_tgt;
    const int32_t* a_lnk;
    // the seeds handed back go to the chained grid stage's list (round 6; null: the host collects them):
    // (index of the seed in the call, seed atom) at a slot of an atomic counter (slots >= kMaxCoSeeds dropped:
    // the stage then sees the count and leaves them to the host)
    int32_t c0;                                     // the call's index of this launch's first seed
    int2* chain;
    uint32_t* chain_n;
    int64_t* clk;                                   // HGX_SB_CLOCK (tracing): [2 n] start / end ticks a seed
};

struct SbShared {
    int32_t h_atom[kSbHash];
    u64 h_val[kSbHash];
    int64_t e_fb[kSbFront];                         // frontier entry: first incidence position
    int32_t e_atom[kSbFront];
    int32_t e_dp[kSbFront + 1];                     // degree prefix (flat item index of the entry's first item)
    int32_t e_sp[kSbFront + 1];                     // 16-byte segment prefix
    union {
        int32_t cand[kSbCand];                      // staged items
        u64 bm[kSbCand / 2];                        // rank bitmap over the level's key space
        struct {
            u64 key[kSbFront];
            int32_t pay[kSbFront];
        } srt;                                      // bitonic sort buffer
    } u;
    int64_t wsum[kSbWaves], wsum2[kSbWaves];
    int32_t cp[kSbThreads];                         // rank bitmap: popcount prefix of each thread's words
    int64_t T, S;
    int32_t cand_n, n_disc, ovf, nn;               // nn: new atoms of the level (compaction reservations)
};

// exclusive block scan (every thread calls it); *total = the block sum
__device__ __forceinline__ int64_t sb_scan(SbShared& sm, int64_t v, int64_t* total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int64_t x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int64_t y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    if (lane == 63) sm.wsum[w] = x;
    __syncthreads();
    int64_t base = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < kSbWaves; ++k) {
        const int64_t t = sm.wsum[k];
        base += k < w ? t : 0;
        tot += t;
    }
    __syncthreads();
    *total = tot;
    return base + x - v;
}

// two exclusive block scans in one pass (the frontier's degree and segment prefixes: one pair of barriers)
__device__ __forceinline__ void sb_scan2(SbShared& sm, int64_t v, int64_t u, int64_t* pv, int64_t* pu, int64_t* tv,
                                         int64_t* tu) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int64_t x = v, y = u;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int64_t xs = __shfl_up(x, off), ys = __shfl_up(y, off);
        if (lane >= off) {
            x += xs;
            y += ys;
        }
    }
    if (lane == 63) {
        sm.wsum[w] = x;
        sm.wsum2[w] = y;
    }
    __syncthreads();
    int64_t bx = 0, by = 0, sx = 0, sy = 0;
#pragma unroll
    for (int k = 0; k < kSbWaves; ++k) {
        const int64_t a = sm.wsum[k], b = sm.wsum2[k];
        bx += k < w ? a : 0;
        by += k < w ? b : 0;
        sx += a;
        sy += b;
    }
    __syncthreads();
    *pv = bx + x - v;
    *pu = by + y - u;
    *tv = sx;
    *tu = sy;
}

// last index i in [0, n) with pre[i] <= x (pre non-decreasing, pre[0] <= x)
__device__ __forceinline__ int sb_search(const int32_t* pre, int n, int64_t x) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (pre[mid] <= x) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

__device__ __forceinline__ uint32_t sb_hash(int32_t t) { return ((uint32_t)t * 0x9E3779B1u) >> 20; }

// Examined-set insert: the first arrival claims a slot (one reservation each, so the table never
// fills), then the value is lowered to val unless the atom was examined at an earlier level.
__device__ __forceinline__ void sb_insert(SbShared& sm, int32_t t, u64 val) {
    uint32_t h = sb_hash(t);
    for (;;) {
        int32_t a = sm.h_atom[h];
        if (a == t) break;
        if (a == -1) {
            if (atomicAdd(&sm.n_disc, 1) >= kSbDisc) {
                sm.ovf = 1;
                return;
            }
            a = atomicCAS(&sm.h_atom[h], -1, t);
            if (a == -1 || a == t) break;
        }
        h = (h + 1) & (kSbHash - 1);
    }
    if (sm.h_val[h] > val) atomicMin(&sm.h_val[h], val);
}

// Frontier table of e_atom[0, F): incidence start, degree and segment prefixes, sm.T / sm.S.
__device__ void sb_frontier(SbShared& sm, const SbArgs& a, int F) {
    const int tid = threadIdx.x;
    int64_t dg[4], sg[4], ds = 0, ss = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int i = tid * 4 + k;
        dg[k] = sg[k] = 0;
        if (i < F) {
            const int32_t p = sm.e_atom[i];
            const int64_t b = a.inc_off[p], e = a.inc_off[p + 1];
            if (a.y_off) {   // items: the yield list; S: the incidence entries (traversed)
                const int64_t yb = a.y_off[p], ye = a.y_off[p + 1];
                sm.e_fb[i] = yb;
                dg[k] = ye - yb;
                sg[k] = e - b;
            } else {
                sm.e_fb[i] = b;
                dg[k] = e - b;
                sg[k] = e > b ? ((e + 15) >> 4) - (b >> 4) : 0;
            }
        }
        ds += dg[k];
        ss += sg[k];
    }
    int64_t T, S, dp, sp;
    sb_scan2(sm, ds, ss, &dp, &sp, &T, &S);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int i = tid * 4 + k;
        if (i < F) {
            sm.e_dp[i] = (int32_t)dp;   // exact whenever T <= t_limit (checked by the level)
            sm.e_sp[i] = (int32_t)sp;
        }
        dp += dg[k];
        sp += sg[k];
    }
    if (tid == 0) {
        sm.e_dp[F] = (int32_t)(T < INT32_MAX ? T : INT32_MAX);
        sm.e_sp[F] = (int32_t)(S < INT32_MAX ? S : INT32_MAX);
        sm.T = T;
        sm.S = S;
        sm.nn = 0;
    }
    __syncthreads();
}

// Staged items (it0 < 0; items it0 + c of a yield list otherwise) -> yields -> examined-set inserts.
// nbytes: the thread's algorithmic bytes (the type, row, target-offset, link-id and target loads).
__device__ void sb_process(SbShared& sm, const SbArgs& a, int F, int cn, int64_t& nbytes, int64_t it0) {
    for (int c = threadIdx.x; c < cn; c += kSbThreads) {
        const int64_t it = it0 < 0 ? (int64_t)sm.u.cand[c] : it0 + c;
        const int i = sb_search(sm.e_dp, F, it);
        const int64_t ii = sm.e_fb[i] + (it - sm.e_dp[i]);
        const int32_t p = sm.e_atom[i];
        if (a.a_tgt) {   // the generator's output itself: target + link atom, key = the pair's index
            nbytes += 8;
            sb_insert(sm, a.a_tgt[ii], (((u64)(uint32_t)it + 1ull) << 32) | (u64)(uint32_t)a.a_lnk[ii]);
            continue;
        }
        int32_t L;
        if (a.y_row) {   // the list holds the wanted type only
            L = a.y_row[ii];
            nbytes += 4;
        } else {
            L = a.inc_row[ii];
            const int32_t ty = a.want_type >= 0 ? a.inc_type[ii] : 0;
            nbytes += a.want_type >= 0 ? 8 : 4;
            if (a.want_type >= 0 && ty != a.want_type) continue;                 // linkPredicate (:300)
        }
        const int64_t b = a.tgt_off[L];
        const int32_t n = (int32_t)(a.tgt_off[L + 1] - b);
        const int32_t la = a.link_atom[L];
        nbytes += 20 + 4 * (int64_t)n;
        if (n < a.min_arity) continue;                                           // minArity (:309)
        const u64 kb = ((u64)(uint32_t)it << a.kbits) + 1ull;
        const u64 lw = (u64)(uint32_t)la;
        if (n <= 8) {
            int32_t tg[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) tg[q] = q < n ? a.tgt_idx[b + q] : -1;
            int32_t lo = 0, hi = n;
            if (a.mode != sSym) {
                int32_t fv = -1, lv = -1;
#pragma unroll
                for (int q = 0; q < 8; ++q)
                    if (tg[q] == p) {
                        if (fv < 0) fv = q;
                        lv = q;
                    }
                if (a.mode == sAfterFirst) lo = fv + 1;
                else if (a.mode == sBeforeFirst) hi = fv;
                else if (a.mode == sBeforeLast) hi = lv;
                else lo = lv + 1;
            }
#pragma unroll
            for (int q = 0; q < 8; ++q)
                if (q >= lo && q < hi && tg[q] != p)
                    sb_insert(sm, tg[q], ((kb + (u64)(a.rev ? n - 1 - q : q)) << 32) | lw);
        } else {
            int32_t lo = 0, hi = n;
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
            for (int32_t q = lo; q < hi; ++q) {
                const int32_t t = a.tgt_idx[b + q];
                if (t != p) sb_insert(sm, t, ((kb + (u64)(a.rev ? n - 1 - q : q)) << 32) | lw);
            }
        }
    }
}

__device__ void sb_bitonic(SbShared& sm, int N2) {
    for (int k = 2; k <= N2; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < N2 / 2; i += kSbThreads) {
                const int lo = ((i & ~(j - 1)) << 1) | (i & (j - 1)), hi = lo | j;
                const bool up = (lo & k) == 0;
                const u64 x = sm.u.srt.key[lo], y = sm.u.srt.key[hi];
                if ((x > y) == up) {
                    sm.u.srt.key[lo] = y;
                    sm.u.srt.key[hi] = x;
                    const int32_t t = sm.u.srt.pay[lo];
                    sm.u.srt.pay[lo] = sm.u.srt.pay[hi];
                    sm.u.srt.pay[hi] = t;
                }
            }
            __syncthreads();
        }
}

// New atom in hash slot sl has rank r of its level: pair r of the level, entry r of the next frontier.
__device__ __forceinline__ void sb_emit(SbShared& sm, const SbArgs& a, int64_t o, int r, int sl, int32_t dist) {
    const int32_t t = sm.h_atom[sl];
    const u64 v = sm.h_val[sl];
    a.out_link[o + r] = (int32_t)(uint32_t)v;
    a.out_atom[o + r] = t;
    a.out_dist[o + r] = dist;
    sm.e_atom[r] = t;
    sm.h_val[sl] = 0ull;   // examined from now on
}

__device__ void sb_run(SbShared& sm, const SbArgs& a, int si) {
    const int tid = threadIdx.x, lane = tid & 63;
    const int32_t seed = a.n <= kSbInline ? a.seed_inline[si] : a.seeds[si];
    if (a.clk && tid == 0) a.clk[2 * (int64_t)si] = (int64_t)__builtin_amdgcn_s_memrealtime();
    for (int i = tid; i < kSbHash; i += kSbThreads) {
        sm.h_atom[i] = -1;
        sm.h_val[i] = ~0ull;
    }
    if (tid == 0) {
        sm.cand_n = 0;
        sm.n_disc = 1;
        sm.ovf = 0;
        sm.e_atom[0] = seed;
    }
    __syncthreads();
    if (tid == 0) {   // examined.put(start, TRUE) (HGBreadthFirstTraversal.java:42-46)
        const uint32_t h = sb_hash(seed);
        sm.h_atom[h] = seed;
        sm.h_val[h] = 0ull;
    }
    sb_frontier(sm, a, 1);
    const int64_t obase = (int64_t)si * kSbPairs;
    int F = 1;
    int64_t trav = 0, out_n = 0, nbytes = 0;
    bool ovf = false;
    for (int32_t d = 0; d < a.maxd && F > 0; ++d) {
        const int64_t T = sm.T, S = sm.S;
        trav += a.y_off ? S : T;
        // frontier offsets (+ the yield lists'), streamed yield flags
        nbytes += tid == 0 ? (a.y_off ? 32 * (int64_t)F : 16 * (int64_t)F + (a.yf ? T : 0)) : 0;
        if (T == 0) break;
        if (T > a.t_limit) {
            ovf = true;
            break;
        }
        // every item of a yield list can yield: no flags to stream, no staging
        for (int64_t c0 = 0; a.y_off && c0 < T && !sm.ovf; c0 += (int64_t)1 << 20) {
            sb_process(sm, a, F, (int)min<int64_t>(T - c0, (int64_t)1 << 20), nbytes, c0);
            __syncthreads();
        }
        // (1) stream the frontier's incidence, stage the entries that can yield: kSbU segments per lane
        // loaded at once, staged one segment at a time (a stage flushes through (2) when full)
        bool stop = false;
        for (int64_t sb = 0; sb < (a.y_off ? 0 : S) && !stop; sb += (int64_t)kSbThreads * kSbU) {
            uint4 v[kSbU];
            int64_t lo_[kSbU], hi_[kSbU], ad_[kSbU], it_[kSbU];
#pragma unroll
            for (int u = 0; u < kSbU; ++u) {
                const int64_t s = sb + (int64_t)u * kSbThreads + tid;
                v[u] = make_uint4(~0u, ~0u, ~0u, ~0u);
                lo_[u] = hi_[u] = ad_[u] = it_[u] = 0;
                if (s < S) {
                    const int i = sb_search(sm.e_sp, F, s);
                    lo_[u] = sm.e_fb[i];
                    hi_[u] = lo_[u] + (sm.e_dp[i + 1] - sm.e_dp[i]);
                    ad_[u] = ((lo_[u] >> 4) + (s - sm.e_sp[i])) << 4;
                    it_[u] = sm.e_dp[i] + (ad_[u] - lo_[u]);
                    if (a.yf) v[u] = *(const uint4*)(a.yf + ad_[u]);
                }
            }
#pragma unroll
            for (int u = 0; u < kSbU; ++u) {
                const uint32_t wv[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
                uint32_t mask = 0;
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const int64_t pos = ad_[u] + q;
                    const bool y = a.yf ? ((wv[q >> 2] >> (8 * (q & 3) + a.mode)) & 1u) != 0 : true;
                    if (pos >= lo_[u] && pos < hi_[u] && y) mask |= 1u << q;
                }
                const int cnt = __popc(mask);
                int x = cnt;
#pragma unroll
                for (int off = 1; off < 64; off <<= 1) {
                    const int y = __shfl_up(x, off);
                    if (lane >= off) x += y;
                }
                const int wtot = __shfl(x, 63);
                int base = 0;
                if (lane == 63 && wtot) base = atomicAdd(&sm.cand_n, wtot);
                base = __shfl(base, 63);
                int o = base + x - cnt;
                while (mask) {
                    const int q = __ffs(mask) - 1;
                    mask &= mask - 1;
                    sm.u.cand[o++] = (int32_t)(it_[u] + q);
                }
                __syncthreads();
                const int cn = sm.cand_n;
                const bool last = sb + (int64_t)(u + 1) * kSbThreads >= S;
                if (cn > 0 && (cn > kSbCand - kSbRound || last)) {
                    // (2) the staged entries' links and yields
                    sb_process(sm, a, F, cn, nbytes, -1);
                    __syncthreads();
                    if (tid == 0) sm.cand_n = 0;
                    __syncthreads();
                    if (sm.ovf) stop = true;
                }
                if (last || stop) break;
            }
        }
        if (sm.ovf) {
            ovf = true;
            break;
        }
        // (3) rank the level's new atoms by key
        uint32_t nm = 0;
#pragma unroll
        for (int k = 0; k < kSbHash / kSbThreads; ++k) {
            const int sl = tid * (kSbHash / kSbThreads) + k;
            if (sm.h_atom[sl] != -1 && sm.h_val[sl] != 0ull) nm |= 1u << k;
        }
        {   // the (value, slot) pairs of the new atoms compacted in any order (reservations on sm.nn): the
            // small-level and sort paths rank them, the bitmap path re-reads the values
            const int cnt = __popc(nm);
            int o = cnt ? atomicAdd(&sm.nn, cnt) : 0;
#pragma unroll
            for (int k = 0; k < kSbHash / kSbThreads; ++k)
                if ((nm >> k) & 1u) {
                    const int sl = tid * (kSbHash / kSbThreads) + k;
                    sm.u.srt.key[o] = sm.h_val[sl];
                    sm.u.srt.pay[o++] = sl;
                }
        }
        __syncthreads();
        const int64_t n_new = sm.nn;
        if (n_new == 0) break;
        const int32_t dist = d + 1;
        const uint64_t nbits = (uint64_t)T << a.kbits;
        if (n_new <= kSbSmallRank) {   // a small level: rank = the number of smaller values (values are
                                       // distinct: a key names one item and yield position)
            if (tid < n_new) {
                const u64 v = sm.u.srt.key[tid];
                int r = 0;
                for (int j = 0; j < (int)n_new; ++j) r += sm.u.srt.key[j] < v ? 1 : 0;
                sb_emit(sm, a, obase + out_n, r, sm.u.srt.pay[tid], dist);
            }
        } else if (nbits <= (uint64_t)kSbCand * 32) {   // bitmap over the key space + popcount prefix
            const int W = (int)((nbits + 63) >> 6);
            for (int w = tid; w < W; w += kSbThreads) sm.u.bm[w] = 0ull;
            __syncthreads();
#pragma unroll
            for (int k = 0; k < kSbHash / kSbThreads; ++k)
                if ((nm >> k) & 1u) {
                    const u64 key = (sm.h_val[tid * (kSbHash / kSbThreads) + k] >> 32) - 1ull;
                    atomicOr(&sm.u.bm[key >> 6], 1ull << (key & 63));
                }
            __syncthreads();
            const int cw = (W + kSbThreads - 1) / kSbThreads;
            const int w0 = min(W, tid * cw), w1 = min(W, w0 + cw);
            int c = 0;
            for (int w = w0; w < w1; ++w) c += __popcll(sm.u.bm[w]);
            int64_t tot;
            const int64_t pre = sb_scan(sm, c, &tot);
            sm.cp[tid] = (int32_t)pre;
            __syncthreads();
            int rk[kSbHash / kSbThreads];
#pragma unroll
            for (int k = 0; k < kSbHash / kSbThreads; ++k) {
                rk[k] = 0;
                if ((nm >> k) & 1u) {
                    const u64 key = (sm.h_val[tid * (kSbHash / kSbThreads) + k] >> 32) - 1ull;
                    const int w = (int)(key >> 6), ch = w / cw;
                    int r = sm.cp[ch];
                    for (int x2 = ch * cw; x2 < w; ++x2) r += __popcll(sm.u.bm[x2]);
                    rk[k] = r + __popcll(sm.u.bm[w] & ((1ull << (key & 63)) - 1ull));
                }
            }
#pragma unroll
            for (int k = 0; k < kSbHash / kSbThreads; ++k)
                if ((nm >> k) & 1u) sb_emit(sm, a, obase + out_n, rk[k], tid * (kSbHash / kSbThreads) + k, dist);
        } else {   // bitonic sort of the compacted (value, slot) pairs
            int N2 = 1;
            while (N2 < n_new) N2 <<= 1;
            for (int r = (int)n_new + tid; r < N2; r += kSbThreads) {
                sm.u.srt.key[r] = ~0ull;
                sm.u.srt.pay[r] = -1;
            }
            __syncthreads();
            sb_bitonic(sm, N2);
            for (int r = tid; r < n_new; r += kSbThreads) sb_emit(sm, a, obase + out_n, r, sm.u.srt.pay[r], dist);
        }
        __syncthreads();
        out_n += n_new;
        nbytes += tid == 0 ? 12 * n_new : 0;   // the pairs written
        F = (int)n_new;
        sb_frontier(sm, a, F);
    }
    int64_t tb;
    sb_scan(sm, nbytes, &tb);
    if (tid == 0) {
        a.meta[3 * (int64_t)si] = ovf ? -1 : out_n;
        a.meta[3 * (int64_t)si + 1] = trav;
        a.meta[3 * (int64_t)si + 2] = tb;
        if (a.clk) a.clk[2 * (int64_t)si + 1] = (int64_t)__builtin_amdgcn_s_memrealtime();
        if (ovf && a.chain_n) {
            const uint32_t q = atomicAdd(a.chain_n, 1u);
            if (q < (uint32_t)kMaxCoSeeds) a.chain[q] = make_int2(a.c0 + si, seed);
        }
    }
}

__global__ void __launch_bounds__(kSbThreads) hgx_seq_block(SbArgs a) {
    __shared__ SbShared sm;
    for (int si = blockIdx.x; si < a.n; si += gridDim.x) {
        sb_run(sm, a, si);
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------------------------
// Set-mode workgroup engine (hgx_bfs_batch, HGX_OPT_BFS_BLOCK): the per-depth visited sets V_d of
// one seed inside one workgroup -- the batched engine's result for a traversal that stays small
// (config 5: 1018 of 1024 hg.subsumed closures and every hg.subsumes closure hold <= 1265 atoms, but
// reach 21-24 levels deep, and the batched engine pays two launches and a host turn-around per level
// for every level of the deepest one).  Same yields as the order-exact engine above (the generator's
// link predicate, minimum arity, position rule and yield flags), without the ranking: a set needs no
// FIFO order, so the first arrival that claims an atom's hash slot makes it a member of the next
// level, and the level is the claimed slots.  LDS per workgroup ~37 KB (four workgroups per CU, 16
// waves): a hash of 2048 slots holding <= 1535 atoms, a 1024-entry frontier table and a 2048-item
// staging area; a seed that outgrows any of them (or meets a frontier of more than kBbItemLimit
// incidence entries) reports -1 and runs on the batched engine.
constexpr int kBbThreads = 256;
constexpr int kBbWaves = kBbThreads / 64;
constexpr int kBbHash = 2048;
constexpr int kBbDisc = 1535;                        // examined atoms incl. the seed (load <= 3/4)
constexpr int kBbPairs = kBbDisc - 1;                // atoms one seed may return past V_0
constexpr int kBbFront = 1024;
constexpr int kBbCand = 2048;
constexpr int kBbU = 2;
constexpr int64_t kBbItemLimit = (int64_t)1 << 22;   // frontier incidence entries of a level (streamed yield flags)
// The symmetric mode has no yield flags: every entry costs a link row and its targets, and a level this
// wide all but certainly discovers more atoms than the workgroup holds (config 2's seeds next to hubs);
// such a seed goes straight to the rows engine instead of paying for a flush before it overflows.
constexpr int64_t kBbItemLimitSym = (int64_t)1 << 14;
constexpr int kBbChunk = 4096;                       // seeds per launch (mapped output per launch)

struct BbArgs {
    int32_t n;
    const int32_t* seeds;                            // device seeds (n > kSbInline)
    int32_t seed_inline[kSbInline];
    const int64_t* inc_off;
    const int32_t* inc_row;
    const int32_t* inc_type;
    const uint8_t* yf;                               // ordered-mode yield flags; null in the symmetric mode
    const int64_t* tgt_off;
    const int32_t* tgt_idx;
    int32_t want_type, min_arity, mode, maxd;
    int32_t* out_atom;                               // [n * kBbPairs] (mapped host memory)
    int32_t* out_cnt;                                // [n * kBbPairs]: |V_{d+1}| at d
    int64_t* meta;                                   // [4 n]: atoms (-1 = rerun), traversed items, bytes,
                                                     //        levels with news | levels expanded << 32
    // the grid stage's selection (null: none): an overflowing seed takes slot atomicAdd(sel_n) and
    // records its batch index (base + si) and atom there when the slot is below sel_cap
    unsigned long long* sel_n;
    int32_t* sel_idx;
    int32_t* sel_seed;
    int32_t sel_cap, base;
    // the generator's yield list (yield_list; null: stream the incidence and its yield flags): a
    // frontier atom's items are then only the links that can yield, already of the wanted type
    const int64_t* y_off;
    const int32_t* y_row;
    const int32_t* a_tgt;                            // or the yield adjacency (y_off its offsets): an item is a target
};

struct BbShared {
    int32_t h_atom[kBbHash];
    uint32_t h_new[kBbHash / 32];                    // slot claimed at the current level
    int64_t e_fb[kBbFront];
    int32_t e_atom[kBbFront];
    int32_t e_dp[kBbFront + 1];
    int32_t e_sp[kBbFront + 1];
    int32_t cand[kBbCand];
    int64_t wsum[kBbWaves], wsum2[kBbWaves];
    int64_t T, S;
    int32_t cand_n, n_disc, ovf;
};

__device__ __forceinline__ int64_t bb_scan(BbShared& sm, int64_t v, int64_t* total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int64_t x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int64_t y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    if (lane == 63) sm.wsum[w] = x;
    __syncthreads();
    int64_t base = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < kBbWaves; ++k) {
        const int64_t t = sm.wsum[k];
        base += k < w ? t : 0;
        tot += t;
    }
    __syncthreads();
    *total = tot;
    return base + x - v;
}

// Two exclusive block scans in one pass (one pair of barriers instead of two).
__device__ __forceinline__ void bb_scan2(BbShared& sm, int64_t v, int64_t u, int64_t& pv, int64_t& pu, int64_t* tv,
                                         int64_t* tu) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int64_t x = v, y = u;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int64_t xs = __shfl_up(x, off), ys = __shfl_up(y, off);
        if (lane >= off) {
            x += xs;
            y += ys;
        }
    }
    if (lane == 63) {
        sm.wsum[w] = x;
        sm.wsum2[w] = y;
    }
    __syncthreads();
    int64_t bx = 0, by = 0, tx = 0, ty = 0;
#pragma unroll
    for (int k = 0; k < kBbWaves; ++k) {
        const int64_t a = sm.wsum[k], b = sm.wsum2[k];
        bx += k < w ? a : 0;
        by += k < w ? b : 0;
        tx += a;
        ty += b;
    }
    __syncthreads();
    *tv = tx;
    *tu = ty;
    pv = bx + x - v;
    pu = by + y - u;
}

__device__ __forceinline__ uint32_t bb_hash(int32_t t) { return ((uint32_t)t * 0x9E3779B1u) >> 21; }

// Examined-set insert: a slot is reserved before it is claimed and the reservation is returned when
// another lane claims it first, so the table never holds more than kBbDisc atoms.
__device__ __forceinline__ void bb_insert(BbShared& sm, int32_t t) {
    uint32_t h = bb_hash(t);
    for (;;) {
        int32_t x = sm.h_atom[h];
        if (x == t) return;
        if (x == -1) {
            if (atomicAdd(&sm.n_disc, 1) >= kBbDisc) {
                sm.ovf = 1;
                return;
            }
            x = atomicCAS(&sm.h_atom[h], -1, t);
            if (x == -1) {
                atomicOr(&sm.h_new[h >> 5], 1u << (h & 31));
                return;
            }
            atomicSub(&sm.n_disc, 1);
            if (x == t) return;
        }
        h = (h + 1) & (kBbHash - 1);
    }
}

__device__ void bb_frontier(BbShared& sm, const BbArgs& a, int F) {
    const int tid = threadIdx.x;
    constexpr int K = kBbFront / kBbThreads;
    int64_t dg[K], sg[K], ds = 0, ss = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int i = tid * K + k;
        dg[k] = sg[k] = 0;
        if (i < F) {
            const int32_t p = sm.e_atom[i];
            const int64_t b = a.inc_off[p], e = a.inc_off[p + 1];
            if (a.y_off) {   // items: the yield list; S: the incidence entries (traversed)
                const int64_t yb = a.y_off[p], ye = a.y_off[p + 1];
                sm.e_fb[i] = yb;
                dg[k] = ye - yb;
                sg[k] = e - b;
            } else {
                sm.e_fb[i] = b;
                dg[k] = e - b;
                sg[k] = e > b ? ((e + 15) >> 4) - (b >> 4) : 0;
            }
        }
        ds += dg[k];
        ss += sg[k];
    }
    int64_t T, S, dp, sp;
    bb_scan2(sm, ds, ss, dp, sp, &T, &S);
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int i = tid * K + k;
        if (i < F) {
            sm.e_dp[i] = (int32_t)dp;   // exact whenever T <= kBbItemLimit (checked by the level)
            sm.e_sp[i] = (int32_t)sp;
        }
        dp += dg[k];
        sp += sg[k];
    }
    if (tid == 0) {
        sm.e_dp[F] = (int32_t)(T < INT32_MAX ? T : INT32_MAX);
        sm.e_sp[F] = (int32_t)(S < INT32_MAX ? S : INT32_MAX);
        sm.T = T;
        sm.S = S;
    }
    __syncthreads();
}

// Staged items (it0 < 0; items it0 + c of a yield list otherwise) -> the generator's yields ->
// examined-set inserts (as sb_process, no keys).
__device__ void bb_process(BbShared& sm, const BbArgs& a, int F, int cn, int64_t& nbytes, int32_t it0) {
    for (int c = threadIdx.x; c < cn; c += kBbThreads) {
        if (sm.ovf) break;   // the seed goes to the rows engine: the rest of the flush is wasted work
        const int32_t it = it0 < 0 ? sm.cand[c] : it0 + c;
        const int i = sb_search(sm.e_dp, F, it);
        const int64_t ii = sm.e_fb[i] + (it - sm.e_dp[i]);
        const int32_t p = sm.e_atom[i];
        if (a.a_tgt) {   // the generator's output itself
            nbytes += 4;
            bb_insert(sm, a.a_tgt[ii]);
            continue;
        }
        int32_t L;
        if (a.y_row) {   // the list holds the wanted type only
            L = a.y_row[ii];
            nbytes += 4;
        } else {
            L = a.inc_row[ii];
            nbytes += a.want_type >= 0 ? 8 : 4;
            if (a.want_type >= 0 && a.inc_type[ii] != a.want_type) continue;   // linkPredicate (:300)
        }
        const int64_t b = a.tgt_off[L];
        const int32_t n = (int32_t)(a.tgt_off[L + 1] - b);
        nbytes += 16 + 4 * (int64_t)n;
        if (n < a.min_arity) continue;                                       // minArity (:309)
        if (n <= 8) {
            int32_t tg[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) tg[q] = q < n ? a.tgt_idx[b + q] : -1;
            int32_t lo = 0, hi = n;
            if (a.mode != sSym) {
                int32_t fv = -1, lv = -1;
#pragma unroll
                for (int q = 0; q < 8; ++q)
                    if (tg[q] == p) {
                        if (fv < 0) fv = q;
                        lv = q;
                    }
                if (a.mode == sAfterFirst) lo = fv + 1;
                else if (a.mode == sBeforeFirst) hi = fv;
                else if (a.mode == sBeforeLast) hi = lv;
                else lo = lv + 1;
            }
#pragma unroll
            for (int q = 0; q < 8; ++q)
                if (q >= lo && q < hi && tg[q] != p) bb_insert(sm, tg[q]);
        } else {
            int32_t lo = 0, hi = n;
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
            for (int32_t q = lo; q < hi; ++q) {
                const int32_t t = a.tgt_idx[b + q];
                if (t != p) bb_insert(sm, t);
            }
        }
    }
}

__device__ void bb_run(BbShared& sm, const BbArgs& a, int si) {
    const int tid = threadIdx.x, lane = tid & 63;
    const int32_t seed = a.n <= kSbInline ? a.seed_inline[si] : a.seeds[si];
    for (int i = tid; i < kBbHash; i += kBbThreads) sm.h_atom[i] = -1;
    if (tid < kBbHash / 32) sm.h_new[tid] = 0u;
    if (tid == 0) {
        sm.cand_n = 0;
        sm.n_disc = 1;
        sm.ovf = 0;
        sm.e_atom[0] = seed;
    }
    __syncthreads();
    if (tid == 0) sm.h_atom[bb_hash(seed)] = seed;   // examined.put(start, TRUE) (HGBreadthFirstTraversal.java:42-46)
    bb_frontier(sm, a, 1);
    const int64_t obase = (int64_t)si * kBbPairs;
    int F = 1;
    int64_t trav = 0, out_n = 0, nbytes = 0, n_lev = 0, n_exp = 0;
    bool ovf = false;
    for (int32_t d = 0; d < a.maxd && F > 0; ++d) {
        const int64_t T = sm.T, S = sm.S;
        trav += a.y_off ? S : T;
        n_exp = d + 1;
        // frontier offsets (+ the yield lists'), streamed yield flags
        nbytes += tid == 0 ? (a.y_off ? 32 * (int64_t)F : 16 * (int64_t)F + (a.yf ? T : 0)) : 0;
        if (T == 0) break;
        if (T > (a.mode != sSym ? kBbItemLimit : kBbItemLimitSym)) {
            ovf = true;
            break;
        }
        if (a.y_off) {   // every item can yield: no flags to stream, no staging
            bb_process(sm, a, F, (int)T, nbytes, 0);
            __syncthreads();
            if (sm.ovf) {
                ovf = true;
                break;
            }
        }
        // (1) stream the frontier's incidence and stage the entries that can yield; a lane keeps the
        // entries that did not fit the staging area and stages them after the next flush through (2)
        bool stop = false;
        for (int64_t sb = 0; sb < (a.y_off ? 0 : S) && !stop; sb += (int64_t)kBbThreads * kBbU) {
            uint4 v[kBbU];
            int64_t lo_[kBbU], hi_[kBbU], ad_[kBbU], it_[kBbU];
#pragma unroll
            for (int u = 0; u < kBbU; ++u) {
                const int64_t s = sb + (int64_t)u * kBbThreads + tid;
                v[u] = make_uint4(~0u, ~0u, ~0u, ~0u);
                lo_[u] = hi_[u] = ad_[u] = it_[u] = 0;
                if (s < S) {
                    const int i = sb_search(sm.e_sp, F, s);
                    lo_[u] = sm.e_fb[i];
                    hi_[u] = lo_[u] + (sm.e_dp[i + 1] - sm.e_dp[i]);
                    ad_[u] = ((lo_[u] >> 4) + (s - sm.e_sp[i])) << 4;
                    it_[u] = sm.e_dp[i] + (ad_[u] - lo_[u]);
                    if (a.yf) v[u] = *(const uint4*)(a.yf + ad_[u]);
                }
            }
            for (int u = 0; u < kBbU; ++u) {
                const uint32_t wv[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
                uint32_t mask = 0;
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const int64_t pos = ad_[u] + q;
                    const bool y = a.yf ? ((wv[q >> 2] >> (8 * (q & 3) + a.mode)) & 1u) != 0 : true;
                    if (pos >= lo_[u] && pos < hi_[u] && y) mask |= 1u << q;
                }
                const bool last = sb + (int64_t)(u + 1) * kBbThreads >= S;
                for (;;) {
                    const int cnt = __popc(mask);
                    int x = cnt;
#pragma unroll
                    for (int off = 1; off < 64; off <<= 1) {
                        const int y = __shfl_up(x, off);
                        if (lane >= off) x += y;
                    }
                    const int wtot = __shfl(x, 63);
                    int base = 0;
                    if (lane == 63 && wtot) base = atomicAdd(&sm.cand_n, wtot);
                    base = __shfl(base, 63);
                    int o = base + x - cnt;
                    for (uint32_t m = mask; m; m &= m - 1, ++o) {
                        const int q = __ffs(m) - 1;
                        if (o < kBbCand) {
                            sm.cand[o] = (int32_t)(it_[u] + q);
                            mask &= ~(1u << q);
                        }
                    }
                    __syncthreads();
                    const int staged = sm.cand_n;
                    const bool more = __syncthreads_or(mask != 0u) != 0;
                    const int cn = min(staged, kBbCand);
                    if (cn > 0 && (more || last || cn > kBbCand / 2)) {
                        // (2) the staged entries' links and yields
                        bb_process(sm, a, F, cn, nbytes, -1);
                        __syncthreads();
                        if (tid == 0) sm.cand_n = 0;
                        __syncthreads();
                        if (sm.ovf) {
                            stop = true;
                            break;
                        }
                    }
                    if (!more) break;
                }
                if (last || stop) break;
            }
        }
        __syncthreads();
        if (sm.ovf) {
            ovf = true;
            break;
        }
        // (3) the claimed slots are V_{d+1}: the next frontier, appended to the seed's output
        constexpr int K = kBbHash / kBbThreads;
        const uint32_t nm = (sm.h_new[tid * K / 32] >> ((tid * K) & 31)) & ((1u << K) - 1u);
        int64_t n_new;
        int o = (int)bb_scan(sm, __popc(nm), &n_new);
        if (n_new == 0) break;
        if (n_new > kBbFront) {
            ovf = true;
            break;
        }
#pragma unroll
        for (int k = 0; k < K; ++k)
            if ((nm >> k) & 1u) {
                const int32_t t = sm.h_atom[tid * K + k];
                sm.e_atom[o] = t;
                a.out_atom[obase + out_n + o] = t;
                ++o;
            }
        __syncthreads();
        if (tid < kBbHash / 32) sm.h_new[tid] = 0u;
        if (tid == 0) a.out_cnt[obase + d] = (int32_t)n_new;
        out_n += n_new;
        n_lev = d + 1;
        nbytes += tid == 0 ? 4 * n_new + 4 : 0;   // the atoms and the level count written
        F = (int)n_new;
        bb_frontier(sm, a, F);
    }
    int64_t tb;
    bb_scan(sm, nbytes, &tb);
    if (tid == 0) {
        a.meta[4 * (int64_t)si] = ovf ? -1 : out_n;
        a.meta[4 * (int64_t)si + 1] = trav;
        a.meta[4 * (int64_t)si + 2] = tb;
        a.meta[4 * (int64_t)si + 3] = n_lev | (n_exp << 32);
        if (ovf && a.sel_n) {
            const u64 j = atomicAdd(a.sel_n, 1ull);
            if (j < (u64)a.sel_cap) {
                a.sel_idx[j] = a.base + si;
                a.sel_seed[j] = seed;
            }
        }
    }
}

__global__ void __launch_bounds__(kBbThreads, 4) hgx_bfs_block(BbArgs a) {
    __shared__ BbShared sm;
    for (int si = blockIdx.x; si < a.n; si += gridDim.x) {
        bb_run(sm, a, si);
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------------------------
// Multi-workgroup level loop (hgx_bfs_batch): the few seeds the workgroup stage hands back (config 5:
// six hg.subsumed closures of 2K-101K atoms over 21 levels) in ONE persistent launch of up to
// kCoBlocks resident workgroups, a grid barrier between levels instead of the rows engine's launches and host
// turn-around per level (~50 us a level for those six seeds).
//   - visited: one bitmap per seed (kCoMaxSeeds x A bits, kept on the graph, zero between calls: the
//     epilogue clears the words of the atoms it found); the first atomicOr that sets an atom's bit
//     discovers it;
//   - work items: a discovered atom appends ceil(deg / kCoChunk) items (atom, seed, chunk) to the
//     next level's list, so a hub's incidence is spread over many waves and a level needs no prefix
//     scan; three lists rotate (level d reads d % 3, appends to (d + 1) % 3, and clears (d + 2) % 3);
//   - output: (atom, seed | level << 8) pairs in device memory in arrival order, per-seed atom counts
//     at the end of every level in mapped host memory (the readout's |V_d|); per-seed lists are built
//     on the host only when a reader asks for a set;
//   - the barrier is a monotonic counter (agent-scope release add, acquire spin) with a 1 s limit
//     measured on the constant clock: a launch whose workgroups cannot all become resident reports a
//     timeout (status 4) instead of hanging, and the seeds rerun on the rows engine.
// The generator rules are those of bb_process.  Status: 1 = a work list overflowed, 2 = the pair list
// overflowed, 3 = more than kCoMaxLevels levels, 4 = barrier timeout.  A level's errors go to a status
// word of its parity, which the blocks read after the next barrier: the word they decide on cannot
// change while some block has not read it yet (the next level writes the other one).
// 256 threads a workgroup (one wave a SIMD): config-5 step 0.412-0.423 -> 0.403 ms concurrent,
// 0.571 -> 0.566 serial against 512 (profiles/r04zx_c5_occ_ab.log; HGX_CO_THREADS=512 for A/B)
constexpr int kCoThreads = 256;
// The grid: kCoBlocks workgroups, all resident (at most 2 per CU, one CU slot left).  Fewer, fuller
// workgroups win: config 5's big closures took 0.75 / 0.64 / 0.59 / 0.55 / 0.58 ms with 512 / 192 /
// 128 / 96 / 64 workgroups (the barrier and the segment counters are shared by fewer arrivals), and
// the config-5 step 1.11 -> 0.85 ms (profiles/r04ze_coop_ab.log; HGX_CO_BLOCKS for A/B).
constexpr int kCoMinBlocks = 64, kCoBlocks = 96, kCoMaxBlocks = 512;
constexpr int kCoChunk = 128;   // incidence entries per work item (default; HGX_CO_CHUNK for A/B)
// Same-address atomics serialise (one per ~20 ns): the work-item / pair counters are split into
// kCoSegs segments (block b appends to segment b % kCoSegs, its own part of the lists) and the barrier
// into kCoBarGroups arrival counters whose last arrival reports to the top counter.
constexpr int kCoSegs = 64;
static_assert(kCoMinBlocks >= kCoSegs && kCoSegs <= 64, "every segment has a block; one wave scans the segments");
constexpr int kCoBarGroups = 16;
// a segment's level counter packs its work items (high 24 bits) and the pairs found (low 40)
constexpr int kCoItemShift = 40;
constexpr unsigned long long kCoPairMask = (1ull << kCoItemShift) - 1ull;
constexpr int kCoMaxLevels = 1024;
constexpr unsigned long long kCoTimeout = 100000000ull;   // s_memrealtime ticks (100 MHz): 1 s (HGX_OPT_CO_TIMEOUT: tests)
// ctl words: [0] barrier top, [1 .. kCoBarGroups] arrival counters, [kCoSt] / [kCoSt + 1] status of
// even / odd levels (the seeding: odd; bits: 1 a segment's work items outgrew it, 2 its pairs did,
// 4 more than kCoMaxLevels levels), [kCoSel] seeds the workgroup
// stage handed over, [kCoLev + slot * kCoSegs + seg] level counters (3 rotating slots), then cur [kcap],
// trav [kcap], and as int32: the seeds' batch indices [kcap] and atoms [kcap]
constexpr int kCoSt = 20, kCoSel = 23, kCoLev = 32, kCoCtlWords = kCoLev + 3 * kCoSegs;

struct CoArgs {
    int32_t k;                                       // seeds (<= kcap); -1: the workgroup stage's overflow
                                                     //   list (ctl[kCoSel] seeds; none run when > kcap)
    int32_t kcap;                                    // seeds the buffers hold (<= kMaxCoSeeds)
    const int32_t* seeds;                            // device [k]
    const int32_t* sel_idx;                          // device [kcap]: batch indices of the handed-over seeds
    const int64_t* inc_off;
    const int32_t* inc_row;
    const int32_t* inc_type;
    const uint8_t* yf;
    const int64_t* tgt_off;
    const int32_t* tgt_idx;
    int32_t want_type, min_arity, mode, maxd;
    const int64_t* y_off;                            // the yield list (BbArgs::y_off), or null
    const int32_t* y_row;
    const int32_t* a_tgt;                            // or the yield adjacency's targets (y_off its offsets)
    int32_t chunk;                                   // incidence entries per work item
    int32_t bgroups;                                 // barrier arrival groups (1 .. kCoBarGroups)
    int32_t lite;                                    // per-level barriers: co_barrier_lite
    int64_t vwords;                                  // words of one seed's bitmap
    u64* vis;                                        // [k * vwords]
    int4* fr;                                        // [3 * kCoSegs * fr_seg] work items (atom, seed, chunk, -)
    int64_t fr_seg;
    u64* ctl;                                        // [kCoCtlWords + 2 kcap] + int32 [2 kcap]
    u64* cur;                                        // [kcap] atoms found per seed
    u64* trav;                                       // [kcap] incidence entries of the seed's expanded atoms
    int2* pairs;                                     // [kCoSegs * pseg] (atom, seed | level << 8)
    int64_t pseg;
    int64_t* hmeta;                                  // mapped: [0] status, [1] levels, [2] seeds, [3] bytes,
                                                     //   (atoms, traversed) [kcap], pairs per segment
                                                     //   [kCoSegs], the seeds' batch indices [kcap]
    int64_t* lvl_end;                                // mapped [kcap * kCoMaxLevels]: cur[s] after level d
    int64_t* lvl_trace;                              // mapped [2 * kCoMaxLevels]: start clock, work items
    int64_t* blk_bytes;                              // mapped [gridDim.x]: each block's algorithmic bytes
    unsigned long long timeout;                      // barrier limit in s_memrealtime ticks (kCoTimeout)
};

// Work items and pairs cross workgroups inside the launch: they are written and read with agent-scope
// atomic stores / loads, which stay coherent across the XCDs' L2s by themselves.  So the per-level
// barrier can be the light one (co_barrier_lite): no agent-scope release / acquire, whose L2
// write-back and invalidate (buffer_wbl2 / buffer_inv) cost every level and leave the graph's
// read-only arrays cold in L2 for the next one.
__device__ __forceinline__ void co_put(int4* p, int4 v) {
    u64* q = (u64*)p;
    __hip_atomic_store(q, (u64)(uint32_t)v.x | (u64)(uint32_t)v.y << 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(q + 1, (u64)(uint32_t)v.z | (u64)(uint32_t)v.w << 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int4 co_get(const int4* p) {
    u64* q = (u64*)p;
    const u64 lo = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const u64 hi = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return make_int4((int32_t)lo, (int32_t)(lo >> 32), (int32_t)hi, (int32_t)(hi >> 32));
}
__device__ __forceinline__ void co_put(int2* p, int2 v) {
    __hip_atomic_store((u64*)p, (u64)(uint32_t)v.x | (u64)(uint32_t)v.y << 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int2 co_get(const int2* p) {
    const u64 x = __hip_atomic_load((u64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return make_int2((int32_t)x, (int32_t)(x >> 32));
}

// Light grid barrier: every thread waits for its own memory operations to complete (the agent-scope
// stores and atomics above are then at the coherence point), the block arrives with a relaxed
// agent-scope add, waiters poll relaxed.  Valid because everything another workgroup reads in the
// loop is an agent-scope atomic operation (co_put / co_get, the bitmaps, counters and status words).
__device__ __forceinline__ bool co_barrier_lite(u64* ctl, u64& gen, u64* status, u64 limit) {
    __shared__ int s_to;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        ++gen;
        __hip_atomic_fetch_add(ctl, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const u64 target = gen * gridDim.x;
        const u64 t0 = __builtin_amdgcn_s_memrealtime();
        int to = 0;
        while (__hip_atomic_load(ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            __builtin_amdgcn_s_sleep(2);
            if (__builtin_amdgcn_s_memrealtime() - t0 > limit) {
                atomicOr(status, 4ull);
                to = 1;
                break;
            }
        }
        s_to = to;
    }
    __syncthreads();
    return s_to != 0;
}

// Grid barrier: arrival at the block's group counter (acq_rel: the last arrival of a group carries
// the group's writes on), the group's last arrival adds to the top counter, everyone polls the top
// counter (relaxed polls, one acquire fence after: an acquire load per poll invalidates the caches on
// every iteration of every waiting block, ~50 us a barrier measured with 128 blocks).
// ng = 1: every block adds to the top counter itself (one atomic on the path instead of two).
__device__ __forceinline__ bool co_barrier(u64* ctl, u64& gen, u64* status, int ng, u64 limit) {
    __shared__ int s_to;
    __syncthreads();   // the block's stores and atomics of this level are issued
    if (threadIdx.x == 0) {
        ++gen;
        u64 target;
        if (ng <= 1) {
            __hip_atomic_fetch_add(ctl, 1ull, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
            target = gen * gridDim.x;
        } else {
            const int grp = blockIdx.x % ng;
            const u64 members = (u64)((gridDim.x - grp + ng - 1) / ng);
            const u64 old = __hip_atomic_fetch_add(ctl + 1 + grp, 1ull, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
            if (old + 1 == gen * members)
                __hip_atomic_fetch_add(ctl, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            target = gen * (u64)min((unsigned)ng, gridDim.x);
        }
        const u64 t0 = __builtin_amdgcn_s_memrealtime();
        int to = 0;
        while (__hip_atomic_load(ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            __builtin_amdgcn_s_sleep(2);
            if (__builtin_amdgcn_s_memrealtime() - t0 > limit) {
                atomicOr(status, 4ull);
                to = 1;
                break;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        s_to = to;
    }
    __syncthreads();
    return s_to != 0;
}

// A work item: atom, seed | entries << 8, first incidence entry (low, high 32 bits).  It carries its
// range, so a level's first load is the item itself, not the atom's incidence offsets as well.
__device__ __forceinline__ int4 co_item(int32_t t, int32_t s, int64_t lo, int64_t n) {
    return make_int4(t, s | (int32_t)(n << 8), (int32_t)(uint32_t)lo, (int32_t)(lo >> 32));
}

// One step of a wave over yielded targets at level d (lane: target t of seed s, t < 0: none): the first
// setter of an atom's bit discovers it; the wave's discoveries take their pair slots and their work
// items for level d + 1 in the block's segment with one atomic, the seeds' counts go to the block's
// LDS counters (flushed once a level).  Every lane of the wave calls it.
__device__ __forceinline__ void co_step(const CoArgs& a, int32_t s, int32_t t, int32_t d, int slot_next, int seg,
                                        u64 pbase_seg, int64_t& nbytes, unsigned long long* cnt_l,
                                        unsigned long long* trav_l) {
    const int lane = threadIdx.x & 63;
    bool nw = false;
    int64_t deg = 0, b0 = 0, trv = 0;   // items (entries, or yield-list entries), incidence entries
    if (t >= 0) {   // the bit and the target's incidence range in flight together
        u64* w = a.vis + (int64_t)s * a.vwords + (t >> 6);
        const u64 bit = 1ull << (t & 63);
        int64_t b1 = 0, i0 = 0, i1 = 0;
        if (d + 1 < a.maxd) {
            i0 = a.inc_off[t];
            i1 = a.inc_off[t + 1];
            if (a.y_off) {
                b0 = a.y_off[t];
                b1 = a.y_off[t + 1];
            } else {
                b0 = i0;
                b1 = i1;
            }
        }
        nw = !(atomicOr(w, bit) & bit);   // [xwg] vis
        deg = b1 - b0;
        trv = i1 - i0;
    }
    const u64 m = __ballot(nw);
    if (!m) return;
    if (nw) atomicAdd(&cnt_l[s], 1ull);
    const u64 nch = nw ? (u64)((deg + a.chunk - 1) / a.chunk) : 0ull;
    if (nw && trv) atomicAdd(&trav_l[s], (unsigned long long)trv);   // expanded at level d + 1
    u64 x = nch;   // the wave's work items and pairs: one packed reservation (items << 40 | pairs)
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const u64 y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    u64 wb = 0;
    if (lane == 63) wb = atomicAdd(a.ctl + kCoLev + slot_next * kCoSegs + seg, (x << kCoItemShift) | (u64)__popcll(m));   // [xwg]
    wb = __shfl(wb, 63);
    if (!nw) return;
    u64* status = a.ctl + kCoSt + (d & 1);
    const u64 pos = pbase_seg + (wb & kCoPairMask) + (u64)__popcll(m & ((1ull << lane) - 1ull));
    if ((int64_t)pos < a.pseg) co_put(a.pairs + (int64_t)seg * a.pseg + (int64_t)pos, make_int2(t, s | (d + 1) << 8));   // [xwg]
    else atomicOr(status, 2ull);   // [xwg]
    nbytes += 8;
    if (nch == 0) return;
    const u64 base = (wb >> kCoItemShift) + x - nch;
    if ((int64_t)(base + nch) > a.fr_seg) {
        atomicOr(status, 1ull);   // [xwg]
        return;
    }
    int4* fr = a.fr + ((int64_t)slot_next * kCoSegs + seg) * a.fr_seg;
    for (u64 c = 0; c < nch; ++c)
        co_put(fr + base + c, co_item(t, s, b0 + (int64_t)c * a.chunk, min<int64_t>(a.chunk, deg - (int64_t)c * a.chunk)));   // [xwg]
    nbytes += 16 * (int64_t)nch;
}

// NT threads a workgroup (kCoThreads; 512 for A/B, HGX_CO_THREADS)
//
// CROSS-WORKGROUP INVARIANT (the precondition of co_barrier_lite, which neither writes back nor
// invalidates the non-coherent per-XCD L2s): inside the level loop every location one workgroup writes
// and another reads is accessed ONLY through agent-scope atomics, each tagged [xwg] below --
//   ctl counters / status words / barrier   __hip_atomic_* and atomicAdd / atomicOr (agent scope)
//   fr (work items)                          co_put / co_get (agent-scope atomic 64-bit store / load)
//   pairs                                    co_put / co_get
//   vis (per-seed bitmaps)                   atomicOr (the discovery test itself)
//   cur / trav (per-seed counts)             atomicAdd, read with __hip_atomic_load
// Everything else is private to a workgroup (LDS, registers), read-only for the launch (the CSR, the
// yield lists, seeds, sel_idx: written before the launch began), or written for the HOST only and read
// after the grid has exited (hmeta, lvl_end, lvl_trace, blk_bytes: mapped memory).  The epilogue's plain
// stores into vis happen after the last barrier, when no workgroup of this launch reads vis again.  A new
// plain store to a shared location in the loop would break the light barrier silently on multi-XCD
// parts; tests/test_gpu_bfs.py::test_grid_stage_stress runs the stage at config-5 scale against the rows
// engine to catch it.
template <int NT>
__global__ void __launch_bounds__(NT) hgx_bfs_coop(CoArgs a) {
    constexpr int kCoThreads = NT, kCoWaves = NT / 64;
    static_assert(NT >= 128 + kMaxCoSeeds, "a level's start reads the seeds' counts with threads 128 ..");
    const int lane = threadIdx.x & 63;
    const int64_t gw = (int64_t)blockIdx.x * kCoWaves + (threadIdx.x >> 6), nw = (int64_t)gridDim.x * kCoWaves;
    const int seg = blockIdx.x % kCoSegs;
    __shared__ unsigned long long cnt_l[kMaxCoSeeds], trav_l[kMaxCoSeeds];   // this block's per-seed counts of a level
    __shared__ int64_t seg_pre[kCoSegs + 1];                                 // the level's items per segment, prefix
    __shared__ u64 seg_pairs;                                                // pairs of this block's segment at the level
    __shared__ u64 s_st;                                                     // the previous level's status
    if (threadIdx.x < kMaxCoSeeds) {
        cnt_l[threadIdx.x] = 0;
        trav_l[threadIdx.x] = 0;
    }
    // the seeds: the host's list, or the workgroup stage's hand-over (written by the launches before
    // this one on the stream; every block reads the same count and leaves together when none fit)
    int32_t k = a.k;
    if (k < 0) {
        const u64 n = __hip_atomic_load(a.ctl + kCoSel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        k = n > (u64)a.kcap ? a.kcap + 1 : (int32_t)n;
        if (blockIdx.x == 0) {
            if (threadIdx.x == 0) a.hmeta[2] = (int64_t)n;   // hmeta[0] stays -1 until a normal exit
            for (int j = threadIdx.x; j < k && j < a.kcap; j += kCoThreads)
                a.hmeta[4 + 2 * a.kcap + kCoSegs + j] = a.sel_idx[j];
        }
        if (k == 0 || k > a.kcap) return;
    }
    u64 gen = 0;
    int64_t nbytes = 0;   // algorithmic bytes of this thread (the block's sum goes to blk_bytes at the end)
    if (blockIdx.x == 0)   // level 0 (segment 0): the seeds (examined.put(start, TRUE), HGBreadthFirstTraversal.java:42-46)
        for (int s = threadIdx.x; s < k; s += kCoThreads) {
            const int32_t t = a.seeds[s];
            atomicOr(a.vis + (int64_t)s * a.vwords + (t >> 6), 1ull << (t & 63));
            const int64_t trv = a.inc_off[t + 1] - a.inc_off[t];
            const int64_t b = a.y_off ? a.y_off[t] : a.inc_off[t];
            const int64_t deg = (a.y_off ? a.y_off[t + 1] : a.inc_off[t + 1]) - b;
            if (a.maxd > 0 && trv > 0) atomicAdd(a.trav + s, (u64)trv);
            if (a.maxd > 0 && deg > 0) {
                const u64 nch = (u64)((deg + a.chunk - 1) / a.chunk);
                const u64 base = atomicAdd(a.ctl + kCoLev, nch << kCoItemShift) >> kCoItemShift;
                if ((int64_t)(base + nch) > a.fr_seg) {
                    atomicOr(a.ctl + kCoSt + 1, 1ull);
                    continue;
                }
                for (u64 c = 0; c < nch; ++c)
                    co_put(a.fr + base + c, co_item(t, s, b + (int64_t)c * a.chunk, min<int64_t>(a.chunk, deg - (int64_t)c * a.chunk)));
            }
        }
    const int ng = a.lite ? 1 : a.bgroups;   // the light barrier adds to the top counter directly
    bool timed_out = a.lite ? co_barrier_lite(a.ctl, gen, a.ctl + kCoSt, a.timeout)
                            : co_barrier(a.ctl, gen, a.ctl + kCoSt, ng, a.timeout);
    int32_t d = 0;
    u64 pbase = 0;   // pairs of this block's segment found before the current level
    for (; !timed_out; ++d) {
        const int slot = d % 3, slot_next = (d + 1) % 3;
        if (threadIdx.x < 64) {   // the level's items per segment -> prefix; this segment's new pairs
            const u64 packed = threadIdx.x < kCoSegs
                                   ? __hip_atomic_load(a.ctl + kCoLev + slot * kCoSegs + threadIdx.x, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT)
                                   : 0ull;
            int64_t x = (int64_t)(packed >> kCoItemShift);
            const int64_t v = x;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const int64_t y = __shfl_up(x, off);
                if ((int)threadIdx.x >= off) x += y;
            }
            if (threadIdx.x < kCoSegs) seg_pre[threadIdx.x] = x - v;
            if (threadIdx.x == kCoSegs - 1) seg_pre[kCoSegs] = x;
            if ((int)threadIdx.x == seg) seg_pairs = packed & kCoPairMask;
        } else if (threadIdx.x == 64) {   // errors of level d - 1 (its parity word; level d writes the other one)
            s_st = __hip_atomic_load(a.ctl + kCoSt + ((d + 1) & 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else if (blockIdx.x == 0 && d > 0 && threadIdx.x >= 128 && (int)threadIdx.x < 128 + k) {
            const int s = threadIdx.x - 128;   // every seed's atom count after level d - 1
            a.lvl_end[(int64_t)s * kCoMaxLevels + d - 1] =
                (int64_t)__hip_atomic_load(a.cur + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();   // (the three loads above come from different waves: in flight together)
        const int64_t nf = seg_pre[kCoSegs];
        pbase += seg_pairs;
        const u64 st = s_st;
        __syncthreads();   // seg_pre / seg_pairs / s_st are read before the next level rewrites them
        if (st != 0 || nf == 0 || d >= a.maxd) break;   // the same decision in every block
        if (d >= kCoMaxLevels) {
            if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(a.ctl + kCoSt, 4ull);
            break;
        }
        if (blockIdx.x == 0) {   // read at level d - 1; appended to at level d + 1
            if (threadIdx.x < kCoSegs)
                __hip_atomic_store(a.ctl + kCoLev + ((d + 2) % 3) * kCoSegs + threadIdx.x, 0ull, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            if (threadIdx.x == 0) {
                a.lvl_trace[2 * d] = (int64_t)__builtin_amdgcn_s_memrealtime();   // level start, work items
                a.lvl_trace[2 * d + 1] = nf;
            }
        }
        const int4* fr = a.fr + (int64_t)slot * kCoSegs * a.fr_seg;
        // a wave takes `per` work items at once (one per lane, per <= 64 spreads the level over every
        // wave of the grid) and walks their incidence entries as one flat range, 64 entries a step (most
        // items are atoms of a few entries: one item per wave would leave most lanes idle)
        const int64_t per = min<int64_t>(64, (nf + nw - 1) / nw);
        for (int64_t it0 = gw * per; it0 < nf; it0 += nw * per) {
            const int64_t it = it0 + lane;
            int32_t ip = -1, is = 0;
            int64_t ilo = 0, icnt = 0;
            if (lane < per && it < nf) {
                int lo = 0, hi = kCoSegs - 1;   // the item's segment: the last with seg_pre <= it
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (seg_pre[mid] <= it) lo = mid;
                    else hi = mid - 1;
                }
                const int4 e = co_get(fr + (int64_t)lo * a.fr_seg + (it - seg_pre[lo]));   // [xwg]
                ip = e.x;
                is = e.y & 0xFF;
                ilo = (int64_t)(uint32_t)e.z | (int64_t)e.w << 32;
                icnt = (int64_t)(e.y >> 8);
                nbytes += 16 + (a.yf && !a.y_row ? icnt : 0);   // the item, the streamed flags
            }
            int64_t x = icnt;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const int64_t y = __shfl_up(x, off);
                if (lane >= off) x += y;
            }
            const int64_t T = __shfl(x, 63), ex = x - icnt;
            for (int64_t f0 = 0; f0 < T; f0 += 64) {   // wave-uniform: every lane reaches co_step
                const int64_t f = f0 + lane;
                int o = 0;   // owner lane: the last lane whose range starts at or before f
#pragma unroll
                for (int step = 32; step > 0; step >>= 1) {
                    const int mid = o + step;
                    if (__shfl(ex, mid) <= f) o = mid;
                }
                const int32_t p = __shfl(ip, o), s = __shfl(is, o);
                const int64_t ii = __shfl(ilo, o) + (f - __shfl(ex, o));
                if (a.a_tgt) {   // the generator's output itself: one target per lane (wave-uniform branch)
                    const int32_t t = f < T ? a.a_tgt[ii] : -1;
                    nbytes += f < T ? 4 : 0;
                    co_step(a, s, t, d, slot_next, seg, pbase, nbytes, cnt_l, trav_l);
                    continue;
                }
                // the flag, the link and its type in flight together
                const bool in = f < T;
                const bool yl = a.y_row != nullptr;   // a yield list: every entry yields, of the wanted type
                const uint8_t yfl = in && !yl && a.yf ? a.yf[ii] : (uint8_t)0xFF;
                const int32_t L = in ? (yl ? a.y_row[ii] : a.inc_row[ii]) : 0;
                const int32_t lty = in && !yl && a.want_type >= 0 ? a.inc_type[ii] : a.want_type;
                bool act = in && ((yfl >> a.mode) & 1);   // a target this mode can yield
                int64_t tb = 0;
                int32_t qlo = 0, qhi = 0;
                if (act) {
                    nbytes += yl || a.want_type < 0 ? 4 : 8;
                    act = lty == a.want_type;   // linkPredicate (:300)
                    if (act) {
                        tb = a.tgt_off[L];
                        const int32_t n = (int32_t)(a.tgt_off[L + 1] - tb);
                        nbytes += 16 + 4 * (int64_t)n;
                        act = n >= a.min_arity;                              // minArity (:309)
                        int32_t fv = -1, lv = -1;
                        if (act && a.mode != sSym)
                            for (int32_t q = 0; q < n; ++q)
                                if (a.tgt_idx[tb + q] == p) {
                                    if (fv < 0) fv = q;
                                    lv = q;
                                }
                        qhi = n;
                        if (a.mode == sAfterFirst) qlo = fv + 1;
                        else if (a.mode == sBeforeFirst) qhi = fv;
                        else if (a.mode == sBeforeLast) qhi = lv;
                        else if (a.mode == sAfterLast) qlo = lv + 1;
                        if (!act) qhi = qlo;
                    }
                }
                for (int32_t q = qlo; __ballot(q < qhi); ++q) {   // one target per lane per step
                    int32_t t = -1;
                    if (q < qhi) {
                        t = a.tgt_idx[tb + q];
                        if (t == p) t = -1;
                    }
                    co_step(a, s, t, d, slot_next, seg, pbase, nbytes, cnt_l, trav_l);
                }
            }
        }
        __syncthreads();   // the block's per-seed counts of this level -> the seed counters
        for (int j = threadIdx.x; j < k; j += kCoThreads) {
            if (cnt_l[j]) atomicAdd(a.cur + j, cnt_l[j]);      // [xwg]
            if (trav_l[j]) atomicAdd(a.trav + j, trav_l[j]);   // [xwg]
            cnt_l[j] = 0;
            trav_l[j] = 0;
        }
        timed_out = a.lite ? co_barrier_lite(a.ctl, gen, a.ctl + kCoSt, a.timeout)
                           : co_barrier(a.ctl, gen, a.ctl + kCoSt, ng, a.timeout);
    }
    if (timed_out) {
        // A block that gave up on a barrier reports it in its own mapped word (the host set it to 0): the
        // status word alone cannot carry it -- a late block may pass a barrier the others already left,
        // or every other block may leave the loop normally after a barrier this block timed out on (a
        // race with the last arrival), and block 0 then writes status 0.  The host reads both after the
        // whole grid has exited, clears the bitmaps and sends the seeds to the rows engine.
        if (threadIdx.x == 0) __hip_atomic_store(a.hmeta + 3, 1ll, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
    }
    // every block left the loop after the same barrier, which every count, status word and pair had
    // reached: no further barrier.  The block's algorithmic bytes go to its own mapped word.
    {
        __shared__ int64_t bsum[kCoWaves];
        for (int off = 32; off > 0; off >>= 1) nbytes += __shfl_xor(nbytes, off);
        if (lane == 0) bsum[threadIdx.x >> 6] = nbytes;
        __syncthreads();
        if (threadIdx.x == 0) {
            int64_t t = 0;
            for (int w = 0; w < kCoWaves; ++w) t += bsum[w];
            a.blk_bytes[blockIdx.x] = t;
        }
    }
    // clear the bitmap words of the atoms found, the blocks of a segment splitting its pairs (the host
    // clears the whole bitmaps when a list overflowed)
    const u64 st = __hip_atomic_load(a.ctl + kCoSt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) |
                   __hip_atomic_load(a.ctl + kCoSt + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int64_t np = min((int64_t)pbase, a.pseg);
    if (st == 0) {
        const int64_t nblk_seg = ((int64_t)gridDim.x - seg + kCoSegs - 1) / kCoSegs;
        for (int64_t i = (int64_t)(blockIdx.x / kCoSegs) * kCoThreads + threadIdx.x; i < np; i += nblk_seg * kCoThreads) {
            const int2 pr = co_get(a.pairs + (int64_t)seg * a.pseg + i);   // [xwg]
            a.vis[(int64_t)(pr.y & 0xFF) * a.vwords + (pr.x >> 6)] = 0ull;
        }
        if (blockIdx.x == 0)
            for (int s = threadIdx.x; s < k; s += kCoThreads) a.vis[(int64_t)s * a.vwords + (a.seeds[s] >> 6)] = 0ull;
    }
    if (blockIdx.x < kCoSegs && threadIdx.x == 0) a.hmeta[4 + 2 * a.kcap + blockIdx.x] = (int64_t)pbase;   // pairs per segment
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        a.hmeta[0] = (int64_t)st;
        a.hmeta[1] = d;
    }
    if (blockIdx.x == 0)
        for (int s = threadIdx.x; s < k; s += kCoThreads) {
            a.hmeta[4 + 2 * s] = (int64_t)__hip_atomic_load(a.cur + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            a.hmeta[5 + 2 * s] = (int64_t)__hip_atomic_load(a.trav + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
}

// ---------------------------------------------------------------------------------------------
// Level-synchronous engine (the traversals a workgroup cannot hold: more than kSbPairs pairs).
//
// A chunk of nb seeds runs level by level with fixed-grid kernels that read every size from device
// memory, so the host never waits inside a level; it enqueues level d+1 before it polls level d's
// frontier size from mapped memory (a finished traversal costs one level of no-op launches).
//
// State (round 5: no per-seed key table):
//   vis    [A x W] u64  examined rows, atom-major, bit s of row t <=> seed s examined t
//                       (HGBreadthFirstTraversal.examined, :36,:59-62); W = ceil(nb / 64)
//   disc / dval         the level's discoveries (seed * A + atom, value), value =
//                       ((it << kbits | k) + 1) << 32 | discovering link atom, it = the flat item index
//                       (entry, link index) of the yield, k its rank in the link -- the reference's
//                       stream order (file header); the minimum over a target's yields is its
//                       discovery (DefaultALGenerator.getNextLink :287-315, HGBreadthFirstTraversal :56-64)
// A level finds its discoveries one of two ways (hgx_ls_prefix decides on the device from the level's
// item count T against the incidence I):
//   push (narrow levels): every item's yields not examined yet lower the value of a level-local open-
//        addressing hash keyed by (seed, atom) with atomicMin; the first claimer of a slot appends it
//        (hgx_ls_expand).  The table is sized to the discovery capacity and cleared slot by slot by the
//        level's own bits pass (no per-level memset).
//   pull (wide levels, the incidence items of an untyped / typed generator without the yield
//        adjacency): every atom t with a seed that has not examined it scans inc(t) -- for each link L
//        and co-target p of t that is on some seed's frontier (the union bitmap), the seeds s with p on
//        their frontier and t not examined get the candidate value with it = pre(s, p) + j(p, L) (the
//        item index of p's entry for s plus the index of L in inc(p), pin_j), k = t's yield rank in L
//        from p.  The minimum per seed is kept in LDS (a wave per light atom, a workgroup per 4096-entry
//        chunk of a heavy atom with one global atomicMin per seed and chunk), so no global table and no
//        atomic per yield: config 2's level 1 (64 seeds, 3.6e8 items, 1.4e9 yields) touches the CSR
//        once instead of 1.4e9 random words of a 25.6 GB key array.
//        The union of the level's frontier atoms (bitmap ubit, list ulist, slot uidx) is built by the
//        expand launch; hgx_lp_efill writes each union slot's frontier row frow[u] (bit s: on seed s's
//        frontier) and item row E[u] (pre(s, p)); the count launch clears them through the union list.
// Then, both ways, the discoveries are ranked by key (hgx_lr_*, below: key buckets, an LDS bitmap per
// bucket; rank r = pair r of the level and entry r of the next frontier, vis bit set).  The level's
// pairs are seed-major because the frontier is.
constexpr int kLsG = 256;               // blocks of the range kernels (contiguous ranges: prefix-able)
constexpr int64_t kLsTile = 256;        // items per expand tile
constexpr int kLsSlots = 4;             // per-level counter slots (ring); slot words:
enum { lsF = 0, lsT = 1, lsN = 2, lsOut = 3, lsW = 4, lsTiles = 5, lsPull = 6, lsU = 7 };
constexpr int kLsSlotWords = 8;
constexpr int kLsStatus = kLsSlots * kLsSlotWords, kLsTrav = kLsStatus + 1, kLsRuns = kLsStatus + 2,
              kLsBytes = kLsStatus + 3, kLsPullN = kLsStatus + 4;
// status bits: 1 discoveries > cap, 2 runs > rcap, (4 unused since round 5), 8 tiles > tcap, 16 keys wider
// than 32 bits, 32 push hash too full, 128 a pull pass's hit list overflowed (long rows: rerun pushing)
// A level's discoveries go to kLsDSegs segments of the list, one counter each (a wave appends to the
// segment of its block): one shared counter took one same-address atomic per wave and round, which
// serialise at ~20 ns each -- the whole of a config-2 level's expand time.
// A segment holds segcap = cap / 64 entries; a wave whose segment is full appends the rest to the
// shared overflow region of cap entries (one counter) behind the segments, so a level whose
// discoveries all come from a few blocks still fits whenever they fit the capacity.
constexpr int kLsDSegs = 32;
constexpr int kLsDSeg = kLsStatus + 8;                           // [kLsSlots][kLsDSegs + 1] counters (+ overflow)
constexpr int kLsProf = kLsDSeg + kLsSlots * (kLsDSegs + 1);  // [8] pull-walk phase timers (HGX_LS_PROF)
constexpr int kLsCtlWords = kLsProf + 8;
constexpr int kLsMaxW = 16;             // row words: chunks of <= 1024 seeds
constexpr int kLrMaxBucketBits = 18;                            // <= 2^18 keys a bucket (a 32 KB LDS bitmap)
constexpr int kLrMaxBuckets = 1 << (32 - kLrMaxBucketBits);     // keys < 2^32
constexpr int kLrG = 512;                                       // blocks of count / scatter / rank
constexpr int kLrU = 4;                                         // independent loads a thread in their loops
constexpr int kLpBlk = 4096;                                    // pairs of a packed block (64 run-start words)
constexpr int kPackWords = 32;                                  // mapped words of the packed counts: [2][kLrParts] {count, seq}
constexpr int kLrParts = 8;   // scatter + rank launches a level (bucket ranges): each part's pairs are copied to the host on
                              // stream2 while the next parts rank (the host learns the parts' rank ranges from
                              // the scan's publication)

__device__ __forceinline__ int lr_bucket_bits(int64_t W, int sub) {
    const u64 keys = (u64)max<int64_t>(W, 1) * 64ull;
    const int lg = 64 - __clzll((unsigned long long)(keys - 1ull));   // ceil(log2(keys)), keys >= 64
    return min(max(lg - sub, 6), kLrMaxBucketBits);
}
__device__ __forceinline__ int lr_buckets(int64_t W, int bs) {
    return (int)(((u64)max<int64_t>(W, 1) * 64ull + (1ull << bs) - 1ull) >> bs);
}
// The rank part of bucket b: the q with q * nbk / kLrParts <= b < (q + 1) * nbk / kLrParts.
__device__ __forceinline__ int lr_part(uint32_t b, int nbk) {
    return (int)(((b + 1u) * (uint32_t)kLrParts - 1u) / (uint32_t)nbk);
}

constexpr int kLsProbes = 64;           // hash probes before a level reports overflow (load <= 1/2)
constexpr u64 kLsEmpty = ~0ull;

struct LsArgs {
    int64_t A;
    const int64_t* inc_off;
    const int32_t* inc_row;
    const int32_t* inc_type;
    const uint8_t* yf;                  // ordered-mode yield flags (null in the symmetric mode)
    const int64_t* tgt_off;
    const int32_t* tgt_idx;
    const int32_t* link_atom;
    int32_t want_type, min_arity, mode, rev, kbits;
    int64_t t_limit;                    // largest item count of a level with 32-bit keys
    int32_t lr_sub;                     // ranking buckets ~ 2^lr_sub a level (lr_bucket_bits)
    int32_t nb, W;                      // seeds of the chunk, row words
    int32_t maxd;                       // depth limit (the last level's discoveries are not expanded)
    u64* vis;                           // [A * W] examined rows (zero at the call's start)
    int64_t cap;                        // frontier / discovery / output capacity (entries)
    int64_t tcap, rcap;                 // tiles, runs
    int64_t* ctl;                       // kLsCtlWords
    int32_t* fa[2];                     // frontier atom / seed (double-buffered)
    int32_t* fs[2];
    int64_t* fbase;                     // [cap] incidence start of entry i
    int64_t* deg;                       // [cap] degree of entry i
    int64_t* pre;                       // [cap + 1] exclusive degree prefix
    int64_t* tile;                      // [tcap] first entry of each item tile
    int64_t* bsum;                      // [kLsG] block sums (entries, then bitmap words)
    int64_t* disc;                      // the level's discoveries (seed * A + atom): kLsDSegs segments of
    u64* dval;                          //   segcap entries, then an overflow region of cap entries; their
    int64_t segcap;                     //   values (push: the hash slot until hgx_ls_bits)
    uint32_t* bcnt;                     // [kLrMaxBuckets] discoveries per key bucket (hgx_lr_*; zeroed by the expand)
    uint32_t* bcur;                     // [kLrMaxBuckets] the buckets' fill cursors
    int64_t* bstart;                    // [kLrMaxBuckets + 1] their first rank
    u64* bk_v;                          // the discoveries by rank part (hgx_lr_split): value, seed * A + atom
    int64_t* bk_sa;
    uint32_t* pcnt;                     // [kLrG][kLrParts] count block's discoveries per rank part
    uint32_t* pcur;                     // [kLrParts] the parts' fill cursors
    int2* out_pair;                     // [cap] (link atom, atom) pairs, level-major (device)
    // packed transfer of large levels (n >= pack_min; hgx_lr_pflag / hgx_lr_pscan / hgx_lr_pemit): per rank
    // part its atoms, a bit per pair where the link changes (the pair starts a new link run), the links of
    // those pairs, and per 4096-pair block the number of runs before it
    int64_t pack_min;
    int32_t* patom;                     // [cap] atoms, level-major like out_pair; abytes bytes each (3 when every
    int32_t abytes;                     //   atom id fits 24 bits: a quarter less to copy than 4-byte ids)
    int32_t* pclink;                    // [cap] a part's run links from its first pair's index on
    u64* pflag;                         // [2 parities][kLrParts][pwcap] run-start bits of a part's pairs
    uint32_t* pbb;                      // [2 parities][kLrParts][pbcap] runs before each 4096-pair block
    int64_t pwcap, pbcap;
    uint32_t* seedcnt;                  // [nb] the level's discoveries per seed (hgx_lr_count; zeroed by the expand)
    int64_t* runs;                      // [rcap * 3]: (distance, seed, first pair) per seed per level
    u64* hflag;                         // mapped coherent host words: {n, status, seq, -} x 2 (level parity), then
                                        //   the rank parts' boundaries [2][kLrParts + 1]
    // the yield adjacency (yield_adj; null: the incidence): an item is one (target, link atom) pair,
    // its index the whole stream position (kbits 0)
    const int64_t* y_off;
    const int32_t* a_tgt;
    const int32_t* a_lnk;
    // push: the level hash (hcap = hmask + 1 slots; key kLsEmpty / value ~0 between levels)
    u64* hkey;
    u64* hval;
    int64_t hmask;
    // pull
    int32_t pull;                       // 0 never, 1 by the level's width, 2 every level (tests)
    int64_t I;                          // incidence entries
    const int32_t* pin_j;               // [P] index of link row L in inc(tgt_idx[p]) for pin p of L
    int32_t prof;                       // HGX_LS_PROF: the pull walk's phase timers into ctl[kLsProf ..]
    const int4* prec;                   // pull records per incidence entry (k_pull_rec), or null
    const int2* pmeta;
    u64* frow;                          // [cap * W] frontier rows of the level by union slot (zero between levels)
    u64* ubit;                          // [A / 64 + 1] union of the level's frontier atoms (zero between levels)
    int32_t* ulist;                     // [cap] the union's atoms (the rows / bits to clear after the level)
    int32_t* uidx;                      // [A] the union atom's position in ulist (valid where ubit is set)
    uint32_t* E;                        // [ecap] row u * nb + s: the item index of the first item of the frontier
    int64_t ecap;                       //   entry (seed s, atom ulist[u]) -- a pull level needs F * nb <= ecap
    int32_t hbits;                      // log2 of the push hash's size
    const HeavyChunk* chunks;           // heavy atoms' 4096-entry chunks (the graph's table)
    int64_t n_chunks, n_heavy;
    const int32_t* heavy_atom;          // [n_heavy]
    u64* hbest;                         // [n_heavy * nb] heavy atoms' minimum values (~0 between levels)
};

__device__ __forceinline__ int64_t* ls_slot(const LsArgs& a, int d) { return a.ctl + (d % kLsSlots) * kLsSlotWords; }
__device__ __forceinline__ int64_t* ls_dseg(const LsArgs& a, int d) {
    return a.ctl + kLsDSeg + (d % kLsSlots) * (kLsDSegs + 1);
}

// The level's discovery count and the segments' prefix pre[0 .. kLsDSegs] (LDS; whole block).
__device__ __forceinline__ int64_t ls_disc_prefix(const LsArgs& a, int d, int64_t* pre) {
    if (threadIdx.x < 64) {   // segment counters past their capacity spilled into the overflow region
        const int64_t ovfcap = a.cap;
        const int64_t c = threadIdx.x <= kLsDSegs ? ls_dseg(a, d)[threadIdx.x] : 0;
        const int64_t v = threadIdx.x < kLsDSegs ? min(c, a.segcap) : threadIdx.x == kLsDSegs ? min(c, ovfcap) : 0;
        int64_t x = v;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int64_t y = __shfl_up(x, off);
            if ((int)threadIdx.x >= off) x += y;
        }
        if (threadIdx.x <= kLsDSegs) pre[threadIdx.x] = x - v;
        if (threadIdx.x == kLsDSegs) pre[kLsDSegs + 1] = x;
    }
    __syncthreads();
    return pre[kLsDSegs + 1];
}

// Position of discovery x of the level (flat index over the segments, then the overflow region).
__device__ __forceinline__ int64_t ls_disc_pos(const LsArgs& a, const int64_t* pre, int64_t x) {
    int lo = 0, hi = kLsDSegs;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (pre[mid] <= x) lo = mid;
        else hi = mid - 1;
    }
    return (int64_t)lo * a.segcap + (x - pre[lo]);
}

// Appends the wave's discoveries (lanes with `isnew`: (sa, val)) to the block's segment of level d's
// list with one atomic per wave (every lane of the wave calls it).
__device__ __forceinline__ void ls_append(const LsArgs& a, int d, bool isnew, int64_t sa, u64 val) {
    const u64 m = __ballot(isnew);
    if (!m) return;
    const int lane = threadIdx.x & 63;
    const int dsg = blockIdx.x % kLsDSegs;
    int64_t* dn = ls_dseg(a, d) + dsg;
    const int leader = __ffsll((long long)m) - 1;
    const u64 cnt = (u64)__popcll(m), segcap = (u64)a.segcap;
    u64 base = 0, ob = 0;
    if (lane == leader) {
        base = atomicAdd((unsigned long long*)dn, cnt);
        const u64 fit = base >= segcap ? 0ull : min(cnt, segcap - base);
        if (fit < cnt) ob = atomicAdd((unsigned long long*)(ls_dseg(a, d) + kLsDSegs), cnt - fit);
    }
    base = __shfl(base, leader);
    ob = __shfl(ob, leader);
    if (isnew) {
        const u64 w = base + (u64)__popcll(m & ((1ull << lane) - 1ull));
        int64_t pos = -1;
        if (w < segcap) {
            pos = (int64_t)dsg * a.segcap + (int64_t)w;
        } else {   // the segment is full: the shared overflow region
            const int64_t o = (int64_t)(ob + (w - max(base, segcap)));
            if (o < a.cap) pos = (int64_t)kLsDSegs * a.segcap + o;
            else atomicOr((unsigned long long*)&a.ctl[kLsStatus], 1ull);   // more discoveries than cap holds
        }
        if (pos >= 0) {
            a.disc[pos] = sa;
            a.dval[pos] = val;
        }
    }
}

// Staged appends (the pull walk, round 5): a wave collects its discoveries in LDS and places up to
// kLsStage of them with ONE reservation -- the per-atom append (an atomic round trip on the segment
// counter for ~27 discoveries) was a tenth of the pull's time on config 2's drop-in level.
constexpr int kLsStage = 80;   // (the pull block's LDS stays under 40 KB: 4 blocks a CU)
__device__ __forceinline__ void ls_stage_flush(const LsArgs& a, int d, const int64_t* ssa, const u64* sv, int n) {
    if (n == 0) return;   // (n is wave-uniform; every lane calls)
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const int lane = threadIdx.x & 63;
    const int dsg = blockIdx.x % kLsDSegs;
    const u64 cnt = (u64)n, segcap = (u64)a.segcap;
    u64 base = 0, ob = 0;
    if (lane == 0) {
        base = atomicAdd((unsigned long long*)(ls_dseg(a, d) + dsg), cnt);
        const u64 fit = base >= segcap ? 0ull : min(cnt, segcap - base);
        if (fit < cnt) ob = atomicAdd((unsigned long long*)(ls_dseg(a, d) + kLsDSegs), cnt - fit);
    }
    base = __shfl(base, 0);
    ob = __shfl(ob, 0);
    for (int k = lane; k < n; k += 64) {
        const u64 w = base + (u64)k;
        int64_t pos = -1;
        if (w < segcap) {
            pos = (int64_t)dsg * a.segcap + (int64_t)w;
        } else {   // the segment is full: the shared overflow region
            const int64_t o = (int64_t)(ob + (w - max(base, segcap)));
            if (o < a.cap) pos = (int64_t)kLsDSegs * a.segcap + o;
            else atomicOr((unsigned long long*)&a.ctl[kLsStatus], 1ull);   // more discoveries than cap holds
        }
        if (pos >= 0) {
            a.disc[pos] = ssa[k];
            a.dval[pos] = sv[k];
        }
    }
    __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ void ls_append_staged(const LsArgs& a, int d, bool isnew, int64_t sa, u64 val, int64_t* ssa,
                                                 u64* sv, int& sn) {
    const u64 m = __ballot(isnew);
    if (!m) return;
    const int c = __popcll(m);
    if (sn + c > kLsStage) {
        ls_stage_flush(a, d, ssa, sv, sn);
        sn = 0;
    }
    if (isnew) {
        const int k = sn + __popcll(m & ((1ull << (threadIdx.x & 63)) - 1ull));
        ssa[k] = sa;
        sv[k] = val;
    }
    sn += c;
}

__device__ __forceinline__ int64_t ls_block_sum(int64_t v, int64_t* ws) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = v;
    __syncthreads();
    const int64_t t = ws[0] + ws[1] + ws[2] + ws[3];
    __syncthreads();
    return t;
}

// exclusive scan over the 256 threads of a block; *tot = the block sum
__device__ __forceinline__ int64_t ls_block_scan(int64_t v, int64_t* ws, int64_t* tot) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int64_t x = v;
    for (int off = 1; off < 64; off <<= 1) {
        const int64_t y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    if (lane == 63) ws[w] = x;
    __syncthreads();
    int64_t base = 0;
    for (int k = 0; k < w; ++k) base += ws[k];
    *tot = ws[0] + ws[1] + ws[2] + ws[3];
    __syncthreads();
    return base + x - v;
}

// exclusive prefix of bsum[0, kLsG) into LDS (every block, redundantly); returns the total
__device__ __forceinline__ int64_t ls_block_offsets(const int64_t* __restrict__ bsum, int64_t* off, int64_t* ws) {
    constexpr int per = kLsG / 256;
    int64_t v[per], s = 0;
#pragma unroll
    for (int k = 0; k < per; ++k) {
        v[k] = bsum[threadIdx.x * per + k];
        s += v[k];
    }
    int64_t tot;
    int64_t b = ls_block_scan(s, ws, &tot);
#pragma unroll
    for (int k = 0; k < per; ++k) {
        off[threadIdx.x * per + k] = b;
        b += v[k];
    }
    __syncthreads();
    return tot;
}

__device__ __forceinline__ int64_t ls_lo(int64_t n, int b) { return n * b / kLsG; }   // n < 2^53

// the block's algorithmic bytes into the call's byte counter (one atomic per block)
__device__ __forceinline__ void ls_add_bytes(const LsArgs& a, int64_t nbytes, int64_t* ws) {
    const int64_t t = ls_block_sum(nbytes, ws);
    if (threadIdx.x == 0 && t) atomicAdd((unsigned long long*)&a.ctl[kLsBytes], (unsigned long long)t);
}

__global__ void __launch_bounds__(256) hgx_ls_degree(LsArgs a, int32_t d) {
    __shared__ int64_t ws[4];
    const int64_t* sl = ls_slot(a, d);
    if (a.ctl[kLsStatus]) return;
    // this frontier = the previous level's pairs, which sit at [Out_d - F, Out_d) of the output
    const int64_t F = sl[lsF], out0 = sl[lsOut] - F;
    const int cur = d & 1;
    const int32_t* fa = a.fa[cur];
    const int64_t lo = ls_lo(F, blockIdx.x), hi = ls_lo(F, blockIdx.x + 1);
    int64_t sum = 0, trv = 0;
    (void)out0;   // (the level's runs come from hgx_lr_scan's per-seed counts)
    for (int64_t i = lo + threadIdx.x; i < hi; i += 256) {
        const int32_t p = fa[i];
        const int64_t b = a.inc_off[p], e = a.inc_off[p + 1];
        if (a.y_off) {   // items: the adjacency's pairs; the incidence entries count as traversed
            const int64_t yb = a.y_off[p], ye = a.y_off[p + 1];
            a.fbase[i] = yb;
            a.deg[i] = ye - yb;
            sum += ye - yb;
            trv += e - b;
        } else {
            a.fbase[i] = b;
            a.deg[i] = e - b;
            sum += e - b;
        }
    }
    sum = ls_block_sum(sum, ws);
    if (threadIdx.x == 0) a.bsum[blockIdx.x] = sum;
    if (a.y_off) {
        trv = ls_block_sum(trv, ws);
        if (threadIdx.x == 0 && trv) atomicAdd((unsigned long long*)&a.ctl[kLsTrav], (unsigned long long)trv);
    }
    if (blockIdx.x == 0 && threadIdx.x < kLsSlotWords && threadIdx.x != lsF && threadIdx.x != lsOut)
        a.ctl[((d + 1) % kLsSlots) * kLsSlotWords + threadIdx.x] = 0;   // the next level's slot counters
    if (blockIdx.x == 0 && threadIdx.x <= kLsDSegs) ls_dseg(a, d + 1)[threadIdx.x] = 0;
}

__global__ void __launch_bounds__(256) hgx_ls_prefix(LsArgs a, int32_t d) {
    __shared__ int64_t ws[4], off[kLsG];
    int64_t* sl = ls_slot(a, d);
    if (a.ctl[kLsStatus]) return;
    const int64_t F = sl[lsF];
    const int64_t T = ls_block_offsets(a.bsum, off, ws);
    const int64_t lo = ls_lo(F, blockIdx.x), hi = ls_lo(F, blockIdx.x + 1);
    // contiguous pieces per thread: local sums, block scan, then the prefix written in order
    const int64_t piece = (hi - lo + 255) / 256, p0 = lo + threadIdx.x * piece, p1 = min(hi, p0 + piece);
    int64_t s = 0;
    for (int64_t i = p0; i < p1; ++i) s += a.deg[i];
    int64_t tot;
    int64_t run = off[blockIdx.x] + ls_block_scan(s, ws, &tot);
    for (int64_t i = p0; i < p1; ++i) {
        const int64_t dg = a.deg[i];
        a.pre[i] = run;
        // the tiles whose first item lies in this entry's items
        for (int64_t k = (run + kLsTile - 1) / kLsTile; k * kLsTile < run + dg; ++k)
            if (k < a.tcap) a.tile[k] = i;
        run += dg;
    }
    if (blockIdx.x == kLsG - 1 && threadIdx.x == 0) {
        a.pre[F] = T;
        sl[lsT] = T;
        const int64_t W = (int64_t)((((u64)T << a.kbits) + 63ull) >> 6);
        sl[lsW] = W;
        sl[lsTiles] = (T + kLsTile - 1) / kLsTile;
        // pull when the level's items are a large part of the incidence (a pull reads all of it)
        sl[lsPull] = (a.pull == 2 || (a.pull == 1 && T * 8 > a.I)) && F * (int64_t)a.nb <= a.ecap ? 1 : 0;
        if (sl[lsPull]) atomicAdd((unsigned long long*)&a.ctl[kLsPullN], 1ull);
        if (!a.y_off) atomicAdd((unsigned long long*)&a.ctl[kLsTrav], (unsigned long long)T);
        int64_t st = 0;
        if (T > a.t_limit) st |= 16;   // keys wider than 32 bits: the chunk is split (or the key-array engine)
        if (sl[lsTiles] > a.tcap) st |= 8;
        if (st) atomicOr((unsigned long long*)&a.ctl[kLsStatus], (unsigned long long)st);
    }
}

// last index i in [lo, hi] with pre[i] <= x
__device__ __forceinline__ int64_t ls_search(const int64_t* __restrict__ pre, int64_t lo, int64_t hi, int64_t x) {
    while (lo < hi) {
        const int64_t mid = (lo + hi + 1) >> 1;
        if (pre[mid] <= x) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

__device__ __forceinline__ u64 ls_hash(u64 key, int bits) { return (key * 0x9E3779B97F4A7C15ull) >> (64 - bits); }

// The push level's hash: lowers the value of (seed, atom) `sa` to v; true (and *slot) when this call
// claimed the slot, i.e. discovered the atom for the seed at this level.  Keys only ever go from empty to
// sa inside a level, so a stale plain read of a key can only say "empty" (the CAS then tells the truth),
// and a stale value is larger than the current one (only an extra atomicMin).
__device__ __forceinline__ bool ls_hash_min(const LsArgs& a, int64_t sa, u64 v, int64_t* slot) {
    u64 h = ls_hash((u64)sa, a.hbits);
    for (int probe = 0; probe < kLsProbes; ++probe) {
        u64 k = a.hkey[h];
        if (k == kLsEmpty) {
            k = atomicCAS((unsigned long long*)&a.hkey[h], kLsEmpty, (unsigned long long)sa);
            if (k == kLsEmpty) {
                atomicMin((unsigned long long*)&a.hval[h], (unsigned long long)v);
                *slot = (int64_t)h;
                return true;
            }
        }
        if (k == (u64)sa) {
            if (a.hval[h] > v) atomicMin((unsigned long long*)&a.hval[h], (unsigned long long)v);
            return false;
        }
        h = (h + 1) & (u64)a.hmask;
    }
    atomicOr((unsigned long long*)&a.ctl[kLsStatus], 32ull);   // the table is too full: grow and rerun
    return false;
}

// Push levels: one incidence item (entry i, link index j) per lane, 256-item tiles (a short search
// inside the tile's entry range).  Pull levels: this launch builds the frontier rows, the union and
// the (seed, atom) -> pre hash from the frontier entries instead.  Both zero the level's rank bitmap.
__global__ void __launch_bounds__(256) hgx_ls_expand(LsArgs a, int32_t d) {
    __shared__ int64_t ws[4];
    int64_t* sl = ls_slot(a, d);
    if (a.ctl[kLsStatus]) return;
    const int64_t F = sl[lsF], T = sl[lsT], W = sl[lsW], nt = sl[lsTiles];
    const int cur = d & 1;
    const int32_t* fa = a.fa[cur];
    const int32_t* fs = a.fs[cur];
    {   // the ranking's bucket counts (hgx_lr_count adds to them)
        const int bs = lr_bucket_bits(W, a.lr_sub), nbk = lr_buckets(W, bs);
        for (int64_t b = blockIdx.x * 256ll + threadIdx.x; b < nbk; b += (int64_t)gridDim.x * 256) a.bcnt[b] = 0u;
        for (int64_t q = blockIdx.x * 256ll + threadIdx.x; q < a.nb; q += (int64_t)gridDim.x * 256) a.seedcnt[q] = 0u;
    }
    const int lane = threadIdx.x & 63;
    int64_t nbytes = 0;
    if (sl[lsPull]) {
        // the union of the frontier atoms (bitmap, list, slot of each); entries in a wave-uniform loop
        // (the union append ballots); hgx_lp_efill then builds the rows by union slot
        for (int64_t i0 = (int64_t)blockIdx.x * 256; i0 < F; i0 += (int64_t)gridDim.x * 256) {
            const int64_t i = i0 + threadIdx.x;
            bool first = false;
            int32_t p = 0;
            if (i < F) {
                p = fa[i];
                const u64 bit = 1ull << (p & 63);
                first = !(atomicOr((unsigned long long*)&a.ubit[p >> 6], bit) & bit);
                nbytes += 8 + 8;
            }
            const u64 m = __ballot(first);
            if (m) {
                const int leader = __ffsll((long long)m) - 1;
                u64 base = 0;
                if (lane == leader) base = atomicAdd((unsigned long long*)&sl[lsU], (unsigned long long)__popcll(m));
                base = __shfl(base, leader);
                if (first) {   // base + rank < F <= cap
                    const int64_t u = (int64_t)base + __popcll(m & ((1ull << lane) - 1ull));
                    a.ulist[u] = p;
                    a.uidx[p] = (int32_t)u;
                }
            }
        }
        ls_add_bytes(a, nbytes, ws);
        return;
    }
    for (int64_t k = blockIdx.x; k < nt; k += gridDim.x) {
        const int64_t e0 = a.tile[k], e1 = k + 1 < nt ? a.tile[k + 1] : F - 1;
        const int64_t it = k * kLsTile + threadIdx.x;
        bool live = it < T;
        int64_t i = 0, j = 0, ii = 0;
        int32_t p = -1, n = 0, la = 0, lo = 0, hi = 0, s = 0;
        int64_t b = 0;
        if (live) {
            i = ls_search(a.pre, e0, e1, it);
            j = it - a.pre[i];
            p = fa[i];
            s = fs[i];
            ii = a.fbase[i] + j;
            nbytes += 24;
            if (!a.a_tgt && a.yf) {
                nbytes += 1;
                if (!((a.yf[ii] >> a.mode) & 1u)) live = false;     // nothing to yield
            }
        }
        int32_t t_adj = 0;
        if (live && a.a_tgt) {   // the generator's output itself: one yield, rank 0
            t_adj = a.a_tgt[ii];
            la = a.a_lnk[ii];
            n = 1;
            hi = 1;
            nbytes += 8;
        } else if (live) {
            const int32_t L = a.inc_row[ii];
            const int32_t ty = a.want_type >= 0 ? a.inc_type[ii] : 0;
            if (a.want_type >= 0 && ty != a.want_type) live = false;             // linkPredicate (:300)
            b = a.tgt_off[L];
            n = (int32_t)(a.tgt_off[L + 1] - b);
            la = a.link_atom[L];
            if (n < a.min_arity) live = false;                                    // minArity (:309)
            nbytes += (a.want_type >= 0 ? 8 : 4) + 20 + 4 * (int64_t)n;
        }
        if (live && !a.a_tgt) {
            hi = n;
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
        }
        const int32_t cnt = live && hi > lo ? hi - lo : 0;
        int32_t rounds = cnt;
        for (int off = 32; off > 0; off >>= 1) rounds = max(rounds, __shfl_xor(rounds, off));
        const int64_t sA = live ? (int64_t)s * a.A : 0;
        const u64 kb = ((u64)it << a.kbits) + 1ull;
        for (int32_t r = 0; r < rounds; ++r) {   // wave-uniform rounds: one append atomic per wave and round
            bool isnew = false;
            int32_t t = 0;
            int64_t slot = 0;
            if (r < cnt) {
                const int32_t q = lo + r;
                t = a.a_tgt ? t_adj : a.tgt_idx[b + q];
                if (t != p) {
                    nbytes += 8;   // the examined word
                    if (!((a.vis[(int64_t)t * a.W + (s >> 6)] >> (s & 63)) & 1ull)) {
                        const u64 rk = a.a_tgt ? 0ull : (u64)(a.rev ? n - 1 - q : q);
                        const u64 v = ((kb + rk) << 32) | (u64)(uint32_t)la;
                        isnew = ls_hash_min(a, sA + t, v, &slot);
                        nbytes += 16;
                    }
                }
            }
            ls_append(a, d, isnew, sA + t, (u64)slot);
        }
    }
    ls_add_bytes(a, nbytes, ws);
}

// Pull levels, after the expand launch built the union: E[u * nb + s] = the item index of the first
// item of seed s's frontier entry of p (u = p's union slot), and bit s of the frontier row frow[u].
__global__ void __launch_bounds__(256) hgx_lp_efill(LsArgs a, int32_t d) {
    const int64_t* sl = ls_slot(a, d);
    if (a.ctl[kLsStatus] || !sl[lsPull]) return;
    const int64_t F = sl[lsF];
    const int32_t* fa = a.fa[d & 1];
    const int32_t* fs = a.fs[d & 1];
    for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < F; i += (int64_t)gridDim.x * 256) {
        const int64_t u = a.uidx[fa[i]];
        const int32_t s = fs[i];
        a.E[u * a.nb + s] = (uint32_t)a.pre[i];
        atomicOr((unsigned long long*)&a.frow[u * a.W + (s >> 6)], 1ull << (s & 63));
    }
}

// A pull hit: co-target p (union slot u) of link L yields atom t (the walk's atom o) at rank kq with
// item offset j; la = the link's atom id (the value's low word).
struct LpHit {
    int32_t u;       // the co-target's union slot (its frontier row frow[u] and item row E[u])
    uint32_t j;
    int32_t la;
    uint32_t kq_o;   // kq | o << 16
};
constexpr int kLpHits = 64 * 8;   // one pass of a wave: <= 64 entries of <= 8 targets (<= 7 hits each)

// The hits of entry e of atom t (a lane's share of a pass): every co-target p of e's link that is on
// some seed's frontier and yields t -- the expand's rules: link predicate, minimum arity, p's first
// occurrence, the mode's positions (3.2), t's best yielded position.  Rows of <= 8 targets: a mask of
// the hit positions over the row in registers; longer rows set long_row (walked by lp_long_row).
struct LpCand {
    int32_t tg[8], pj[8];   // pj: the hits' pin indices
    uint32_t qt;            // t's best yielded position for co-target q: 4 bits each
    uint32_t mask;
    int64_t tb;
    int32_t rown, la;
};
__device__ __forceinline__ int lp_hits_count(const LsArgs& a, int32_t t, int64_t e, bool have, LpCand& c, bool& long_row,
                                             int64_t& nbytes) {
    c.mask = 0u;
    c.tb = 0;
    c.rown = 0;
    c.la = 0;
    long_row = false;
    if (!have) return 0;
    int32_t n;
    if (a.pmeta) {   // the entry's pull record: (link atom, arity), <= 8 targets, their pin indices -- streamed
        // in entry order and loaded together with the type (one round trip before the union probes)
        // (nontemporal loads of the records measured no faster: 119 vs 116 ms a config-2 drop-in call)
        const int32_t ty = a.want_type >= 0 ? a.inc_type[e] : 0;
        const int2 m = a.pmeta[e];
        const int4 r0 = a.prec[4 * e], r1 = a.prec[4 * e + 1], r2 = a.prec[4 * e + 2], r3 = a.prec[4 * e + 3];
        if (a.want_type >= 0 && ty != a.want_type) {   // linkPredicate (:300)
            nbytes += 4;
            return 0;
        }
        n = m.y;
        nbytes += (a.want_type >= 0 ? 4 : 0) + 8;
        if (n < a.min_arity) return 0;   // minArity (:309)
        c.rown = n;
        c.la = m.x;
        if (n > 8) {
            const int32_t L = a.inc_row[e];
            c.tb = a.tgt_off[L];
            nbytes += 12 + 4 * (int64_t)n + 4 * (int64_t)n;
            long_row = true;
            return 0;
        }
        c.tg[0] = r0.x; c.tg[1] = r0.y; c.tg[2] = r0.z; c.tg[3] = r0.w;
        c.tg[4] = r1.x; c.tg[5] = r1.y; c.tg[6] = r1.z; c.tg[7] = r1.w;
        c.pj[0] = r2.x; c.pj[1] = r2.y; c.pj[2] = r2.z; c.pj[3] = r2.w;
        c.pj[4] = r3.x; c.pj[5] = r3.y; c.pj[6] = r3.z; c.pj[7] = r3.w;
        nbytes += 64 + 8 * (int64_t)n;   // the record, the targets' union words
    } else {
        if (a.want_type >= 0 && a.inc_type[e] != a.want_type) {   // linkPredicate (:300)
            nbytes += 4;
            return 0;
        }
        const int32_t L = a.inc_row[e];
        const int64_t tb = a.tgt_off[L];
        n = (int32_t)(a.tgt_off[L + 1] - tb);
        nbytes += (a.want_type >= 0 ? 8 : 4) + 16;
        if (n < a.min_arity) return 0;   // minArity (:309)
        nbytes += 4 * (int64_t)n + 4 + 8 * (int64_t)n;
        c.tb = tb;
        c.rown = n;
        c.la = a.link_atom[L];
        if (n > 8) {
            long_row = true;
            return 0;
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) c.tg[q] = q < n ? a.tgt_idx[tb + q] : -1;
    }
    uint32_t onf[8];   // union bits of the co-targets, loaded together (32-bit words: fewer registers in flight)
    const uint32_t* ub = (const uint32_t*)a.ubit;
#pragma unroll
    for (int q = 0; q < 8; ++q) onf[q] = (q < n && c.tg[q] != t) ? ub[c.tg[q] >> 5] >> (c.tg[q] & 31) : 0u;
    c.qt = 0u;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        if (!(onf[q] & 1u)) continue;   // on no seed's frontier (or t itself, or past the row)
        const int32_t p = c.tg[q];
        bool dup = false;   // p's first occurrence only
#pragma unroll
        for (int q2 = 0; q2 < q; ++q2) dup |= c.tg[q2] == p;
        if (dup) continue;
        int32_t lp = q;
#pragma unroll
        for (int q2 = q + 1; q2 < 8; ++q2)
            if (c.tg[q2] == p) lp = q2;
        int32_t lo = 0, hi = n;   // positions p yields (3.2)
        if (a.mode == sAfterFirst) lo = q + 1;
        else if (a.mode == sBeforeFirst) hi = q;
        else if (a.mode == sBeforeLast) hi = lp;
        else if (a.mode == sAfterLast) lo = lp + 1;
        int32_t qt = -1;   // t's best yielded position
#pragma unroll
        for (int q2 = 0; q2 < 8; ++q2)
            if (q2 >= lo && q2 < hi && c.tg[q2] == t && (qt < 0 || a.rev)) qt = q2;
        if (qt >= 0) {
            c.qt |= (uint32_t)qt << (4 * q);
            c.mask |= 1u << q;
        }
    }
    if (!a.pmeta && c.mask) {   // the hits' pin indices at random (no pull records)
#pragma unroll
        for (int q = 0; q < 8; ++q) c.pj[q] = ((c.mask >> q) & 1u) ? a.pin_j[c.tb + q] : 0;
    }
    return __popc(c.mask);
}

// Walks a long row (> 8 targets) of atom t: f(p, q, qt) for every hit (from memory).
template <class F>
__device__ __forceinline__ void lp_long_row(const LsArgs& a, int32_t t, int64_t tb, int32_t n, F&& f) {
    for (int32_t q = 0; q < n; ++q) {
        const int32_t p = a.tgt_idx[tb + q];
        if (p == t || !((a.ubit[p >> 6] >> (p & 63)) & 1ull)) continue;
        bool dup = false;
        for (int32_t q2 = 0; q2 < q; ++q2) dup |= a.tgt_idx[tb + q2] == p;
        if (dup) continue;
        int32_t lp = q;
        for (int32_t q2 = q + 1; q2 < n; ++q2)
            if (a.tgt_idx[tb + q2] == p) lp = q2;
        int32_t lo = 0, hi = n;
        if (a.mode == sAfterFirst) lo = q + 1;
        else if (a.mode == sBeforeFirst) hi = q;
        else if (a.mode == sBeforeLast) hi = lp;
        else if (a.mode == sAfterLast) lo = lp + 1;
        int32_t qt = -1;
        for (int32_t q2 = lo; q2 < hi; ++q2)
            if (a.tgt_idx[tb + q2] == t && (qt < 0 || a.rev)) qt = q2;
        if (qt >= 0) f(p, q, qt);
    }
}

// Wave timers of the pull (HGX_LS_PROF, s_memrealtime ticks of 10 ns, summed over waves): phase A,
// phase B, flushes, then passes, phase-B steps, flushes, heavy-chunk time, kernel time.
struct LpProf {
    int64_t v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
};

// The k-th set bit (k < popcount) of w.
__device__ __forceinline__ int lp_select_bit(u64 w, int k) {
    int pos = 0;
#pragma unroll
    for (int sh = 32; sh > 0; sh >>= 1) {
        const u64 lo = w & ((1ull << sh) - 1ull);
        const int c = __popcll(lo);
        if (k >= c) {
            k -= c;
            w >>= sh;
            pos += sh;
        } else {
            w = lo;
        }
    }
    return pos;
}

// Phase B of the pull walk for <= 64 seeds (round 6): a lane per (hit, seed) candidate
// for the loads.  The lane-per-seed steps (HB = 8 hits of one atom, a frontier-row word and a 256-byte item
// row each) took one dependent round trip per 8 hits with most lanes idle (a hit yields ~7 candidate seeds
// of 64 on config 2's drop-in level).  Here the wave loads the frontier rows of 64 hits at once (a lane per
// hit), masks them with the hit atom's unexamined seeds, flattens the set bits into candidates (wave
// prefix; a candidate finds its hit by binary search over the prefix and its seed by bit selection) and
// loads the item offsets E[u * nb + s] of kLpCB x 64 candidates at once (4 bytes each instead of whole
// rows).  The minima stay lane-per-seed (best, flushed per atom as before): a batch's candidates are in
// hit order, so one atom's are consecutive; per atom segment of a chunk the candidates lower the wave's LDS
// row brow[s] (ds atomicMin), then lane s folds brow[s] into best and clears it.
constexpr int kLpCB = 4;   // candidate chunks of 64 whose loads are in flight together
template <class FlushCur>
__device__ __forceinline__ void lp_phase_b1(const LsArgs& a, const LpHit* hits, int total, u64 vw0, u64 lastmask,
                                            int& cur, u64* best, u64* brow, int64_t& nbytes, FlushCur&& flush_cur) {
    const int lane = threadIdx.x & 63;
    for (int g0 = 0; g0 < total; g0 += 64) {   // hits a lane each (wave-uniform)
        const int h = g0 + lane;
        LpHit hq = {0, 0u, 0, 0u};
        if (h < total) hq = hits[h];
        // (every lane shuffles: a lane shuffle reads 0 from a source lane that is inactive at the call)
        const u64 need = ~__shfl(vw0, (int)(hq.kq_o >> 16)) & lastmask;   // the seeds that have not examined the hit's atom
        u64 fw = 0ull;
        if (h < total) fw = a.frow[(int64_t)hq.u] & need;                 // (W == 1: one word a union slot)
        const int nc = __popcll(fw);
        int px = nc;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int y = __shfl_up(px, off);
            if (lane >= off) px += y;
        }
        const int ncand = __shfl(px, 63), exc = px - nc;
        nbytes += h < total ? 8 : 0;
        for (int c0 = 0; c0 < ncand; c0 += 64 * kLpCB) {   // kLpCB chunks of candidates, a lane each (wave-uniform)
            u64 v[kLpCB];
            int sd[kLpCB], od[kLpCB];
#pragma unroll
            for (int q = 0; q < kLpCB; ++q) {
                const int c = c0 + q * 64 + lane;
                int hl = 0;   // the candidate's hit lane: the last lane whose candidates start at or before c
#pragma unroll
                for (int step = 32; step > 0; step >>= 1) {
                    const int mid = hl + step;
                    if (__shfl(exc, mid) <= c) hl = mid;
                }
                const u64 fwh = __shfl(fw, hl);
                const int32_t u = __shfl(hq.u, hl);
                const uint32_t j = __shfl(hq.j, hl);
                const int32_t la = __shfl(hq.la, hl);
                const uint32_t kq_o = __shfl(hq.kq_o, hl);
                const int exh = __shfl(exc, hl);
                const bool live = c < ncand;
                sd[q] = live ? lp_select_bit(fwh, c - exh) : 0;
                od[q] = (int)(kq_o >> 16);
                v[q] = ~0ull;
                if (live) {
                    const uint32_t pre = a.E[(int64_t)u * a.nb + sd[q]];
                    v[q] = ((((((u64)pre + j) << a.kbits) | (kq_o & 0xFFFFu)) + 1ull) << 32) | (u64)(uint32_t)la;
                    nbytes += 4;
                }
            }
#pragma unroll
            for (int q = 0; q < kLpCB; ++q) {
                const int m = min(64, ncand - c0 - q * 64);   // live lanes of chunk q (wave-uniform)
                if (m <= 0) break;
                for (int k = 0; k < m;) {   // the chunk's atom segments, in order (wave-uniform)
                    const int ok = __builtin_amdgcn_readlane(od[q], k);
                    const u64 seg = __ballot(lane >= k && lane < m && od[q] == ok);
                    if (ok != cur) {   // the candidates moved on to the next atom: flush the finished one
                        if (cur >= 0) flush_cur();
                        cur = ok;
                    }
                    if ((seg >> lane) & 1ull) atomicMin((unsigned long long*)&brow[sd[q]], (unsigned long long)v[q]);
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    if (lane < a.nb) {   // (the wave's row holds nb seeds)
                        best[0] = min(best[0], brow[lane]);
                        brow[lane] = ~0ull;
                    }
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    k = 64 - __clzll((unsigned long long)seg);   // past the segment's last lane
                }
            }
        }
    }
}

// The pull walk of one wave over the concatenated incidence ranges of up to 64 atoms (lane o: atom
// at, entries [eb, eb + cnt), examined words vw[]): 64 entries a pass.  Phase A, a lane per entry:
// its hits, written into the wave's LDS list in entry order (so each atom's hits are contiguous).
// Phase B, a lane per seed (seed w * 64 + lane keeps its minimum in register best[w]): the hits in
// order, up to HB of one atom at a time (their frontier-row words and E rows -- one broadcast and one
// coalesced load each -- all in flight together); when the hits move on to the next atom the finished
// one is flushed -- flush(o, best), every lane calls it -- and best reset.  A hit's co-target is on
// ~1.1 seeds' frontiers on average but the power-law hubs on 10-26 (config 2's drop-in level: 238M hits,
// 1.7e9 (hit, seed) candidates), so the seeds stay on the lanes; HB = 16 / WW hits a step keeps the
// wave's loads in flight (4 a step: 87 ms for that level, latency-bound at ~4 us a step).
template <int WW, class Flush>
__device__ __forceinline__ void lp_walk(const LsArgs& a, int32_t at, int64_t eb, int64_t cnt, const u64* vw, LpHit* hits, u64* brow,
                                        u64* best, int64_t& nbytes, LpProf& pf, Flush&& flush) {
    constexpr int HB = WW >= 4 ? 2 : 8 / WW;
    const int lane = threadIdx.x & 63;
    int64_t x = cnt;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int64_t y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    const int64_t T = __shfl(x, 63), ex = x - cnt;
    const u64 lastmask = (a.nb & 63) ? (1ull << (a.nb & 63)) - 1ull : ~0ull;
    int cur = -1;   // the atom (lane) whose minima best[] holds (wave-uniform)
    u64 needb[WW];  // the current atom's examined words, inverted (seeds that have not examined it)
#pragma unroll
    for (int w = 0; w < WW; ++w) needb[w] = 0ull;
    auto flush_cur = [&]() {   // every lane
        const int64_t t0 = a.prof ? (int64_t)wall_clock64() : 0;
        flush(cur, best);
#pragma unroll
        for (int w = 0; w < WW; ++w) best[w] = ~0ull;
        if (a.prof) {
            pf.v[2] += (int64_t)wall_clock64() - t0;
            pf.v[5] += 1;
        }
    };
    for (int64_t f0 = 0; f0 < T; f0 += 64) {   // wave-uniform
        const int64_t f = f0 + lane;
        int o = 0;   // owner lane: the last lane whose range starts at or before f
#pragma unroll
        for (int step = 32; step > 0; step >>= 1) {
            const int mid = o + step;
            if (__shfl(ex, mid) <= f) o = mid;
        }
        const int32_t t = __shfl(at, o);
        const int64_t e = __shfl(eb, o) + (f - __shfl(ex, o));
        const int64_t ta = a.prof ? (int64_t)wall_clock64() : 0;
        LpCand c;
        bool lr;
        const int nh = lp_hits_count(a, t, e, f < T, c, lr, nbytes);
        int nl = 0;   // a long row's hits, counted first
        if (lr) lp_long_row(a, t, c.tb, c.rown, [&](int32_t, int32_t, int32_t) { ++nl; });
        const int mine = nh + nl;
        int px = mine;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int y = __shfl_up(px, off);
            if (lane >= off) px += y;
        }
        const int total = __shfl(px, 63);
        if (total > kLpHits) {   // only long rows can fill the list: the chunk reruns pushing
            if (lane == 0) atomicOr((unsigned long long*)&a.ctl[kLsStatus], 128ull);
            return;
        }
        int pos = px - mine;
        int32_t us[8];   // the hits' union slots, loaded together
#pragma unroll
        for (int q = 0; q < 8; ++q) us[q] = ((c.mask >> q) & 1u) ? a.uidx[c.tg[q]] : 0;
#pragma unroll
        for (int q = 0; q < 8; ++q)
            if ((c.mask >> q) & 1u) {
                LpHit h;
                h.u = us[q];
                h.j = (uint32_t)c.pj[q];
                h.la = c.la;
                const int32_t qt = (int32_t)((c.qt >> (4 * q)) & 15u);
                h.kq_o = (uint32_t)(a.rev ? c.rown - 1 - qt : qt) | (uint32_t)o << 16;
                hits[pos++] = h;
            }
        if (lr)
            lp_long_row(a, t, c.tb, c.rown, [&](int32_t p, int32_t q, int32_t qt) {
                LpHit h;
                h.u = a.uidx[p];
                h.j = (uint32_t)a.pin_j[c.tb + q];
                h.la = c.la;
                h.kq_o = (uint32_t)(a.rev ? c.rown - 1 - qt : qt) | (uint32_t)o << 16;
                hits[pos++] = h;
            });
        nbytes += 4 * (int64_t)mine;   // the union slots
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        const int64_t tb_ = a.prof ? (int64_t)wall_clock64() : 0;
        if (a.prof) {
            pf.v[0] += tb_ - ta;
            pf.v[3] += 1;
        }
        if constexpr (WW == 1) {   // phase B over (hit, seed) candidates (<= 64 seeds: one row word)
            lp_phase_b1(a, hits, total, vw[0], lastmask, cur, best, brow, nbytes, flush_cur);
        } else
        for (int h0 = 0; h0 < total;) {   // phase B (wave-uniform)
            // only the union slots stay in registers while the rows load (the other fields are read
            // from LDS again after): 2 waves/SIMD at 235 VGPRs with whole hits held
            int32_t hu[HB];
            const int ho = (int)(hits[h0].kq_o >> 16);
            int hn = 1;   // up to HB consecutive hits of the same atom
#pragma unroll
            for (int q = 0; q < HB; ++q) {
                const LpHit hq = hits[min(h0 + q, total - 1)];
                hu[q] = hq.u;
                if (q > 0 && hn == q && h0 + q < total && (int)(hq.kq_o >> 16) == ho) ++hn;
            }
            if (ho != cur) {   // the hits moved on to the next atom: flush the finished one
                if (cur >= 0) flush_cur();
                cur = ho;
#pragma unroll
                for (int w = 0; w < WW; ++w) {
                    const u64 v = w < a.W ? ~__shfl(vw[w], cur) : 0ull;
                    needb[w] = w == a.W - 1 ? v & lastmask : v;
                }
            }
            u64 fw[HB][WW];
            uint32_t pre[HB][WW];
#pragma unroll
            for (int q = 0; q < HB; ++q)
#pragma unroll
                for (int w = 0; w < WW; ++w) {
                    fw[q][w] = 0ull;
                    pre[q][w] = 0u;
                    if (q < hn && w < a.W) {
                        fw[q][w] = a.frow[(int64_t)hu[q] * a.W + w];
                        if (w * 64 + lane < a.nb) pre[q][w] = a.E[(int64_t)hu[q] * a.nb + w * 64 + lane];
                    }
                }
#pragma unroll
            for (int q = 0; q < HB; ++q) {
                if (q >= hn) break;
                const LpHit hq = hits[h0 + q];
#pragma unroll
                for (int w = 0; w < WW; ++w) {
                    if (w >= a.W || !(((fw[q][w] & needb[w]) >> lane) & 1ull)) continue;
                    const u64 it = (u64)pre[q][w] + hq.j;
                    const u64 v = ((((it << a.kbits) | (hq.kq_o & 0xFFFFu)) + 1ull) << 32) | (u64)(uint32_t)hq.la;
                    best[w] = min(best[w], v);
                }
            }
            nbytes += lane == 0 ? (int64_t)hn * (8 * a.W + 4 * (int64_t)a.nb) : 0;
            h0 += hn;
            if (a.prof) pf.v[4] += 1;
        }
        if (a.prof) pf.v[1] += (int64_t)wall_clock64() - tb_;
        __builtin_amdgcn_wave_barrier();
    }
    if (cur >= 0) flush_cur();
}

// Pull levels: heavy atoms by 4096-entry chunks (a workgroup each, its four waves walking a quarter
// each; their minima merged through LDS and lowered into hbest with one global atomicMin per seed),
// then the light atoms: a wave takes 64 consecutive atoms (a lane each: incidence range, examined row)
// and walks the entries of those with incidence, <= kHeavyDegree entries and a seed that has not
// examined them; each atom's discoveries are appended when the walk leaves it.  WW: the row words
// rounded up to a power of two (register minima).
template <int WW>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) hgx_lp_pull(LsArgs a, int32_t d) {
    extern __shared__ u64 lp_merge[];   // [4][nb]
    __shared__ LpHit lp_hits_l[4][kLpHits];
    __shared__ int64_t lp_ssa[4][kLsStage];   // each wave's staged discoveries
    __shared__ u64 lp_sv[4][kLsStage];
    __shared__ int64_t ws[4];
    const int64_t* sl = ls_slot(a, d);
    if (a.ctl[kLsStatus] || !sl[lsPull]) return;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int nb = a.nb, W = a.W;
    LpHit* hits = lp_hits_l[wave];
    for (int s = threadIdx.x; s < 4 * nb; s += 256) lp_merge[s] = ~0ull;
    int64_t* ssa = lp_ssa[wave];
    u64* sv = lp_sv[wave];
    int sn = 0;   // staged discoveries of this wave (wave-uniform)
    LpProf pf;
    const int64_t tk0 = a.prof ? (int64_t)wall_clock64() : 0;
    __syncthreads();
    u64 best[WW];
#pragma unroll
    for (int w = 0; w < WW; ++w) best[w] = ~0ull;
    int64_t nbytes = 0;
    // heavy chunks
    for (int64_t c = blockIdx.x; c < a.n_chunks; c += gridDim.x) {   // block-uniform
        const HeavyChunk ch = a.chunks[c];
        const int32_t t = ch.atom;
        u64 vw[WW];
#pragma unroll
        for (int w = 0; w < WW; ++w) vw[w] = w < W ? a.vis[(int64_t)t * W + w] : 0ull;
        nbytes += lane == 0 ? 24 + 8 * W : 0;
        const int64_t q = (ch.end - ch.beg + 3) / 4;
        const int64_t b = ch.beg + wave * q, e = min(ch.end, b + q);
        // one "atom" on lane 0: this wave's quarter of the chunk
        lp_walk<WW>(a, t, lane == 0 ? b : 0, lane == 0 ? max<int64_t>(e - b, 0) : 0, vw, hits, lp_merge + (int64_t)wave * nb, best, nbytes, pf,
                    [&](int, u64* bst) {
#pragma unroll
                        for (int w = 0; w < WW; ++w)
                            if (w < W && w * 64 + lane < nb) lp_merge[(int64_t)wave * nb + w * 64 + lane] = bst[w];
                    });
        __syncthreads();
        for (int s = threadIdx.x; s < nb; s += 256) {   // the four waves' minima -> the heavy atom's row
            u64 v = ~0ull;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                v = min(v, lp_merge[(int64_t)k * nb + s]);
                lp_merge[(int64_t)k * nb + s] = ~0ull;
            }
            if (v != ~0ull) {
                atomicMin((unsigned long long*)&a.hbest[(int64_t)ch.slot * nb + s], (unsigned long long)v);
                nbytes += 8;
            }
        }
        __syncthreads();
    }
    if (a.prof) pf.v[6] += (int64_t)wall_clock64() - tk0;
    // light atoms
    const int64_t nwv = (int64_t)gridDim.x * 4;
    for (int64_t t0 = ((int64_t)blockIdx.x * 4 + wave) * 64; t0 < a.A; t0 += nwv * 64) {
        const int64_t t = t0 + lane;
        int64_t eb = 0, cnt = 0;
        u64 vw[WW];
#pragma unroll
        for (int w = 0; w < WW; ++w) vw[w] = ~0ull;
        const u64 lastmask = (nb & 63) ? (1ull << (nb & 63)) - 1ull : ~0ull;
        if (t < a.A) {
            eb = a.inc_off[t];
            const int64_t ee = a.inc_off[t + 1];
            nbytes += 8;
            if (ee > eb && ee - eb <= kHeavyDegree) {
                u64 any = 0;
#pragma unroll
                for (int w = 0; w < WW; ++w) {
                    vw[w] = w < W ? a.vis[t * W + w] : ~0ull;
                    if (w < W) any |= w == W - 1 ? ~vw[w] & lastmask : ~vw[w];
                }
                nbytes += 8 * W;
                if (any) cnt = ee - eb;
            }
        }
        lp_walk<WW>(a, (int32_t)t, eb, cnt, vw, hits, lp_merge + (int64_t)wave * nb, best, nbytes, pf, [&](int o, u64* bst) {
#pragma unroll
            for (int w = 0; w < WW; ++w) {   // the atom's discoveries: a lane per seed
                if (w >= W) break;
                const int s = w * 64 + lane;
                ls_append_staged(a, d, s < nb && bst[w] != ~0ull, (int64_t)s * a.A + (t0 + o), bst[w], ssa, sv, sn);
            }
        });
    }
    ls_stage_flush(a, d, ssa, sv, sn);
    if (a.prof) {
        pf.v[7] += (int64_t)wall_clock64() - tk0;
        if (lane == 0)
            for (int k = 0; k < 8; ++k)
                if (pf.v[k]) atomicAdd((unsigned long long*)&a.ctl[kLsProf + k], (unsigned long long)pf.v[k]);
    }
    ls_add_bytes(a, nbytes, ws);
}

// Pull levels: the heavy atoms' rows -> their discoveries (a wave per heavy atom, a lane per seed); the
// rows go back to ~0.
__global__ void __launch_bounds__(256) hgx_lp_hfinal(LsArgs a, int32_t d) {
    const int64_t* sl = ls_slot(a, d);
    if (a.ctl[kLsStatus] || !sl[lsPull]) return;
    const int lane = threadIdx.x & 63;
    const int64_t nwv = (int64_t)gridDim.x * 4;
    for (int64_t h = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); h < a.n_heavy; h += nwv) {
        const int32_t t = a.heavy_atom[h];
        for (int w = 0; w < a.W; ++w) {
            const int s = w * 64 + lane;
            u64 v = ~0ull;
            if (s < a.nb) {
                v = a.hbest[h * a.nb + s];
                if (v != ~0ull) a.hbest[h * a.nb + s] = ~0ull;
            }
            ls_append(a, d, v != ~0ull, (int64_t)s * a.A + t, v);
        }
    }
}

// Ranking a level's discoveries by key (round 5; it replaced a bit per discovery in a global bitmap over
// the level's key space, a popcount prefix per word and an emit that read the word and its prefix at
// random: config 2's drop-in level of 258M discoveries fetched 70 GB and wrote 25 GB in that emit).
// The key space is cut into buckets of 2^bs keys (~2^lr_sub = 2048 buckets of 64 .. 2^18 keys; up to 16384
// buckets of 2^18 keys for 32-bit keys), the buckets into kLrParts rank parts (consecutive bucket ranges):
//   hgx_lr_count    per block an LDS histogram of its range of the discovery list, one global add per
//                   bucket it touched, the block's count per part (push levels first take the value out of
//                   the hash slot and clear the slot; pull levels clear the frontier rows and the union
//                   bitmap)
//   hgx_lr_scan     one block: bucket starts (the level's ranks are key order, so bucket b's ranks are
//                   [start b, start b+1)), the level's size published to the host and the next level
//   hgx_lr_split    per block the same range again into the parts' regions (8 write streams a block)
//   then per part, so that part q's pairs go to the host while part q+1 is ordered:
//   hgx_lr_scatter  per block a range of the part's region: a contiguous slot range per bucket claimed
//                   with one global add, the discoveries copied into it (runs of a bucket per block)
//   hgx_lr_rank     a workgroup per bucket: an LDS bitmap of its keys and a popcount prefix per word;
//                   rank = start + prefix + bits below; pair `rank` of the level, entry `rank` of the next
//                   frontier, the examined bit.  The writes of a bucket land in one window of the outputs.
__global__ void __launch_bounds__(256) hgx_lr_count(LsArgs a, int32_t d) {
    __shared__ int64_t pre[kLsDSegs + 2];
    __shared__ uint32_t hist[kLrMaxBuckets];
    __shared__ uint32_t scnt[kLsMaxW * 64];   // the block's discoveries per seed (the level's runs)
    __shared__ uint32_t pc[kLrParts];
    const int64_t* sl = ls_slot(a, d);
    if (a.ctl[kLsStatus]) return;
    const bool pull = sl[lsPull] != 0;
    const int bs = lr_bucket_bits(sl[lsW], a.lr_sub);
    const int nbk = lr_buckets(sl[lsW], bs);
    for (int b = threadIdx.x; b < nbk; b += 256) hist[b] = 0u;
    if (threadIdx.x < kLrParts) pc[threadIdx.x] = 0u;
    for (int q = threadIdx.x; q < a.nb; q += 256) scnt[q] = 0u;
    const int64_t n = ls_disc_prefix(a, d, pre);   // (syncs the block)
    const int64_t lo = n * blockIdx.x / gridDim.x, hi = n * (blockIdx.x + 1) / gridDim.x;
    for (int64_t x0 = lo + threadIdx.x; x0 < hi; x0 += 256 * kLrU) {   // kLrU independent loads a thread
        int64_t pos[kLrU];
        u64 v[kLrU];
        int64_t sa[kLrU];
#pragma unroll
        for (int u = 0; u < kLrU; ++u) {
            const int64_t x = x0 + 256 * u;
            pos[u] = x < hi ? ls_disc_pos(a, pre, x) : -1;
            v[u] = pos[u] >= 0 ? a.dval[pos[u]] : 0ull;
            sa[u] = pos[u] >= 0 ? a.disc[pos[u]] : 0;
        }
#pragma unroll
        for (int u = 0; u < kLrU; ++u) {
            if (pos[u] < 0) continue;
            if (!pull) {   // v is the hash slot
                const u64 hs = v[u];
                v[u] = a.hval[hs];
                a.dval[pos[u]] = v[u];
                a.hkey[hs] = kLsEmpty;
                a.hval[hs] = ~0ull;
            }
            atomicAdd(&hist[((v[u] >> 32) - 1ull) >> bs], 1u);
            atomicAdd(&scnt[(int)(sa[u] / a.A)], 1u);
        }
    }
    __syncthreads();
    for (int b = threadIdx.x; b < nbk; b += 256)
        if (hist[b]) {
            atomicAdd(&a.bcnt[b], hist[b]);
            atomicAdd(&pc[lr_part((uint32_t)b, nbk)], hist[b]);
        }
    for (int q = threadIdx.x; q < a.nb; q += 256)
        if (scnt[q]) atomicAdd(&a.seedcnt[q], scnt[q]);
    __syncthreads();
    if (threadIdx.x < kLrParts) a.pcnt[blockIdx.x * kLrParts + threadIdx.x] = pc[threadIdx.x];   // (hgx_lr_split)
    if (pull) {
        const int64_t nu = sl[lsU];
        for (int64_t u = blockIdx.x * 256ll + threadIdx.x; u < nu; u += (int64_t)gridDim.x * 256) {
            const int32_t p = a.ulist[u];
            for (int w = 0; w < a.W; ++w) a.frow[u * a.W + w] = 0ull;
            a.ubit[p >> 6] = 0ull;
        }
    }
}

// One block of 1024 threads.
__global__ void __launch_bounds__(1024) hgx_lr_scan(LsArgs a, int32_t d, u64 seq) {
    __shared__ int64_t pre[kLsDSegs + 2];
    __shared__ int64_t wsum[16];
    int64_t* sl = ls_slot(a, d);
    int64_t status = a.ctl[kLsStatus];
    const int64_t out0 = sl[lsOut];
    int64_t n = ls_disc_prefix(a, d, pre);
    if (!status && (n > a.cap || out0 + n > a.cap)) status = 1;   // the pairs outgrow the output
    if (status) n = 0;
    // two host slots by level parity: the host reads level d while level d+1 may already be publishing
    // (it never enqueues level d+2 before it has read level d)
    u64* hf = a.hflag + 4 * (d & 1);
    auto publish = [&]() {   // thread 0, after every word the host reads with it was stored
        __hip_atomic_store(hf, (u64)n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(hf + 1, (u64)status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __threadfence_system();
        __hip_atomic_store(hf + 2, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    };
    if (threadIdx.x == 0) {
        if (status) atomicOr((unsigned long long*)&a.ctl[kLsStatus], (unsigned long long)status);
        int64_t* nx = a.ctl + ((d + 1) % kLsSlots) * kLsSlotWords;
        nx[lsF] = n;
        nx[lsOut] = out0 + n;
        sl[lsN] = n;
        if (n == 0) publish();
    }
    if (n == 0) return;   // (every thread: n is the block's)
    {   // the level's runs: seed s's pairs (distance d + 1) start after the earlier seeds' (seed-major ranks)
        __shared__ int s_ovf;
        if (threadIdx.x == 0) s_ovf = 0;
        const int q = threadIdx.x;   // nb <= 1024 seeds, a thread each
        const int64_t c = q < a.nb ? (int64_t)a.seedcnt[q] : 0;
        int64_t x = c;
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int64_t y = __shfl_up(x, off);
            if (lane >= off) x += y;
        }
        if (lane == 63) wsum[w] = x;
        __syncthreads();
        int64_t before = x - c;
        for (int k = 0; k < w; ++k) before += wsum[k];
        if (c > 0) {
            const int64_t r = atomicAdd((unsigned long long*)&a.ctl[kLsRuns], 1ull);
            if (r < a.rcap) {
                a.runs[3 * r] = d + 1;
                a.runs[3 * r + 1] = q;
                a.runs[3 * r + 2] = out0 + before;
            } else {
                atomicOr((unsigned long long*)&a.ctl[kLsStatus], 2ull);   // more runs than rcap
                s_ovf = 1;
            }
        }
        __syncthreads();   // (wsum is reused below)
        if (s_ovf) {   // the host grows rcap and reruns the chunk
            if (threadIdx.x == 0) {
                status = 2;
                publish();
            }
            return;
        }
    }
    const int bs = lr_bucket_bits(sl[lsW], a.lr_sub);
    const int nbk = lr_buckets(sl[lsW], bs);
    constexpr int per = kLrMaxBuckets / 1024;
    const int b0 = threadIdx.x * per;
    int64_t c[per], s = 0;
#pragma unroll
    for (int k = 0; k < per; ++k) {
        c[k] = b0 + k < nbk ? (int64_t)a.bcnt[b0 + k] : 0;
        s += c[k];
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int64_t x = s;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int64_t y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    int64_t run = x - s;
    for (int k = 0; k < w; ++k) run += wsum[k];
    u64* bnd = a.hflag + 8 + (kLrParts + 1) * (d & 1);   // the rank parts' first ranks (mapped)
    bool wrote = false;
#pragma unroll
    for (int k = 0; k < per; ++k) {
        if (b0 + k < nbk) {
            a.bstart[b0 + k] = run;
            a.bcur[b0 + k] = (uint32_t)run;
            for (int q = 0; q < kLrParts; ++q)
                if (q * nbk / kLrParts == b0 + k) {
                    __hip_atomic_store(bnd + q, (u64)run, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    a.pcur[q] = (uint32_t)run;
                    wrote = true;
                }
        }
        run += c[k];
    }
    if (threadIdx.x == 1023) {
        a.bstart[nbk] = run;   // == n
        __hip_atomic_store(bnd + kLrParts, (u64)run, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        wrote = true;
    }
    if (wrote) __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) publish();
}

// The level's discoveries into kLrParts regions by rank part (bk_v / bk_sa; part q's region is its rank
// range [start of its first bucket, start of the next part's)): the count pass's per-block part counts give
// each block its slot ranges, a wave claims a part's slots with one LDS add, so a wave's writes to one part
// are consecutive.  The same block ranges as hgx_lr_count (both launch kLrG blocks).
__global__ void __launch_bounds__(256) hgx_lr_split(LsArgs a, int32_t d) {
    __shared__ int64_t pre[kLsDSegs + 2];
    __shared__ uint32_t slot[kLrParts];
    const int64_t* sl = ls_slot(a, d);
    if (a.ctl[kLsStatus]) return;
    const int bs = lr_bucket_bits(sl[lsW], a.lr_sub);
    const int nbk = lr_buckets(sl[lsW], bs);
    if (threadIdx.x < kLrParts) {
        const uint32_t c = a.pcnt[blockIdx.x * kLrParts + threadIdx.x];
        slot[threadIdx.x] = c ? atomicAdd(&a.pcur[threadIdx.x], c) : 0u;
    }
    const int64_t n = ls_disc_prefix(a, d, pre);   // (syncs the block)
    const int64_t lo = n * blockIdx.x / gridDim.x, hi = n * (blockIdx.x + 1) / gridDim.x;
    const int lane = threadIdx.x & 63;
    for (int64_t x0 = lo + threadIdx.x; x0 < hi; x0 += 256 * kLrU) {
        int64_t pos[kLrU];
        u64 v[kLrU];
        int64_t sa[kLrU];
#pragma unroll
        for (int u = 0; u < kLrU; ++u) {
            const int64_t x = x0 + 256 * u;
            pos[u] = x < hi ? ls_disc_pos(a, pre, x) : -1;
            v[u] = pos[u] >= 0 ? a.dval[pos[u]] : 0ull;
            sa[u] = pos[u] >= 0 ? a.disc[pos[u]] : 0;
        }
#pragma unroll
        for (int u = 0; u < kLrU; ++u) {
            const int q = pos[u] >= 0 ? lr_part((uint32_t)(((v[u] >> 32) - 1ull) >> bs), nbk) : -1;
            u64 rem = __ballot(q >= 0);   // (the lanes still in the loop)
            uint32_t my = 0;
            while (rem) {   // one LDS add per part present in the wave
                const int lead = __ffsll((long long)rem) - 1;
                const int qq = __shfl(q, lead);
                const u64 m = __ballot(q == qq);
                uint32_t base = 0;
                if (lane == lead) base = atomicAdd(&slot[qq], (uint32_t)__popcll(m));
                base = __shfl(base, lead);
                if (q == qq) my = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
                rem &= ~m;
            }
            if (q >= 0) {
                a.bk_v[my] = v[u];
                a.bk_sa[my] = sa[u];
            }
        }
    }
}

// Part `part` of kLrParts: its region of bk_v / bk_sa into bucket order, in place of the level's
// discovery list (dval / disc, dead after hgx_lr_split), each block a contiguous range of the region with
// a contiguous slot range per bucket claimed with one global add.
__global__ void __launch_bounds__(256) hgx_lr_scatter(LsArgs a, int32_t d, int32_t part) {
    __shared__ uint32_t slot[kLrMaxBuckets / kLrParts];
    const int64_t* sl = ls_slot(a, d);
    if (a.ctl[kLsStatus] || sl[lsN] == 0) return;
    const int bs = lr_bucket_bits(sl[lsW], a.lr_sub);
    const int nbk = lr_buckets(sl[lsW], bs);
    const uint32_t blo = (uint32_t)(part * nbk / kLrParts), nbp = (uint32_t)((part + 1) * nbk / kLrParts) - blo;
    if (nbp == 0) return;
    const int64_t p0 = a.bstart[blo], np = a.bstart[blo + nbp] - p0;
    if (np == 0) return;
    for (uint32_t b = threadIdx.x; b < nbp; b += 256) slot[b] = 0u;
    __syncthreads();
    const int64_t lo = p0 + np * blockIdx.x / gridDim.x, hi = p0 + np * (blockIdx.x + 1) / gridDim.x;
    for (int64_t x0 = lo + threadIdx.x; x0 < hi; x0 += 256 * kLrU) {
        uint32_t b[kLrU];
#pragma unroll
        for (int u = 0; u < kLrU; ++u) {
            const int64_t x = x0 + 256 * u;
            b[u] = x < hi ? (uint32_t)(((a.bk_v[x] >> 32) - 1ull) >> bs) - blo : ~0u;
        }
#pragma unroll
        for (int u = 0; u < kLrU; ++u)
            if (b[u] < nbp) atomicAdd(&slot[b[u]], 1u);
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nbp; b += 256)   // this block's slot range of each bucket it holds
        if (slot[b]) slot[b] = atomicAdd(&a.bcur[blo + b], slot[b]);
    __syncthreads();
    for (int64_t x0 = lo + threadIdx.x; x0 < hi; x0 += 256 * kLrU) {
        u64 v[kLrU];
        int64_t sa[kLrU];
#pragma unroll
        for (int u = 0; u < kLrU; ++u) {
            const int64_t x = x0 + 256 * u;
            v[u] = x < hi ? a.bk_v[x] : 0ull;
            sa[u] = x < hi ? a.bk_sa[x] : -1;
        }
#pragma unroll
        for (int u = 0; u < kLrU; ++u) {
            if (sa[u] < 0) continue;
            const uint32_t q = atomicAdd(&slot[(uint32_t)(((v[u] >> 32) - 1ull) >> bs) - blo], 1u);
            a.dval[q] = v[u];
            a.disc[q] = sa[u];
        }
    }
}

// Part `part` of kLrParts: the buckets [part * nbk / kLrParts, (part + 1) * nbk / kLrParts).
__global__ void __launch_bounds__(256) hgx_lr_rank(LsArgs a, int32_t d, int32_t part) {
    __shared__ u64 bm[1 << (kLrMaxBucketBits - 6)];
    __shared__ uint32_t wp[1 << (kLrMaxBucketBits - 6)];
    __shared__ int64_t ws[4];
    const int64_t* sl = ls_slot(a, d);
    if (a.ctl[kLsStatus] || sl[lsN] == 0) return;
    const int64_t out0 = sl[lsOut];
    const int bs = lr_bucket_bits(sl[lsW], a.lr_sub);
    const int nbk = lr_buckets(sl[lsW], bs);
    const int nw = 1 << (bs - 6);                 // bitmap words of a bucket
    const int per = (nw + 255) / 256;
    const int nx = (d + 1) & 1;
    const bool last = d + 1 >= a.maxd;
    const int blo = part * nbk / kLrParts, bhi = (part + 1) * nbk / kLrParts;
    for (int b = blo + blockIdx.x; b < bhi; b += gridDim.x) {   // block-uniform
        const int64_t s0 = a.bstart[b], s1 = a.bstart[b + 1];
        if (s0 == s1) continue;
        for (int w = threadIdx.x; w < nw; w += 256) bm[w] = 0ull;
        __syncthreads();
        const u64 kb = (u64)b << bs;
        for (int64_t i0 = s0 + threadIdx.x; i0 < s1; i0 += 256 * kLrU) {
            u64 kk[kLrU];
#pragma unroll
            for (int u = 0; u < kLrU; ++u) {
                const int64_t i = i0 + 256 * u;
                kk[u] = i < s1 ? (a.dval[i] >> 32) - 1ull - kb : ~0ull;
            }
#pragma unroll
            for (int u = 0; u < kLrU; ++u)
                if (kk[u] != ~0ull) atomicOr((unsigned long long*)&bm[kk[u] >> 6], 1ull << (kk[u] & 63));
        }
        __syncthreads();
        const int w0 = threadIdx.x * per;
        int64_t c = 0;
        for (int k = 0; k < per && w0 + k < nw; ++k) c += __popcll(bm[w0 + k]);
        int64_t tot;
        int64_t run = ls_block_scan(c, ws, &tot);   // (syncs)
        for (int k = 0; k < per && w0 + k < nw; ++k) {
            wp[w0 + k] = (uint32_t)run;
            run += __popcll(bm[w0 + k]);
        }
        __syncthreads();
        for (int64_t i0 = s0 + threadIdx.x; i0 < s1; i0 += 256 * kLrU) {
          u64 vv[kLrU];
          int64_t sv[kLrU];
#pragma unroll
          for (int u = 0; u < kLrU; ++u) {
            const int64_t i = i0 + 256 * u;
            vv[u] = i < s1 ? a.dval[i] : 0ull;
            sv[u] = i < s1 ? a.disc[i] : -1;
          }
#pragma unroll
          for (int u = 0; u < kLrU; ++u) {
            if (sv[u] < 0) continue;
            const u64 v = vv[u];
            const int64_t sa = sv[u];
            const u64 kk = (v >> 32) - 1ull - kb;
            const int64_t r = s0 + wp[kk >> 6] + __popcll(bm[kk >> 6] & ((1ull << (kk & 63)) - 1ull));
            const int32_t s = (int32_t)(sa / a.A), t = (int32_t)(sa - (int64_t)s * a.A);
            a.out_pair[out0 + r] = make_int2((int32_t)(uint32_t)v, t);   // one 8-byte store a pair
            if (!last) {       // the next frontier and the examined bit, unless no level follows
                a.fs[nx][r] = s;
                a.fa[nx][r] = t;
                atomicOr((unsigned long long*)&a.vis[(int64_t)t * a.W + (s >> 6)], 1ull << (s & 63));   // examined from now on
            }
          }
        }
        __syncthreads();   // bm / wp are reused by the next bucket
    }
}

// Packed transfer of a large level's rank part (the pairs cross PCIe at ~54 GB/s, the device-time floor
// of config 2's drop-in call): consecutive pairs share their link 58% of the time on config 2's level 2,
// so a part goes to the host as its atoms (4 B a pair), a run-start bit per pair, the links of the run
// starts (4 B each) and a count per 4096-pair block: ~5.8 instead of 8 bytes a pair.
__device__ __forceinline__ bool lr_part_range(const LsArgs& a, int32_t d, int32_t part, int64_t& out0, int64_t& pb, int64_t& np) {
    const int64_t* sl = ls_slot(a, d);
    if (a.ctl[kLsStatus] || sl[lsN] < a.pack_min || sl[lsN] == 0) return false;
    const int bs = lr_bucket_bits(sl[lsW], a.lr_sub);
    const int nbk = lr_buckets(sl[lsW], bs);
    const int blo = part * nbk / kLrParts, bhi = (part + 1) * nbk / kLrParts;
    out0 = sl[lsOut];
    pb = a.bstart[blo];
    np = a.bstart[bhi] - pb;
    return np > 0;
}

// The part's run-start bits (word w = part pairs [64w, 64w + 64)) and each 4096-pair block's run count.
__global__ void __launch_bounds__(256) hgx_lr_pflag(LsArgs a, int32_t d, int32_t part) {
    __shared__ uint32_t ws[4];
    int64_t out0, pb, np;
    if (!lr_part_range(a, d, part, out0, pb, np)) return;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    u64* fl = a.pflag + ((int64_t)(d & 1) * kLrParts + part) * a.pwcap;
    uint32_t* bb = a.pbb + ((int64_t)(d & 1) * kLrParts + part) * a.pbcap;
    const int2* pr = a.out_pair + out0 + pb;
    const int64_t nblk = (np + kLpBlk - 1) / kLpBlk;
    for (int64_t b = blockIdx.x; b < nblk; b += gridDim.x) {   // block-uniform
        uint32_t c = 0;
#pragma unroll 4
        for (int k = 0; k < 16; ++k) {   // 16 words a wave
            const int64_t w = b * 64 + wave * 16 + k;
            const int64_t i = w * 64 + lane;
            const bool ok = i < np;
            const int32_t l = ok ? pr[i].x : 0;
            int32_t prev = __shfl_up(l, 1);
            if (lane == 0) prev = (ok && i > 0) ? pr[i - 1].x : l;
            const u64 m = __ballot(ok && (i == 0 || l != prev));
            if (lane == 0 && w * 64 < np) fl[w] = m;
            c += (uint32_t)__popcll(m);
        }
        if (lane == 0) ws[wave] = c;
        __syncthreads();
        if (threadIdx.x == 0) bb[b] = ws[0] + ws[1] + ws[2] + ws[3];
        __syncthreads();
    }
}

// One block of 1024 threads: the blocks' run counts -> exclusive prefix in place; the part's run count
// published to the host (always, so that the host's wait ends: 0 when the part is not packed).
__global__ void __launch_bounds__(1024) hgx_lr_pscan(LsArgs a, int32_t d, int32_t part, u64 seq) {
    __shared__ int64_t wsum[16];
    int64_t out0 = 0, pb = 0, np = 0;
    const bool on = lr_part_range(a, d, part, out0, pb, np);
    const int64_t nblk = on ? (np + kLpBlk - 1) / kLpBlk : 0;
    uint32_t* bb = a.pbb + ((int64_t)(d & 1) * kLrParts + part) * a.pbcap;
    const int64_t per = (nblk + 1023) / 1024;
    const int64_t k0 = (int64_t)threadIdx.x * per;
    int64_t c = 0;
    for (int64_t k = k0; k < k0 + per && k < nblk; ++k) c += bb[k];
    int64_t x = c;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int64_t y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    int64_t run = x - c;
    for (int k = 0; k < w; ++k) run += wsum[k];
    for (int64_t k = k0; k < k0 + per && k < nblk; ++k) {
        const uint32_t v = bb[k];
        bb[k] = (uint32_t)run;
        run += v;
    }
    if (threadIdx.x == 1023) {
        u64* hp = a.hflag + kPackWords + 2 * ((d & 1) * kLrParts + part);
        __hip_atomic_store(hp, (u64)run, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __threadfence_system();
        __hip_atomic_store(hp + 1, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// The part's atoms and run links: run start i goes to pclink[out0 + pb + (runs before i)].
__global__ void __launch_bounds__(256) hgx_lr_pemit(LsArgs a, int32_t d, int32_t part) {
    __shared__ u64 s_fl[64];
    __shared__ uint32_t s_pre[64];
    int64_t out0, pb, np;
    if (!lr_part_range(a, d, part, out0, pb, np)) return;
    const u64* fl = a.pflag + ((int64_t)(d & 1) * kLrParts + part) * a.pwcap;
    const uint32_t* bb = a.pbb + ((int64_t)(d & 1) * kLrParts + part) * a.pbcap;
    const int2* pr = a.out_pair + out0 + pb;
    int32_t* at = a.patom + out0 + pb;
    int32_t* lk = a.pclink + out0 + pb;
    const int64_t nblk = (np + kLpBlk - 1) / kLpBlk;
    const int lane = threadIdx.x & 63;
    for (int64_t b = blockIdx.x; b < nblk; b += gridDim.x) {
        if (threadIdx.x < 64) {
            const int64_t w = b * 64 + lane;
            const u64 m = w * 64 < np ? fl[w] : 0ull;
            const uint32_t c = (uint32_t)__popcll(m);
            uint32_t x = c;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t y = __shfl_up(x, off);
                if (lane >= off) x += y;
            }
            s_fl[lane] = m;
            s_pre[lane] = bb[b] + x - c;
        }
        __syncthreads();
        const int64_t i0 = b * kLpBlk, i1 = min<int64_t>(np, i0 + kLpBlk);
        for (int64_t i = i0 + threadIdx.x; i < i1; i += 256) {
            const int2 v = pr[i];
            if (a.abytes == 4) {
                at[i] = v.y;
            } else {   // 3 bytes, little-endian, at byte 3 (out0 + pb + i)
                uint8_t* q = (uint8_t*)a.patom + 3 * (out0 + pb + i);
                q[0] = (uint8_t)v.y;
                q[1] = (uint8_t)(v.y >> 8);
                q[2] = (uint8_t)(v.y >> 16);
            }
            const int wl = (int)((i - i0) >> 6), bit = (int)(i & 63);
            const u64 m = s_fl[wl];
            if ((m >> bit) & 1ull) lk[s_pre[wl] + __popcll(m & ((1ull << bit) - 1ull))] = v.x;
        }
        __syncthreads();
    }
}

__global__ void hgx_ls_seed(LsArgs a, int32_t nb, const int32_t* __restrict__ seeds) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nb) {   // examined.put(start, TRUE) (:42-46)
        atomicOr((unsigned long long*)&a.vis[(int64_t)seeds[i] * a.W + (i >> 6)], 1ull << (i & 63));
        a.fa[0][i] = seeds[i];
        a.fs[0][i] = i;
    }
    if (i == 0) {
        a.ctl[lsF] = nb;
        a.ctl[lsOut] = 0;
    }
}

// pin_j[p] for pin p of link row L = the index of L in inc(tgt_idx[p]) (a binary search of the target's
// incidence row; a target repeated in L gets its one entry's index at every position)
__global__ void __launch_bounds__(256) k_pin_j(int64_t M, const int64_t* __restrict__ tgt_off,
                                               const int32_t* __restrict__ tgt_idx, const int64_t* __restrict__ inc_off,
                                               const int32_t* __restrict__ inc_row, int32_t* __restrict__ pin_j) {
    for (int64_t L = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; L < M; L += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = tgt_off[L], e = tgt_off[L + 1];
        for (int64_t q = b; q < e; ++q) {
            const int32_t t = tgt_idx[q];
            int64_t lo = inc_off[t], hi = inc_off[t + 1];
            const int64_t base = lo;
            while (lo < hi) {
                const int64_t mid = (lo + hi) >> 1;
                if (inc_row[mid] < (int32_t)L) lo = mid + 1;
                else hi = mid;
            }
            pin_j[q] = (int32_t)(lo - base);
        }
    }
}

// Pull records: for incidence entry e = (t, L) -- the entry pin q of L points at, inc_off[t] + pin_j[q] --
// rec[4e .. 4e+1] = L's targets (<= 8, -1 padded), rec[4e+2 .. 4e+3] = their pin_j, meta[e] = (link
// atom, arity).  The pull walk reads them in entry order (streamed) instead of L's offsets, link atom,
// target row and pin indices at random (four lines per entry for ~40 useful bytes).  A thread per link;
// a target repeated in L writes its one entry several times with the same bytes.  Rows of > 8 targets
// get the meta only (the walk reads them through tgt_off).
__global__ void __launch_bounds__(256) k_pull_rec(int64_t M, const int64_t* __restrict__ tgt_off,
                                                  const int32_t* __restrict__ tgt_idx, const int64_t* __restrict__ inc_off,
                                                  const int32_t* __restrict__ pin_j, const int32_t* __restrict__ link_atom,
                                                  int4* __restrict__ rec, int2* __restrict__ meta) {
    for (int64_t L = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; L < M; L += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = tgt_off[L];
        const int32_t n = (int32_t)(tgt_off[L + 1] - b);
        int32_t tg[8], pj[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            tg[q] = q < n ? tgt_idx[b + q] : -1;
            pj[q] = q < n ? pin_j[b + q] : 0;
        }
        const int2 m = make_int2(link_atom[L], n);
        for (int32_t q = 0; q < n; ++q) {
            const int32_t t = q < 8 ? tg[q] : tgt_idx[b + q];
            const int64_t e = inc_off[t] + (q < 8 ? pj[q] : pin_j[b + q]);
            meta[e] = m;
            if (n <= 8) {
                rec[4 * e] = make_int4(tg[0], tg[1], tg[2], tg[3]);
                rec[4 * e + 1] = make_int4(tg[4], tg[5], tg[6], tg[7]);
                rec[4 * e + 2] = make_int4(pj[0], pj[1], pj[2], pj[3]);
                rec[4 * e + 3] = make_int4(pj[4], pj[5], pj[6], pj[7]);
            }
        }
    }
}


// ---------------------------------------------------------------------------------------------
// Order-exact multi-workgroup stage (hgx_seq_coop; round 5; two phases a level since
// round 6): the <= 64 seeds the order-exact workgroup engine (hgx_seq_block) hands back -- config 5's six
// big hg.subsumed closures, 2K-101K pairs over 21 levels -- in ONE persistent launch of resident workgroups
// instead of the level engine's launches per level.  Items are yield-adjacency pairs (the generator's
// (target, link) output in stream order, so an item's index IS its stream position and the key needs no
// yield rank).  A level is two phases separated by the light grid barrier (co_barrier_lite; every
// cross-workgroup access is an agent-scope atomic or co_put / co_get, [xwg] below):
//   P1 expand   work items (a frontier entry's pairs, <= kScChunk each, carrying the entry's first item
//               index) -> every pair (t, link) of seed s with t not examined: the level hash keyed by
//               (s, t) keeps the minimum value ((it + 1) << 32 | link) (HGBreadthFirstTraversal.java:56-64).
//               The item whose atomicMin LOWERS the value is the slot's minimum so far: it counts its own
//               key (= its item index) +1 and the displaced key -1 -- per key, per 64-key word, and the
//               word's degree sum (both keys have the same target, so the same degree) -- and records its
//               key: (t, s, link, slot) and t's degree.  Adds commute, so whatever the order of the updates
//               every key ends at 1 exactly when it is its slot's minimum, i.e. a discovery.
//   P2 emit     every workgroup reads the words' counts and degree sums (coalesced) into LDS prefixes; a
//               wave per non-empty word, a lane per key: rank = the count below the key (the level's FIFO
//               order), first item index of the new frontier entry = the degree prefix below it (a wave
//               scan); pair `rank` of the level, the examined bit, the hash slot and the key count back to
//               empty, the next level's work items, per-seed pair counts.
// Round 5 had a third phase between them (the discoveries appended by their first claimers, finalised after
// the hash settled: key bit, degree, key -> discovery): one grid barrier and one phase of dependent round
// trips more per level.
// The key space of a level is its item count T (<= kScKeyCap, else the seeds go to the level engine).
constexpr int kScChunk = 64;                       // adjacency pairs per work item
constexpr int64_t kScKeyCap = (int64_t)1 << 18;    // keys (items) of one level: an LDS prefix of 4096 words
constexpr int kScWords = (int)(kScKeyCap / 64);
constexpr int kScProbes = 64;
constexpr int kScPairs = 2;                        // expand: pairs a lane works on together
// ctl words: [0] barrier, [kScSt .. +1] status by phase parity, [kScSt + 2] sticky status, [kScChain] the chained list's
// length (low 32 bits), [kScItm + p*kCoSegs +
// seg] work-item counters (parity p), then lcnt [kCoMaxLevels x 64]
constexpr int kScSt = 4, kScChain = 7, kScItm = 8, kScLcnt = kScItm + 2 * kCoSegs;
constexpr int64_t kScCtlWords = kScLcnt + (int64_t)kCoMaxLevels * 64;

struct ScArgs {
    int32_t k;                                       // seeds (<= kMaxCoSeeds); -1: chained, from the list below
    int32_t seeds[kMaxCoSeeds];                      // inline in the kernel arguments (no upload)
    const int2* chain;                               // chained: the workgroup engine's (seed index, atom) list
    const uint32_t* chain_n;                         //   and its length (the seeds it handed back)
    int64_t* chain_idx;                              // mapped [kMaxCoSeeds]: the chained seeds' indices, for the host
    int64_t A;
    const int64_t* inc_off;                          // traversed items: incidence entries of expanded atoms
    const int64_t* y_off;                            // the yield adjacency
    const int32_t* a_tgt;
    const int32_t* a_lnk;
    int32_t maxd;
    int64_t vwords;
    u64* vis;                                        // [k * vwords] examined bitmaps (zero between calls)
    u64* hkey;                                       // level hash (hmask + 1 slots, empty between levels)
    u64* hval;
    int64_t hmask;
    int32_t hbits;
    uint32_t* kcnt;                                  // [kScKeyCap] per key: 1 <=> the key is its slot's minimum (0 between levels)
    int4* krec;                                      // [kScKeyCap] the key's (t, s, link, slot), written by its item
    uint32_t* kdeg;                                  // [kScKeyCap] the degree of the key's target
    u64* wcnt;                                       // [2 parities][kScWords] keys counted per 64-key word
    u64* wdeg;                                       // [2 parities][kScWords] their degree sums
    int4* items;                                     // [2 parities][kCoSegs][iseg] (t, s | cnt << 8, ybase, it0)
    int64_t iseg;
    int32_t* out_link;                               // [pcap] pairs, level-major, rank order
    int32_t* out_atom;
    int32_t* out_seed;
    int64_t pcap;
    u64* ctl;
    int64_t* hmeta;                                  // mapped: [0] status (-1 until block 0's normal exit), [1] levels,
                                                     //   [2] pairs, [3] timed out, [4] traversed items
    int64_t* blk_bytes;                              // mapped [gridDim.x]
    int64_t* blk_trav;                               // mapped [gridDim.x] traversed items per block
    int32_t* h_link;                                 // mapped [pcap] the result read out by the kernel's end: links,
    int32_t* h_atom;                                 //   atoms (level-major, rank order)
    int64_t* h_lcnt;                                 //   and [levels x 64] pairs per level and seed
    int64_t* trace;                                  // mapped [3 x kCoMaxLevels] or null (HGX_CO_TRACE): block 0's clock
                                                     //   at each level's start, after its P1 barrier, after its P2 work
    u64 timeout;
};

__device__ __forceinline__ u64 sc_ld(const u64* p) { return __hip_atomic_load((u64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ void sc_st(u64* p, u64 v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ uint32_t sc_ld32(const uint32_t* p) {
    return __hip_atomic_load((uint32_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void sc_st32(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The 64 segment counters at c (agent-scope loads) -> exclusive prefix pre[0 .. kCoSegs] (LDS; whole block).
__device__ __forceinline__ int64_t sc_seg_prefix(const u64* c, int64_t cap, int64_t* pre) {
    if (threadIdx.x < 64) {
        const u64 raw = threadIdx.x < kCoSegs ? sc_ld(c + threadIdx.x) : 0ull;   // [xwg]
        const int64_t v = min((int64_t)raw, cap);
        int64_t x = v;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int64_t y = __shfl_up(x, off);
            if ((int)threadIdx.x >= off) x += y;
        }
        if (threadIdx.x < kCoSegs) pre[threadIdx.x] = x - v;
        if (threadIdx.x == kCoSegs - 1) pre[kCoSegs] = x;
    }
    __syncthreads();
    return pre[kCoSegs];
}

__device__ __forceinline__ int sc_seg_of(const int64_t* pre, int64_t x) {
    int lo = 0, hi = kCoSegs - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (pre[mid] <= x) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// Appends one work item per lane that has one (wave-aggregated; every lane of the wave calls it).
__device__ __forceinline__ void sc_put_items(const ScArgs& a, int par, int seg, int32_t t, int32_t s, int64_t deg,
                                             int64_t ybase, int64_t it0, u64* status) {
    const int lane = threadIdx.x & 63;
    const int64_t nch = (deg + kScChunk - 1) / kScChunk;
    int64_t x = nch;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int64_t y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    const int64_t tot = __shfl(x, 63);
    if (!tot) return;
    u64 b = 0;
    if (lane == 63) b = atomicAdd(a.ctl + kScItm + par * kCoSegs + seg, (u64)tot);   // [xwg]
    b = __shfl(b, 63);
    const int64_t base = (int64_t)b + x - nch;
    if (nch == 0) return;
    if (base + nch > a.iseg) {
        atomicOr(status, 1ull);   // [xwg]
        return;
    }
    int4* L = a.items + ((int64_t)par * kCoSegs + seg) * a.iseg;
    for (int64_t c = 0; c < nch; ++c) {
        const int32_t cnt = (int32_t)min<int64_t>(kScChunk, deg - c * kScChunk);
        co_put(L + base + c, make_int4(t, s | (cnt << 8), (int32_t)(ybase + c * kScChunk), (int32_t)(it0 + c * kScChunk)));   // [xwg]
    }
}

template <int NT>
__global__ void __launch_bounds__(NT) hgx_seq_coop(ScArgs a) {
    constexpr int kWaves = NT / 64;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t gw = (int64_t)blockIdx.x * kWaves + wave, nw = (int64_t)gridDim.x * kWaves;
    const int seg = blockIdx.x % kCoSegs;
    __shared__ uint32_t s_cpre[kScWords + 1], s_dpre[kScWords + 1];
    __shared__ int64_t s_pre[kCoSegs + 1];
    __shared__ int64_t s_T;
    __shared__ u64 s_st;
    __shared__ unsigned long long s_cnt[kMaxCoSeeds];
    __shared__ int64_t s_ws[kWaves];
    __shared__ int32_t s_seeds[kMaxCoSeeds];
    if (threadIdx.x < kMaxCoSeeds) s_cnt[threadIdx.x] = 0;
    // the seeds: the arguments', or chained, the list the workgroup engine's launches filled (every block reads
    // the same length: the previous kernel's writes are visible at this launch's start)
    const int32_t k = a.k >= 0 ? a.k : (int32_t)min<uint32_t>(*a.chain_n, (uint32_t)kMaxCoSeeds + 1u);
    if (a.k < 0 && (k == 0 || k > kMaxCoSeeds)) {   // nothing handed back, or more than one launch holds
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            a.hmeta[5] = k;
            a.hmeta[1] = a.hmeta[2] = 0;
            __hip_atomic_store(a.hmeta, k == 0 ? 0ll : 128ll, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        return;   // (every block: no barrier was reached)
    }
    if (threadIdx.x < k) {
        if (a.k >= 0) {
            s_seeds[threadIdx.x] = a.seeds[threadIdx.x];
        } else {
            const int2 c = a.chain[threadIdx.x];
            s_seeds[threadIdx.x] = c.y;
            if (blockIdx.x == 0) a.chain_idx[threadIdx.x] = c.x;
        }
    }
    __syncthreads();
    int64_t nbytes = 0, trav = 0;
    u64* st_sticky = a.ctl + kScSt + 2;
    u64 gen = 0;
    // level 0: the seeds (examined.put(start, TRUE), HGBreadthFirstTraversal.java:42-46); their items in
    // seed order, seed s's first item index = the degrees of the seeds before it
    int64_t T = 0;
    for (int s = 0; s < k; ++s) T += a.y_off[s_seeds[s] + 1] - a.y_off[s_seeds[s]];
    if (blockIdx.x == 0) {
        if (threadIdx.x < k) {
            const int32_t t = s_seeds[threadIdx.x];
            atomicOr(a.vis + (int64_t)threadIdx.x * a.vwords + (t >> 6), 1ull << (t & 63));   // [xwg]
        }
        for (int s0 = 0; s0 < k; s0 += 64) {   // wave 0: seeds 64 at a time (wave-uniform loop)
            if (wave != 0) break;
            const int s = s0 + lane;
            int32_t t = 0;
            int64_t dg = 0, it0 = 0;
            if (s < k) {
                t = s_seeds[s];
                dg = a.maxd > 0 ? a.y_off[t + 1] - a.y_off[t] : 0;
                for (int q = 0; q < s; ++q) it0 += a.y_off[s_seeds[q] + 1] - a.y_off[s_seeds[q]];
                if (a.maxd > 0) trav += a.inc_off[t + 1] - a.inc_off[t];
            }
            sc_put_items(a, 0, 0, t, s, dg, s < k ? a.y_off[t] : 0, it0, a.ctl + kScSt + 1);
        }
    }
    bool timed_out = co_barrier_lite(a.ctl, gen, a.ctl + kScSt + 1, a.timeout);
    int32_t d = 0;
    int64_t out0 = 0;
    int64_t Tprev = 0;
    u64 ph = 1;   // phases completed (the seeding was phase 0... its errors: word 1)
    bool done = false;   // the traversal ended (no error): every block leaves with the same value
    for (; !timed_out; ++d) {
        const int par = d & 1;
        u64* wcnt = a.wcnt + (int64_t)par * kScWords;
        u64* wdeg = a.wdeg + (int64_t)par * kScWords;
        // ---- P1: expand ----
        if (a.trace && blockIdx.x == 0 && threadIdx.x == 0 && d < kCoMaxLevels) a.trace[3 * d] = (int64_t)wall_clock64();
        if (threadIdx.x == 0) s_st = sc_ld(a.ctl + kScSt + (ph & 1)) | sc_ld(st_sticky);   // [xwg] the last phase's errors
        const int64_t nf = sc_seg_prefix(a.ctl + kScItm + par * kCoSegs, a.iseg, s_pre);
        const u64 st = s_st;
        __syncthreads();
        if (st) {
            if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(st_sticky, st);
            break;
        }
        if (nf == 0 || d >= a.maxd) {   // the same decision in every block
            done = true;
            break;
        }
        if (T > kScKeyCap || d >= kCoMaxLevels) {
            if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(st_sticky, 8ull);
            break;
        }
        u64* stw = a.ctl + kScSt + ((ph + 1) & 1);   // this phase's error word
        // the next level's item counters -> 0 (last read in the previous level's P1; appended to in this
        // level's P2) and the previous level's word counts and degree sums -> 0 (read in its P2, written again
        // in the next level's P1)
        if (blockIdx.x == 0 && threadIdx.x < kCoSegs)
            sc_st(a.ctl + kScItm + (par ^ 1) * kCoSegs + threadIdx.x, 0ull);   // [xwg]
        if (blockIdx.x == 0 && threadIdx.x < 64)   // this level's per-seed pair counts (added in its P2) -> 0
            sc_st(a.ctl + kScLcnt + (int64_t)d * 64 + threadIdx.x, 0ull);    // [xwg]
        for (int64_t w = (int64_t)blockIdx.x * NT + threadIdx.x; w < (Tprev + 63) / 64; w += (int64_t)gridDim.x * NT) {
            sc_st(a.wcnt + (int64_t)(par ^ 1) * kScWords + w, 0ull);   // [xwg]
            sc_st(a.wdeg + (int64_t)(par ^ 1) * kScWords + w, 0ull);   // [xwg]
        }
        const bool expand_next = d + 1 < a.maxd;
        {
            const int4* L = a.items + (int64_t)par * kCoSegs * a.iseg;
            const int64_t per = min<int64_t>(64, (nf + nw - 1) / nw);
            for (int64_t i0 = gw * per; i0 < nf; i0 += nw * per) {
                const int64_t i = i0 + lane;
                int32_t is = 0;
                int64_t yb = 0, itb = 0, cnt = 0;
                if (lane < per && i < nf) {
                    const int sg = sc_seg_of(s_pre, i);
                    const int4 e = co_get(L + (int64_t)sg * a.iseg + (i - s_pre[sg]));   // [xwg]
                    is = e.y & 0xFF;
                    cnt = e.y >> 8;
                    yb = (int64_t)(uint32_t)e.z;
                    itb = (int64_t)(uint32_t)e.w;
                    nbytes += 16;
                }
                int64_t x = cnt;
#pragma unroll
                for (int off = 1; off < 64; off <<= 1) {
                    const int64_t y = __shfl_up(x, off);
                    if (lane >= off) x += y;
                }
                const int64_t TT = __shfl(x, 63), ex = x - cnt;
                // kScPairs pairs a lane per step (wave-uniform): their dependent round trips (target, examined word,
                // slot claim, minimum) overlap instead of following each other
                for (int64_t f0 = 0; f0 < TT; f0 += 64 * kScPairs) {
                    int32_t ts[kScPairs], ss[kScPairs], las[kScPairs];
                    int64_t its[kScPairs];
                    bool ok[kScPairs];
#pragma unroll
                    for (int q = 0; q < kScPairs; ++q) {
                        const int64_t f = f0 + q * 64 + lane;
                        int o = 0;
#pragma unroll
                        for (int step = 32; step > 0; step >>= 1) {
                            const int mid = o + step;
                            if (__shfl(ex, mid) <= f) o = mid;
                        }
                        ss[q] = __shfl(is, o);
                        const int64_t off_ = f - __shfl(ex, o);
                        const int64_t ii = __shfl(yb, o) + off_;
                        its[q] = __shfl(itb, o) + off_;
                        ok[q] = f < TT;
                        ts[q] = ok[q] ? a.a_tgt[ii] : 0;
                        las[q] = ok[q] ? a.a_lnk[ii] : 0;
                        nbytes += ok[q] ? 8 : 0;
                    }
                    u64 vws[kScPairs];
#pragma unroll
                    for (int q = 0; q < kScPairs; ++q)
                        vws[q] = ok[q] ? sc_ld(a.vis + (int64_t)ss[q] * a.vwords + (ts[q] >> 6)) : ~0ull;   // [xwg]
                    u64 keys[kScPairs], vs[kScPairs], hs[kScPairs], olds[kScPairs];
                    bool pend[kScPairs];
#pragma unroll
                    for (int q = 0; q < kScPairs; ++q) {
                        nbytes += ok[q] ? 8 : 0;
                        pend[q] = ok[q] && !((vws[q] >> (ts[q] & 63)) & 1ull);   // not examined yet
                        keys[q] = (u64)(uint32_t)ss[q] << 32 | (u64)(uint32_t)ts[q];
                        vs[q] = ((u64)(its[q] + 1) << 32) | (u64)(uint32_t)las[q];
                        hs[q] = ls_hash(keys[q], a.hbits);
                        olds[q] = 0ull;   // the slot's value before this pair's atomicMin (0: no update made)
                    }
                    // the level hash: claim (CAS) or find the key's slot, then lower its value; every pending pair's
                    // CAS of a probe round in flight together
                    for (int probe = 0; probe < kScProbes; ++probe) {
                        bool any = false;
#pragma unroll
                        for (int q = 0; q < kScPairs; ++q) any |= pend[q];
                        if (!any) break;
                        u64 kk[kScPairs];
#pragma unroll
                        for (int q = 0; q < kScPairs; ++q)
                            kk[q] = pend[q] ? atomicCAS((unsigned long long*)(a.hkey + hs[q]), kLsEmpty, (unsigned long long)keys[q]) : 0ull;   // [xwg]
#pragma unroll
                        for (int q = 0; q < kScPairs; ++q) {
                            if (!pend[q]) continue;
                            if (kk[q] == kLsEmpty || kk[q] == keys[q]) {   // claimed now, or the key's slot
                                olds[q] = atomicMin((unsigned long long*)(a.hval + hs[q]), (unsigned long long)vs[q]);   // [xwg]
                                pend[q] = false;
                                nbytes += 24;
                            } else {
                                hs[q] = (hs[q] + 1) & (u64)a.hmask;
                            }
                        }
                    }
#pragma unroll
                    for (int q = 0; q < kScPairs; ++q) {
                        if (pend[q]) atomicOr(stw, 4ull);   // [xwg] the hash is too full
                        const u64 old = olds[q], v = vs[q];
                        const bool mine = ok[q] && !pend[q] && old > v;   // (old == 0: no update; else a lower value was first)
                        const int32_t t = ts[q];
                        const uint32_t mykey = (uint32_t)its[q];
                        const uint32_t dg = mine && expand_next ? (uint32_t)(a.y_off[t + 1] - a.y_off[t]) : 0u;
                        // the +1s of the wave's new minima, one atomic pair per 64-key word (a wave's pairs are
                        // consecutive items, so their keys share one or two words)
                        u64 rem = __ballot(mine);
                        while (rem) {   // wave-uniform
                            const int ld = __ffsll((long long)rem) - 1;
                            const uint32_t wl = (uint32_t)__shfl((int)(mykey >> 6), ld);
                            const u64 grp = __ballot(mine && (mykey >> 6) == wl);
                            uint64_t sd = ((grp >> lane) & 1ull) ? (uint64_t)dg : 0ull;
#pragma unroll
                            for (int off = 32; off > 0; off >>= 1) sd += __shfl_xor(sd, off);
                            if (lane == ld) {
                                atomicAdd((unsigned long long*)(wcnt + wl), (unsigned long long)__popcll(grp));   // [xwg]
                                if (sd) atomicAdd((unsigned long long*)(wdeg + wl), (unsigned long long)sd);      // [xwg]
                            }
                            rem &= ~grp;
                        }
                        if (!mine) continue;
                        // this pair is the slot's minimum so far: count its key, uncount the displaced one
                        co_put(a.krec + mykey, make_int4(t, ss[q], las[q], (int32_t)(uint32_t)hs[q]));   // [xwg]
                        sc_st32(a.kdeg + mykey, dg);                                                      // [xwg]
                        atomicAdd(a.kcnt + mykey, 1u);                                                    // [xwg]
                        nbytes += 16 + 4 + 4 + 8 + (dg ? 8 : 0);
                        if (old != ~0ull) {   // the displaced minimum (same target: same degree)
                            const uint32_t okey = (uint32_t)((old >> 32) - 1ull);
                            atomicSub(a.kcnt + okey, 1u);                                                 // [xwg]
                            atomicAdd((unsigned long long*)(wcnt + (okey >> 6)), ~0ull);                  // [xwg] -1
                            if (dg) atomicAdd((unsigned long long*)(wdeg + (okey >> 6)), (unsigned long long)(0ull - (u64)dg));   // [xwg]
                            nbytes += 4 + 8 + (dg ? 8 : 0);
                        }
                    }
                }
            }
        }
        timed_out = co_barrier_lite(a.ctl, gen, stw, a.timeout);
        ++ph;
        if (timed_out) break;
        // ---- P2: rank, emit, next items ----
        if (a.trace && blockIdx.x == 0 && threadIdx.x == 0) a.trace[3 * d + 1] = (int64_t)wall_clock64();
        if (threadIdx.x == 0) s_st = sc_ld(a.ctl + kScSt + (ph & 1));   // [xwg]
        const int64_t Wn = (T + 63) / 64;
        {   // the words' counts and degree sums -> exclusive prefixes in LDS (every block; coalesced loads, each
            // thread's run of `per` words then scanned in registers)
            constexpr int per = kScWords / NT;
            for (int64_t w = threadIdx.x; w < (int64_t)kScWords; w += NT) {
                u64 cc = 0, dd = 0;
                if (w < Wn) {
                    cc = sc_ld(wcnt + w);   // [xwg]
                    dd = sc_ld(wdeg + w);   // [xwg]
                }
                s_cpre[w] = (uint32_t)cc;
                s_dpre[w] = (uint32_t)dd;   // (a level's items stay < 2^32)
            }
            __syncthreads();
            int64_t c = 0, g2 = 0;
            uint32_t cw[per], dw[per];
#pragma unroll
            for (int q = 0; q < per; ++q) {   // this thread's run of words (it alone rewrites them below)
                cw[q] = s_cpre[threadIdx.x * per + q];
                dw[q] = s_dpre[threadIdx.x * per + q];
                c += cw[q];
                g2 += dw[q];
            }
            // block exclusive scans of (c, g2): wave shuffles, then the wave sums through LDS
            int64_t xc = c, xg = g2;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const int64_t yc = __shfl_up(xc, off), yg = __shfl_up(xg, off);
                if (lane >= off) {
                    xc += yc;
                    xg += yg;
                }
            }
            __shared__ int64_t s_wc[kWaves], s_wg[kWaves];
            if (lane == 63) {
                s_wc[wave] = xc;
                s_wg[wave] = xg;
            }
            __syncthreads();
            int64_t bc = 0, bg = 0, tc = 0, tg = 0;
#pragma unroll
            for (int q = 0; q < kWaves; ++q) {
                bc += q < wave ? s_wc[q] : 0;
                bg += q < wave ? s_wg[q] : 0;
                tc += s_wc[q];
                tg += s_wg[q];
            }
            int64_t rc = bc + xc - c, rg = bg + xg - g2;
#pragma unroll
            for (int q = 0; q < per; ++q) {
                s_cpre[threadIdx.x * per + q] = (uint32_t)rc;
                s_dpre[threadIdx.x * per + q] = (uint32_t)rg;
                rc += cw[q];
                rg += dw[q];
            }
            if (threadIdx.x == 0) {
                s_cpre[kScWords] = (uint32_t)tc;
                s_T = tg;
            }
            __syncthreads();
        }
        if (s_st) break;
        stw = a.ctl + kScSt + ((ph + 1) & 1);
        const int64_t nd = s_cpre[kScWords];   // the level's discoveries
        const int64_t Tn = s_T;                // the next level's items
        if (out0 + nd > a.pcap) {
            if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(stw, 2ull);   // [xwg]
        } else {
            for (int64_t w = gw; w < Wn; w += nw) {   // a wave per non-empty word, a lane per key
                if (s_cpre[w + 1] == s_cpre[w]) continue;   // wave-uniform
                const uint32_t key = (uint32_t)(w * 64 + lane);
                // the key's count, record and degree loaded together (the record and degree only mean something
                // where the count is 1: one round trip instead of two)
                const bool set = sc_ld32(a.kcnt + key) != 0u;   // [xwg] (1: the key is its slot's minimum)
                int4 rec = co_get(a.krec + key);                // [xwg] (t, s, link, slot)
                uint32_t dg = sc_ld32(a.kdeg + key);            // [xwg]
                const u64 m = __ballot(set);
                if (!set) {
                    rec = make_int4(0, 0, 0, 0);
                    dg = 0;
                }
                int64_t ex = dg;
#pragma unroll
                for (int off = 1; off < 64; off <<= 1) {
                    const int64_t y = __shfl_up(ex, off);
                    if (lane >= off) ex += y;
                }
                ex -= dg;
                const int32_t t = rec.x, s = rec.y;
                if (set) {
                    const int64_t r = out0 + s_cpre[w] + __popcll(m & ((1ull << lane) - 1ull));
                    sc_st32((uint32_t*)a.out_link + r, (uint32_t)rec.z);   // [xwg] read out by another block at the end
                    sc_st32((uint32_t*)a.out_atom + r, (uint32_t)t);       // [xwg]
                    sc_st32((uint32_t*)a.out_seed + r, (uint32_t)s);       // [xwg]
                    atomicAdd(&s_cnt[s], 1ull);
                    const u64 slot = (u64)(uint32_t)rec.w;
                    sc_st32(a.kcnt + key, 0u);          // [xwg] the key, its hash slot: empty for the next level
                    sc_st(a.hkey + slot, kLsEmpty);     // [xwg]
                    sc_st(a.hval + slot, ~0ull);        // [xwg]
                    atomicOr(a.vis + (int64_t)s * a.vwords + (t >> 6), 1ull << (t & 63));   // [xwg] examined from now on
                    if (d + 1 < a.maxd) trav += a.inc_off[t + 1] - a.inc_off[t];   // expanded at level d + 1
                    nbytes += 4 + 16 + 4 + 12 + 4 + 16 + 8;
                }
                sc_put_items(a, par ^ 1, seg, t, s, (int64_t)dg, set ? a.y_off[t] : 0, (int64_t)s_dpre[w] + ex, stw);
            }
        }
        __syncthreads();
        for (int s = threadIdx.x; s < k; s += NT)
            if (s_cnt[s]) {
                atomicAdd(a.ctl + kScLcnt + (int64_t)d * 64 + s, s_cnt[s]);   // [xwg] read by the host
                s_cnt[s] = 0;
            }
        if (a.trace && blockIdx.x == 0 && threadIdx.x == 0) a.trace[3 * d + 2] = (int64_t)wall_clock64();
        out0 += nd;
        Tprev = T;
        T = Tn;
        timed_out = co_barrier_lite(a.ctl, gen, stw, a.timeout);
        ++ph;
    }
    if (timed_out) {   // reported in its own mapped word (as hgx_bfs_coop): the host falls back
        if (threadIdx.x == 0) __hip_atomic_store(a.hmeta + 3, 1ll, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
    }
    // every block left the loop after the same barrier: the bytes and the traversed items of this block
    {
        for (int off = 32; off > 0; off >>= 1) {
            nbytes += __shfl_xor(nbytes, off);
            trav += __shfl_xor(trav, off);
        }
        __syncthreads();
        if (lane == 0) s_ws[wave] = nbytes;
        __syncthreads();
        if (threadIdx.x == 0) {
            int64_t tb = 0;
            for (int q = 0; q < kWaves; ++q) tb += s_ws[q];
            a.blk_bytes[blockIdx.x] = tb;
        }
        __syncthreads();
        if (lane == 0) s_ws[wave] = trav;
        __syncthreads();
        if (threadIdx.x == 0) {
            int64_t tt = 0;
            for (int q = 0; q < kWaves; ++q) tt += s_ws[q];
            a.blk_trav[blockIdx.x] = tt;
        }
    }
    // the readout and the examined bits' reset, by the kernel itself (round 6: the host's copies and clear launch
    // behind a finished stage cost ~0.24 ms of round trips): every pair, level count and examined word is final
    // once the blocks left the loop after the same barrier; each block moves a slice of the pairs into the
    // caller-visible mapped buffer and clears their examined bits (only after a clean end: otherwise the host
    // clears the bitmaps whole and reruns the seeds elsewhere)
    if (done) {
        const int64_t n = min(out0, a.pcap);
        const int64_t lo = n * blockIdx.x / gridDim.x, hi = n * (blockIdx.x + 1) / gridDim.x;
        for (int64_t i = lo + threadIdx.x; i < hi; i += NT) {
            const int32_t t = (int32_t)sc_ld32((const uint32_t*)a.out_atom + i);   // [xwg]
            a.h_link[i] = (int32_t)sc_ld32((const uint32_t*)a.out_link + i);      // [xwg]
            a.h_atom[i] = t;
            a.vis[(int64_t)(int32_t)sc_ld32((const uint32_t*)a.out_seed + i) * a.vwords + (t >> 6)] = 0ull;   // [xwg]
        }
        // the word counts and degree sums back to 0 for the next call (the hash slots and key counts are
        // empty again already: every claimed slot's minimum was emitted and cleared it)
        for (int64_t w = (int64_t)blockIdx.x * NT + threadIdx.x; w < 4 * (int64_t)kScWords; w += (int64_t)gridDim.x * NT)
            a.wcnt[w] = 0ull;   // (wcnt and wdeg are one allocation)
        if (blockIdx.x == 0) {
            for (int s = threadIdx.x; s < k; s += NT) a.vis[(int64_t)s * a.vwords + (s_seeds[s] >> 6)] = 0ull;
            for (int64_t x = threadIdx.x; x < (int64_t)d * 64; x += NT) a.h_lcnt[x] = (int64_t)sc_ld(a.ctl + kScLcnt + x);
        }
    }
    __syncthreads();
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        a.hmeta[1] = d;
        a.hmeta[2] = out0;
        a.hmeta[5] = k;
        u64 sa = sc_ld(st_sticky) | sc_ld(a.ctl + kScSt) | sc_ld(a.ctl + kScSt + 1);
        if (!done && !sa) sa = 64ull;   // (left the loop without a recorded cause: never clean)
        a.hmeta[0] = (int64_t)sa;
    }
}

// Device buffers of one call, given back to the graph's pool at scope exit.
struct SeqScratch {
    hgx_graph* g;
    std::vector<std::pair<void*, size_t>> t;
    void* take(size_t bytes) {
        void* p = g->alloc(bytes);
        t.push_back({p, bytes});
        return p;
    }
    ~SeqScratch() {
        for (auto& x : t) g->release(x.first, x.second);
    }
};

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

// Where the pairs of a seed live: segments of mapped host buffers (dist = nullptr: every pair of the
// segment has distance dist_c).
struct Seg {
    const int32_t *link, *atom, *dist;
    int64_t n;
    int32_t dist_c;
    int32_t stride = 1;   // 2: link / atom interleaved (the level engine's (link, atom) pairs); 0: packed
    // packed (a large level's rank part, hgx_lr_pemit): link = the part's run links, flags = its run-start
    // bits, bb = runs before each 4096-pair block, pi = the part index of the segment's first pair
    const u64* flags = nullptr;
    const uint32_t* bb = nullptr;
    int64_t pi = 0;
    int32_t ab = 4;               // packed: bytes an atom (3: 24-bit little-endian ids; atom is then a byte address)
    hipEvent_t ready = nullptr;   // the copy into its buffer (level engine): readers wait for it
};

// n pairs of a segment from index so on into links / atoms (either may be null): two copies, or one pass
// over interleaved (link, atom) pairs
inline void copy_pairs(const Seg& s, int64_t so, int64_t n, int32_t* links, int32_t* atoms) {
    if (s.stride == 0) {
        if (atoms && s.ab == 4) {
            std::memcpy(atoms, s.atom + so, sizeof(int32_t) * (size_t)n);
        } else if (atoms) {
            const uint8_t* q = (const uint8_t*)s.atom + 3 * so;
            for (int64_t k = 0; k < n; ++k, q += 3) atoms[k] = (int32_t)((uint32_t)q[0] | (uint32_t)q[1] << 8 | (uint32_t)q[2] << 16);
        }
        if (!links || n <= 0) return;
        int64_t i = s.pi + so;
        // the run of pair i: the runs before its 4096-pair block, the run starts before it in the block, its own
        int64_t c = s.bb[i >> 12];
        for (int64_t w = (i >> 12) << 6; w < (i >> 6); ++w) c += __builtin_popcountll(s.flags[w]);
        const int bit = (int)(i & 63);
        c += __builtin_popcountll(s.flags[i >> 6] & (bit == 63 ? ~0ull : (2ull << bit) - 1ull)) - 1;
        int64_t k = 0;
        links[k++] = s.link[c];
        ++i;
        while (k < n) {   // a run-start word at a time: a word without run starts is one fill
            const int b0 = (int)(i & 63);
            const int64_t m = std::min<int64_t>(n - k, 64 - b0);
            const u64 f = (s.flags[i >> 6] >> b0) & (m == 64 ? ~0ull : (1ull << m) - 1ull);
            if (!f) {
                std::fill(links + k, links + k + m, s.link[c]);
            } else {
                for (int64_t j = 0; j < m; ++j) {
                    c += (int64_t)((f >> j) & 1ull);
                    links[k + j] = s.link[c];
                }
            }
            k += m;
            i += m;
        }
        return;
    }
    if (s.stride == 1) {
        if (links) std::memcpy(links, s.link + so, sizeof(int32_t) * (size_t)n);
        if (atoms) std::memcpy(atoms, s.atom + so, sizeof(int32_t) * (size_t)n);
        return;
    }
    const int2* p = (const int2*)(s.link + 2 * so);
    if (links && atoms) {
        for (int64_t i = 0; i < n; ++i) {
            const int2 v = p[i];
            links[i] = v.x;
            atoms[i] = v.y;
        }
    } else if (links) {
        for (int64_t i = 0; i < n; ++i) links[i] = p[i].x;
    } else if (atoms) {
        for (int64_t i = 0; i < n; ++i) atoms[i] = p[i].y;
    }
}

// The level-synchronous engine's output: per seed its segments (one per level it reached), the
// mapped buffers they live in (the result owns them), traversed items, deepest distance.
struct SeqOut {
    std::vector<std::vector<Seg>> segs;   // [n seeds]
    std::vector<PoolBuf> bufs;
    std::vector<hipEvent_t> evs;          // the segments' copy events (owned; waited for before bufs go back)
    double traversed = 0;
    int32_t deepest = 0;
    double bytes = 0;                     // the level engine's algorithmic bytes (kernel counters)
    int64_t pull_levels = 0;              // its levels that ran as pulls
};

PoolBuf take_host_buf(hgx_graph* g, size_t bytes);

// Timing events from the graph's pool (caller holds g->mu): creating and destroying two events per
// call cost more than the short launches they time.
hipEvent_t ev_take(hgx_graph* g) {
    if (!g->ev_pool.empty()) {
        hipEvent_t e = g->ev_pool.back();
        g->ev_pool.pop_back();
        return e;
    }
    hipEvent_t e;
    HGX_HIP(hipEventCreate(&e));
    return e;
}
void ev_give(hgx_graph* g, hipEvent_t e) {
    if (e) g->ev_pool.push_back(e);
}

// The yield list the workgroup and grid stages read (HGX_YIELD_LISTS=0, for A/B: stream the incidence
// and its yield flags instead).
const YieldList* stage_yield_list(hgx_graph* g, int mode, int32_t type) {
    static const bool off = ab_int("HGX_YIELD_LISTS", 1) == 0;
    return off ? nullptr : yield_list(g, mode, type);
}

// The yield adjacency the stages read first (HGX_YIELD_ADJ=0, for A/B: the yield list instead).
const YieldAdj* stage_yield_adj(hgx_graph* g, int mode, const hgx_algen_opts& o) {
    static const bool off = ab_int("HGX_YIELD_ADJ", 1) == 0;
    return off ? nullptr : yield_adj(g, mode, o.link_type, o.return_source ? 1 : 2, o.reverse_order != 0);
}

// Items of the set-mode stages: the yield adjacency, else the yield list, else the incidence.
template <class Args>
void stage_items(hgx_graph* g, int mode, const hgx_algen_opts& o, Args& a) {
    if (const YieldAdj* ya = stage_yield_adj(g, mode, o)) {
        a.y_off = ya->off;
        a.a_tgt = ya->tgt;
    } else if (const YieldList* yl = stage_yield_list(g, mode, o.link_type)) {
        a.y_off = yl->off;
        a.y_row = yl->row;
    }
}

// Key widths of the level-synchronous engine and the block engine's yield rank (once per snapshot).
void seq_maxes(hgx_graph* g) {
    if (g->max_deg >= 0) return;
    hipStream_t st = g->stream;
    u64* d = (u64*)g->alloc(16);
    HGX_HIP(hipMemsetAsync(d, 0, 16, st));
    k_seq_maxes<<<grid_for(std::max(g->M, g->A), 256), 256, 0, st>>>(g->M, g->tgt_off, g->A, g->inc_off, d);
    HGX_CHECK_LAUNCH();
    u64* h = (u64*)g->pinned_buf(16);
    HGX_HIP(hipMemcpyAsync(h, d, 16, hipMemcpyDeviceToHost, st));
    HGX_HIP(hipStreamSynchronize(st));
    g->release(d, 16);
    g->max_arity = (int64_t)h[0];
    g->max_deg = (int64_t)h[1];
}

// The level-synchronous engine: every level of a chunk of seeds is degree prefix -> expand (one
// incidence item per lane, atomicMin of stream keys on key[seed][atom]) -> sort of the level's
// discoveries by key -> decode.  Any traversal size; two host round trips per level.  Caller holds
// g->mu, g's device is current.
void seq_levels(hgx_graph* g, const int32_t* seeds, int32_t n_seeds, int32_t maxd, const hgx_algen_opts& o,
                SeqOut& out) {
    hipStream_t st = g->stream;
    const int64_t A = g->A;
    seq_maxes(g);
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
    out.segs.assign((size_t)n_seeds, {});
    // per level of a chunk: the mapped buffer [first nb int64][last nb int64][link nn][atom nn]
    struct Level {
        int64_t chunk0, nb, nn;
        int32_t depth;
        char* h;
    };
    std::vector<Level> levels;
    DevBuf<u64> key(g), knew(g), ksort(g);
    DevBuf<int32_t> fa(g), fs(g), na(g), ns(g), dseeds(g);
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
            spin_sync(st);
            const int64_t T = (int64_t)h_cnt[0];
            out.traversed += (double)T;
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
            spin_sync(st);
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
            const size_t hbytes = 16 * (size_t)nb + 8 * (size_t)nn;
            PoolBuf hb = take_host_buf(g, hbytes);
            out.bufs.push_back(hb);
            std::memset(hb.p, 0, 16 * (size_t)nb);   // seeds the level does not reach: empty ranges
            void* dv = nullptr;
            HGX_HIP(hipHostGetDevicePointer(&dv, hb.p, 0));
            int64_t* dfirst = (int64_t*)dv;
            int32_t* dlink = (int32_t*)(dfirst + 2 * nb);
            hgx_seq_decode<<<grid_for(nn, 256), 256, 0, st>>>(nn, dks, dls, e_base - (u64)F, sh_e, sh_j, jmask, A,
                                                              cur_a, cur_s, g->inc_off, g->inc_row, g->link_atom,
                                                              nxa, nxs, dlink, dlink + nn, dfirst, dfirst + nb);
            HGX_CHECK_LAUNCH();
            levels.push_back({c0, nb, nn, d + 1, (char*)hb.p});
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
    spin_sync(st);
    // per seed, its segment of every level it reached (levels in order)
    for (auto& lv : levels) {
        const int64_t* first = (const int64_t*)lv.h;
        const int64_t* last = first + lv.nb;
        const int32_t* lk = (const int32_t*)(first + 2 * lv.nb);
        const int32_t* at = lk + lv.nn;
        for (int64_t s = 0; s < lv.nb; ++s) {
            const int64_t n = last[s] - first[s];
            if (n > 0) out.segs[(size_t)(lv.chunk0 + s)].push_back({lk + first[s], at + first[s], nullptr, n, lv.depth});
        }
    }
    out.deepest = deepest;
}

// A mapped host buffer of the graph's result pool (best fit within 8x), or a new one.
PoolBuf take_host_buf(hgx_graph* g, size_t bytes) {
    {
        std::lock_guard<std::mutex> lk(g->seq_mu);
        size_t best = (size_t)-1;
        for (size_t i = 0; i < g->seq_hbufs.size(); ++i) {
            const size_t n = g->seq_hbufs[i].n;
            if (n >= bytes && n <= std::max<size_t>(8 * bytes, (size_t)1 << 20) &&
                (best == (size_t)-1 || n < g->seq_hbufs[best].n))
                best = i;
        }
        if (best != (size_t)-1) {
            PoolBuf b = g->seq_hbufs[best];
            g->seq_hbufs.erase(g->seq_hbufs.begin() + best);
            return b;
        }
    }
    void* p = nullptr;
    HGX_HIP(hipHostMalloc(&p, bytes, hipHostMallocMapped));
    return PoolBuf{p, bytes};
}

// pin_j of the snapshot (built on first use on the snapshot, shared by its contexts, dropped by
// hgx_graph_update with the other derived tables); caller holds g->mu.
const int32_t* ensure_pin_j(hgx_graph* g) {
    hgx_graph* root = g->base ? g->base : g;
    std::lock_guard<std::mutex> lk(root->ylist_mu);
    if (!root->pin_j && root->P > 0) {
        int32_t* pj = nullptr;
        HGX_HIP(hipMalloc(&pj, sizeof(int32_t) * (size_t)root->P));
        k_pin_j<<<grid_for(root->M, 256, 16384), 256, 0, g->stream>>>(root->M, root->tgt_off, root->tgt_idx,
                                                                     root->inc_off, root->inc_row, pj);
        HGX_CHECK_LAUNCH();
        HGX_HIP(hipStreamSynchronize(g->stream));
        root->pin_j = pj;
    }
    return root->pin_j;
}

// The pull records (k_pull_rec) of the snapshot, built after pin_j on the first pull call; 72 bytes per
// incidence entry (config 2: 14.4 GB), so a snapshot whose records would take more than half of the
// traversal budget (HGX_OPT_SEQ_BUDGET, 48 GiB by default) keeps the random reads instead
// (HGX_LS_PULL_REC=0 as well: A/B).
void ensure_pull_rec(hgx_graph* g, const int32_t* pin_j) {
    hgx_graph* root = g->base ? g->base : g;
    std::lock_guard<std::mutex> lk(root->ylist_mu);
    if (root->pull_rec_state != 0 || root->I <= 0) return;
    const char* ev = ab_env("HGX_LS_PULL_REC");
    const size_t bytes = (size_t)72 * (size_t)root->I;
    if ((ev && std::atoi(ev) == 0) || (int64_t)bytes > g->seq_budget_bytes / 2) {
        root->pull_rec_state = -1;
        return;
    }
    int4* rec = nullptr;
    int2* meta = nullptr;
    if (hipMalloc(&rec, 64 * (size_t)root->I) != hipSuccess || hipMalloc(&meta, 8 * (size_t)root->I) != hipSuccess) {
        (void)hipGetLastError();   // no room: the walk keeps its random reads
        if (rec) (void)hipFree(rec);
        root->pull_rec_state = -1;
        return;
    }
    k_pull_rec<<<grid_for(root->M, 256, 16384), 256, 0, g->stream>>>(root->M, root->tgt_off, root->tgt_idx, root->inc_off,
                                                                    pin_j, root->link_atom, rec, meta);
    HGX_CHECK_LAUNCH();
    HGX_HIP(hipStreamSynchronize(g->stream));
    root->pull_rec = rec;
    root->pull_meta = meta;
    root->pull_rec_state = 1;
}

int log2_ceil(int64_t x) {
    int b = 0;
    while (((int64_t)1 << b) < x) ++b;
    return b;
}

// The level-synchronous engine (hgx_ls_* / hgx_lp_* kernels) over a chunk of <= 1024 seeds; false when
// a level's keys do not fit 32 bits (the caller splits the chunk).  Capacities start small, grow x4 on
// overflow and are kept on the graph.
bool seq_levels2_chunk(hgx_graph* g, const int32_t* seeds, int32_t nb, int32_t maxd, const hgx_algen_opts& o,
                       SeqOut& out, int64_t seed0) {
    hipStream_t st = g->stream;
    const int64_t A = g->A;
    const int mode = seq_mode(o);
    // pull levels (HGX_OPT_SEQ_PULL: 0 never, 1 by the level's width (default), 2 every level -- tests) read
    // the incidence items; with the yield adjacency the items are its pairs and every level pushes
    // (forced pulls drop the adjacency, so the tests reach the pull in every generator mode)
    const int pull_env = std::min(2, std::max(0, (int)g->seq_pull));
    const YieldAdj* ya = pull_env == 2 ? nullptr : stage_yield_adj(g, mode, o);   // a pair's index is its stream position
    const int kbits = ya ? 0 : bitlen(g->max_arity > 1 ? (u64)(g->max_arity - 1) : 0);
    const int32_t W = (nb + 63) / 64;
    if (W > kLsMaxW) fail(HGX_E_INVALID, "hgx_bfs_sequence: a level-engine chunk holds at most 1024 seeds");
    const int pull = ya ? 0 : pull_env;
    bool pull_off = false;   // set when a pull pass overflowed its hit list (rows of > 8 targets)
    const int32_t* pin_j = pull ? ensure_pin_j(g) : nullptr;
    hgx_graph* root = g->base ? g->base : g;
    if (!g->seq_flag) {   // mapped, coherent: the scan kernel's level sizes and rank-part bounds (once per graph)
        void* hp = nullptr;
        HGX_HIP(hipHostMalloc(&hp, 1024, hipHostMallocMapped | hipHostMallocCoherent));
        std::memset(hp, 0, 1024);
        g->seq_flag = (u64*)hp;
    }
    static_assert(2 * kLrParts <= 16 && 8 + 2 * (kLrParts + 1) <= kPackWords && kPackWords + 4 * kLrParts <= 128,
                  "rank-part events / bounds / packed counts");
    for (hipEvent_t& e : g->ls_cev)
        if (!e) HGX_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (hipEvent_t& e : g->ls_ev)
        if (!e) HGX_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    if (!g->stream2) HGX_HIP(hipStreamCreateWithFlags(&g->stream2, hipStreamNonBlocking));
    hipStream_t cs = g->stream2;   // the pairs' copies to the host, a level (part) at a time
    // packed rank parts alternate between two copy streams (two DMA engines side by side; A/B builds:
    // HGX_LS_COPY_STREAMS=1 keeps one)
    static const int ncs = ab_int("HGX_LS_COPY_STREAMS", 2);
    if (ncs > 1 && !g->stream3) HGX_HIP(hipStreamCreateWithFlags(&g->stream3, hipStreamNonBlocking));
    hipStream_t cs2 = ncs > 1 ? g->stream3 : cs;
    u64* hflag_d = nullptr;
    HGX_HIP(hipHostGetDevicePointer((void**)&hflag_d, g->seq_flag, 0));
    const int64_t full = (int64_t)nb * A;
    // starting capacities (grown x4 on overflow and kept on the graph); HGX_OPT_SEQ_SMALL (tests) starts
    // them tiny so that every growth path runs
    const bool small = g->seq_small != 0;
    for (int attempt = 0;; ++attempt) {
        const int64_t cap = std::min(full, std::max<int64_t>(g->ls_cap, small ? 64 : (int64_t)1 << 20));
        const int64_t tcap = std::max<int64_t>(g->ls_tcap, small ? 8 : (int64_t)1 << 16);
        const int64_t rcap = std::max<int64_t>(g->ls_rcap, small ? 4 : (int64_t)1 << 14);
        const int hbits = std::max<int>(log2_ceil(std::max<int64_t>(g->ls_hcap, small ? 64 : (int64_t)1 << 21)), 6);
        LsArgs a{};
        a.A = A;
        a.inc_off = g->inc_off;
        if (ya) {
            a.y_off = ya->off;
            a.a_tgt = ya->tgt;
            a.a_lnk = ya->lnk;
        }
        a.inc_row = g->inc_row;
        a.inc_type = g->inc_type;
        a.yf = mode != sSym ? g->inc_yf : nullptr;
        a.tgt_off = g->tgt_off;
        a.tgt_idx = g->tgt_idx;
        a.link_atom = g->link_atom;
        a.want_type = o.link_type;
        a.min_arity = o.return_source ? 1 : 2;
        a.mode = mode;
        a.rev = o.reverse_order ? 1 : 0;
        a.kbits = kbits;
        a.t_limit = std::min<int64_t>(INT32_MAX - 1, (int64_t)(0xFFFFFFFFull >> kbits));
        static const int lr_sub = ab_int("HGX_LR_SUB", 11);   // A/B builds (buckets ~ 2^lr_sub)
        a.lr_sub = std::min(std::max(lr_sub, 1), 14);
        if (g->seq_tlimit > 0) a.t_limit = std::min<int64_t>(a.t_limit, g->seq_tlimit);   // HGX_OPT_SEQ_TLIMIT (tests)
        a.nb = nb;
        a.W = W;
        a.maxd = maxd;
        a.cap = cap;
        a.tcap = tcap;
        a.rcap = rcap;
        a.hflag = hflag_d;
        SeqScratch w{g, {}};
        const size_t rows = sizeof(u64) * (size_t)A * (size_t)W;
        a.vis = (u64*)w.take(rows);
        a.ctl = (int64_t*)w.take(sizeof(int64_t) * kLsCtlWords);
        for (int k = 0; k < 2; ++k) {
            a.fa[k] = (int32_t*)w.take(sizeof(int32_t) * (size_t)std::max<int64_t>(cap, nb));
            a.fs[k] = (int32_t*)w.take(sizeof(int32_t) * (size_t)std::max<int64_t>(cap, nb));
        }
        a.fbase = (int64_t*)w.take(sizeof(int64_t) * (size_t)std::max<int64_t>(cap, nb));
        a.deg = (int64_t*)w.take(sizeof(int64_t) * (size_t)std::max<int64_t>(cap, nb));
        a.pre = (int64_t*)w.take(sizeof(int64_t) * (size_t)(std::max<int64_t>(cap, nb) + 1));
        a.tile = (int64_t*)w.take(sizeof(int64_t) * (size_t)tcap);
        a.bsum = (int64_t*)w.take(sizeof(int64_t) * kLsG);
        a.segcap = cap / (2 * kLsDSegs);   // the segments (half of cap), then an overflow region of cap
        const size_t nd = (size_t)(cap + kLsDSegs * a.segcap);
        a.disc = (int64_t*)w.take(sizeof(int64_t) * nd);
        a.dval = (u64*)w.take(sizeof(u64) * nd);
        a.bcnt = (uint32_t*)w.take(sizeof(uint32_t) * kLrMaxBuckets);
        a.bcur = (uint32_t*)w.take(sizeof(uint32_t) * kLrMaxBuckets);
        a.bstart = (int64_t*)w.take(sizeof(int64_t) * (kLrMaxBuckets + 1));
        a.bk_v = (u64*)w.take(sizeof(u64) * nd);
        a.bk_sa = (int64_t*)w.take(sizeof(int64_t) * nd);
        a.pcnt = (uint32_t*)w.take(sizeof(uint32_t) * kLrG * kLrParts);
        a.pcur = (uint32_t*)w.take(sizeof(uint32_t) * kLrParts);
        a.out_pair = (int2*)w.take(sizeof(int2) * (size_t)cap);
        // levels of >= pack_min pairs go to the host packed (HGX_OPT_SEQ_PACK_MIN: tests pack tiny levels)
        a.pack_min = g->seq_pack_min > 0 ? g->seq_pack_min : (int64_t)1 << 20;
        a.pack_min = std::max<int64_t>(a.pack_min, 1);
        a.abytes = g->A <= ((int64_t)1 << 24) ? 3 : 4;
        if (a.pack_min <= cap) {
            a.patom = (int32_t*)w.take(sizeof(int32_t) * (size_t)cap);
            a.pclink = (int32_t*)w.take(sizeof(int32_t) * (size_t)cap);
            a.pwcap = cap / 64 + 2;
            a.pbcap = cap / kLpBlk + 2;
            a.pflag = (u64*)w.take(sizeof(u64) * 2 * kLrParts * (size_t)a.pwcap);
            a.pbb = (uint32_t*)w.take(sizeof(uint32_t) * 2 * kLrParts * (size_t)a.pbcap);
        } else {
            a.pack_min = INT64_MAX;   // no level can reach it
        }
        a.seedcnt = (uint32_t*)w.take(sizeof(uint32_t) * (size_t)kLsMaxW * 64);
        a.runs = (int64_t*)w.take(sizeof(int64_t) * 3 * (size_t)rcap);
        a.hbits = hbits;
        a.hmask = ((int64_t)1 << hbits) - 1;
        a.hkey = (u64*)w.take(sizeof(u64) << hbits);
        a.hval = (u64*)w.take(sizeof(u64) << hbits);
        a.pull = pull_off ? 0 : pull;
        a.I = g->I;
        a.pin_j = pin_j;
        a.prof = trace_env("HGX_LS_PROF") ? 1 : 0;
        if (a.pull && pin_j) {
            ensure_pull_rec(g, pin_j);
            a.prec = root->pull_rec;
            a.pmeta = root->pull_meta;
        }
        if (a.pull) {
            const size_t urows = sizeof(u64) * (size_t)std::max<int64_t>(std::min(cap, A), nb) * (size_t)W;   // |union| <= min(F, A)
            a.frow = (u64*)w.take(urows);
            a.ubit = (u64*)w.take(sizeof(u64) * (size_t)(A / 64 + 1));
            a.ulist = (int32_t*)w.take(sizeof(int32_t) * (size_t)std::max<int64_t>(cap, nb));
            a.uidx = (int32_t*)w.take(sizeof(int32_t) * (size_t)std::max<int64_t>(A, 1));
            a.ecap = std::min<int64_t>(std::max<int64_t>(cap, nb) * nb, (int64_t)1 << 28);   // <= 1 GB of rows
            a.E = (uint32_t*)w.take(sizeof(uint32_t) * (size_t)a.ecap);
            a.chunks = root->chunks;
            a.n_chunks = root->n_chunks;
            a.n_heavy = root->n_heavy;
            a.heavy_atom = root->heavy_atom;
            a.hbest = (u64*)w.take(sizeof(u64) * (size_t)std::max<int64_t>(root->n_heavy * nb, 1));
            HGX_HIP(hipMemsetAsync(a.frow, 0, urows, st));
            HGX_HIP(hipMemsetAsync(a.ubit, 0, sizeof(u64) * (size_t)(A / 64 + 1), st));
            HGX_HIP(hipMemsetAsync(a.hbest, 0xFF, sizeof(u64) * (size_t)std::max<int64_t>(root->n_heavy * nb, 1), st));
        }
        int32_t* dseeds = (int32_t*)w.take(sizeof(int32_t) * (size_t)nb);
        int32_t* hs = (int32_t*)g->pinned_buf(sizeof(int32_t) * (size_t)nb);
        std::memcpy(hs, seeds, sizeof(int32_t) * (size_t)nb);
        HGX_HIP(hipMemcpyAsync(dseeds, hs, sizeof(int32_t) * (size_t)nb, hipMemcpyHostToDevice, st));
        // the examined rows (A x W words: 400 MB for config 2's 64 seeds, where the round-4 key array
        // was 64 x A x 8 = 25.6 GB) and the push hash start empty; every per-level table is cleared by
        // the level itself
        HGX_HIP(hipMemsetAsync(a.vis, 0, rows, st));
        HGX_HIP(hipMemsetAsync(a.hkey, 0xFF, sizeof(u64) << hbits, st));
        HGX_HIP(hipMemsetAsync(a.hval, 0xFF, sizeof(u64) << hbits, st));
        HGX_HIP(hipMemsetAsync(a.ctl, 0, sizeof(int64_t) * kLsCtlWords, st));
        hgx_ls_seed<<<grid_for(nb, 256), 256, 0, st>>>(a, nb, dseeds);
        HGX_CHECK_LAUNCH();
        const u64 base = g->seq_flag_seq;
        static const int lr_scatter_g = ab_int("HGX_LR_SCATTER_G", kLrG);   // A/B builds
        static const int lr_rank_g = ab_int("HGX_LR_RANK_G", kLrG);
        const size_t lp_smem = sizeof(u64) * 4 * (size_t)nb;
        auto enqueue = [&](int32_t d) {
            // grids: thousands of idle workgroups cost ~10 us a launch on small levels;
            // the expand's tiles and the pull's atoms are the work that needs more than a block per CU
            hgx_ls_degree<<<kLsG, 256, 0, st>>>(a, d);
            hgx_ls_prefix<<<kLsG, 256, 0, st>>>(a, d);
            hgx_ls_expand<<<1024, 256, 0, st>>>(a, d);
            if (a.pull) {
                hgx_lp_efill<<<512, 256, 0, st>>>(a, d);
                if (W <= 1) hgx_lp_pull<1><<<2048, 256, lp_smem, st>>>(a, d);
                else if (W <= 2) hgx_lp_pull<2><<<2048, 256, lp_smem, st>>>(a, d);
                else if (W <= 4) hgx_lp_pull<4><<<2048, 256, lp_smem, st>>>(a, d);
                else if (W <= 8) hgx_lp_pull<8><<<2048, 256, lp_smem, st>>>(a, d);
                else hgx_lp_pull<16><<<2048, 256, lp_smem, st>>>(a, d);
                hgx_lp_hfinal<<<256, 256, 0, st>>>(a, d);
            }
            hgx_lr_count<<<kLrG, 256, 0, st>>>(a, d);
            hgx_lr_scan<<<1, 1024, 0, st>>>(a, d, base + (u64)d + 1);
            hgx_lr_split<<<kLrG, 256, 0, st>>>(a, d);   // (the count's block ranges)
            // the packed parts' run bits / block counts of level d - 2 (same parity) must have reached the host
            if (d >= 2 && a.pack_min != INT64_MAX) HGX_HIP(hipStreamWaitEvent(st, g->ls_cev[d & 1], 0));
            for (int q = 0; q < kLrParts; ++q) {
                hgx_lr_scatter<<<lr_scatter_g, 256, 0, st>>>(a, d, q);
                hgx_lr_rank<<<lr_rank_g, 256, 0, st>>>(a, d, q);
                if (a.pack_min != INT64_MAX) {
                    hgx_lr_pflag<<<kLrG, 256, 0, st>>>(a, d, q);
                    hgx_lr_pscan<<<1, 1024, 0, st>>>(a, d, q, base + (u64)d + 1);
                    hgx_lr_pemit<<<kLrG, 256, 0, st>>>(a, d, q);
                }
                HGX_HIP(hipEventRecord(g->ls_ev[kLrParts * (d & 1) + q], st));
            }
            HGX_CHECK_LAUNCH();
        };
        // each level's pairs go to the host on the copy stream as soon as the host has read the level's
        // size: a host buffer per level, one copy per rank part after that part's event (the last level's
        // copies overlap its later rank parts and the final runs pass)
        struct LevelPart {   // a packed level's rank part in the level buffer
            int64_t b, e;
            const int32_t* link;
            const u64* flags;
            const uint32_t* bb;
            hipEvent_t ready;
        };
        struct LevelBuf {
            PoolBuf b;
            int64_t out0, n;
            bool packed = false;
            std::vector<LevelPart> parts;
            int ab = 4;                   // (packed) bytes an atom
            hipEvent_t ready = nullptr;   // (unpacked: after all its copies)
        };
        // the pair copies complete after the call returns (the readers wait per segment): an event after
        // each copy group, owned by the result
        std::vector<hipEvent_t> cevs;
        struct EvGuard {   // an attempt that fails drops its events
            std::vector<hipEvent_t>* v;
            bool keep = false;
            ~EvGuard() {
                if (keep) return;
                for (hipEvent_t e : *v) (void)hipEventDestroy(e);
                v->clear();
            }
        } ev_guard{&cevs};
        auto new_copy_event = [&](hipStream_t on) {
            hipEvent_t e = nullptr;
            HGX_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            cevs.push_back(e);
            HGX_HIP(hipEventRecord(e, on));
            return e;
        };
        std::vector<LevelBuf> lbufs;
        struct GiveBack {   // an attempt that fails returns its level buffers after the copies drained
            hgx_graph* g;
            hipStream_t cs;
            std::vector<LevelBuf>* v;
            bool keep = false;
            ~GiveBack() {
                if (keep || v->empty()) return;
                (void)hipStreamSynchronize(cs);
                std::lock_guard<std::mutex> lk(g->seq_mu);
                for (auto& x : *v) g->seq_hbufs.push_back(x.b);
            }
        } give_back{g, cs, &lbufs};
        // waits for a mapped word the device stores with seq (the stream is asked every 1024 polls)
        auto wait_seq = [&](const u64* p, u64 want, const char* what) {
            for (unsigned spin = 0; __atomic_load_n(p, __ATOMIC_ACQUIRE) != want; ++spin) {
                if ((spin & 1023u) != 1023u) continue;
                const hipError_t e = hipStreamQuery(st);
                if (e == hipErrorNotReady) continue;
                if (e != hipSuccess) HGX_HIP(e);
                if (__atomic_load_n(p, __ATOMIC_ACQUIRE) != want) fail(HGX_E_DEVICE, std::string("hgx_bfs_sequence: ") + what);
            }
        };
        auto copy_level = [&](int32_t d, int64_t out0, int64_t n) {
            const u64* bnd = g->seq_flag + 8 + (kLrParts + 1) * (d & 1);
            if (n < a.pack_min) {
                PoolBuf hb = take_host_buf(g, 8 * (size_t)n);   // (link, atom) interleaved
                lbufs.push_back({hb, out0, n});
                int2* hp = (int2*)hb.p;
                for (int q = 0; q < kLrParts; ++q) {
                    const int64_t b = (int64_t)bnd[q], e = (int64_t)bnd[q + 1];
                    if (b < 0 || e > n || e < b) fail(HGX_E_DEVICE, "hgx_bfs_sequence: rank-part bounds inconsistent");
                    if (e == b) continue;
                    HGX_HIP(hipStreamWaitEvent(cs, g->ls_ev[kLrParts * (d & 1) + q], 0));
                    HGX_HIP(hipMemcpyAsync(hp + b, a.out_pair + out0 + b, sizeof(int2) * (size_t)(e - b),
                                           hipMemcpyDeviceToHost, cs));
                }
                HGX_HIP(hipEventRecord(g->ls_cev[d & 1], cs));
                lbufs.back().ready = new_copy_event(cs);
                return;
            }
            // packed: atoms [n] (abytes each) | run links [n] | run-start words [n / 64 + kLrParts + 1] | block counts
            const int ab = a.abytes;
            const size_t nw = (size_t)(n / 64 + kLrParts + 1), nbb = (size_t)(n / kLpBlk + kLrParts + 1);
            const size_t areg = ((size_t)ab * (size_t)n + 7) & ~(size_t)7;
            PoolBuf hb = take_host_buf(g, areg + 4 * (size_t)n + 8 * nw + 4 * nbb);
            LevelBuf lb{hb, out0, n, true, {}};
            lb.ab = ab;
            char* h_atom = (char*)hb.p;
            int32_t* h_link = (int32_t*)(h_atom + areg);
            u64* h_flag = (u64*)(h_link + n);
            uint32_t* h_bb = (uint32_t*)(h_flag + nw);
            for (int q = 0; q < kLrParts; ++q) {
                const int64_t b = (int64_t)bnd[q], e = (int64_t)bnd[q + 1];
                if (b < 0 || e > n || e < b) fail(HGX_E_DEVICE, "hgx_bfs_sequence: rank-part bounds inconsistent");
                if (e == b) continue;
                const u64* hp = g->seq_flag + kPackWords + 2 * ((d & 1) * kLrParts + q);
                wait_seq(hp + 1, base + (u64)d + 1, "a packed part's run count never arrived");
                const int64_t runs = (int64_t)__atomic_load_n(hp, __ATOMIC_RELAXED);
                const int64_t np = e - b, pw = (np + 63) / 64, pbk = (np + kLpBlk - 1) / kLpBlk;
                if (runs < 1 || runs > np) fail(HGX_E_DEVICE, "hgx_bfs_sequence: packed part inconsistent");
                // a part's words / block counts start after the earlier parts' (b / 64 + q >= their end)
                u64* hf = h_flag + b / 64 + q;
                uint32_t* hbk = h_bb + b / kLpBlk + q;
                const hipStream_t c = (q & 1) ? cs2 : cs;
                const int64_t slot = (int64_t)(d & 1) * kLrParts + q;
                HGX_HIP(hipStreamWaitEvent(c, g->ls_ev[kLrParts * (d & 1) + q], 0));
                // the copies start at a 64-byte boundary of the level (out0 + b0): the extra leading atoms are
                // the previous part's, already final (same values), the extra leading links fall in the previous
                // part's link area past its runs or are its own final values
                const int64_t al = ab == 4 ? 16 : 64;   // pairs a 64-byte boundary of the atoms spans
                const int64_t b0 = std::max<int64_t>(0, ((out0 + b) & ~(al - 1)) - out0);
                static const bool align = ab_int("HGX_LS_PACK_ALIGN", 1) != 0;   // A/B builds
                const int64_t bc = align ? b0 : b;
                HGX_HIP(hipMemcpyAsync(h_atom + (size_t)ab * bc, (const char*)a.patom + (size_t)ab * (out0 + bc),
                                       (size_t)ab * (size_t)(e - bc), hipMemcpyDeviceToHost, c));
                HGX_HIP(hipMemcpyAsync(h_link + bc, a.pclink + out0 + bc, sizeof(int32_t) * (size_t)(b + runs - bc),
                                       hipMemcpyDeviceToHost, c));
                HGX_HIP(hipMemcpyAsync(hf, a.pflag + slot * a.pwcap, sizeof(u64) * (size_t)pw, hipMemcpyDeviceToHost, c));
                HGX_HIP(hipMemcpyAsync(hbk, a.pbb + slot * a.pbcap, sizeof(uint32_t) * (size_t)pbk, hipMemcpyDeviceToHost, c));
                lb.parts.push_back({b, e, h_link + b, hf, hbk, new_copy_event(c)});
            }
            if (cs2 != cs) HGX_HIP(hipStreamWaitEvent(cs, new_copy_event(cs2), 0));   // the level's copies joined on cs
            HGX_HIP(hipEventRecord(g->ls_cev[d & 1], cs));
            new_copy_event(cs);   // (the last event of the call: covers both copy streams)
            lbufs.push_back(std::move(lb));
        };
        int64_t total = 0, status = 0;
        int32_t dw = 0, enq = 0;
        if (maxd > 0) {
            enqueue(0);
            enq = 1;
        }
        while (dw < enq) {
            if (enq < maxd && enq == dw + 1) enqueue(enq++);   // one level ahead of the host
            const u64 want = base + (u64)dw + 1;
            const u64* hf = g->seq_flag + 4 * (dw & 1);
            for (unsigned spin = 0; __atomic_load_n(hf + 2, __ATOMIC_ACQUIRE) != want; ++spin) {
                if ((spin & 1023u) != 1023u) continue;   // the stream is asked every 1024 polls
                const hipError_t e = hipStreamQuery(st);
                if (e == hipErrorNotReady) continue;
                if (e != hipSuccess) HGX_HIP(e);
                if (__atomic_load_n(hf + 2, __ATOMIC_ACQUIRE) != want)
                    fail(HGX_E_DEVICE, "hgx_bfs_sequence: a level's size never arrived");
            }
            const int64_t n = (int64_t)__atomic_load_n(hf, __ATOMIC_RELAXED);
            status = (int64_t)__atomic_load_n(hf + 1, __ATOMIC_RELAXED);
            if (status) break;
            seq_mark("level size read");
            if (n > 0) copy_level(dw, total, n);
            total += n;
            ++dw;
            if (n == 0) break;
        }
        g->seq_flag_seq = base + (u64)enq + 2;
        seq_mark("levels read");
        std::vector<int64_t> ctl(kLsCtlWords);
        HGX_HIP(hipMemcpyAsync(ctl.data(), a.ctl, sizeof(int64_t) * kLsCtlWords, hipMemcpyDeviceToHost, st));
        spin_sync(st);
        status |= ctl[kLsStatus];
        if (status) {
            if (status & 16) return false;   // 32-bit level keys do not fit: the caller splits the chunk
            // each attempt stops at the first level that overflows, so a tiny start (HGX_LS_SMALL) may need
            // one attempt per capacity and level; the default starts converge in a few
            if (attempt > 48) fail(HGX_E_DEVICE, "hgx_bfs_sequence: level-synchronous capacities did not converge");
            if (status & 1) g->ls_cap = std::min(full, cap * 4);
            if (status & 2) g->ls_rcap = rcap * 4;
            if (status & 8) g->ls_tcap = tcap * 4;
            if (status & 32) g->ls_hcap = ((int64_t)1 << hbits) * 4;
            if (status & 128) pull_off = true;   // a pull pass's hit list overflowed: this call pushes
            continue;   // rerun the chunk with the grown capacities (kept on the graph)
        }
        const int64_t nruns = ctl[kLsRuns];
        give_back.keep = true;
        for (auto& x : lbufs) out.bufs.push_back(x.b);
        ev_guard.keep = true;
        for (hipEvent_t e : cevs) out.evs.push_back(e);
        out.traversed += (double)ctl[kLsTrav];
        out.bytes += (double)ctl[kLsBytes];
        out.pull_levels += ctl[kLsPullN];
        if (a.prof)
            std::fprintf(stderr, "[hgx ls prof] pull walk (wave-ms summed): phase A %.1f, phase B %.1f, flush %.1f, heavy %.1f, "
                                 "all %.1f; passes %lld, B iterations %lld, flushes %lld\n",
                         ctl[kLsProf] * 1e-5, ctl[kLsProf + 1] * 1e-5, ctl[kLsProf + 2] * 1e-5, ctl[kLsProf + 6] * 1e-5,
                         ctl[kLsProf + 7] * 1e-5, (long long)ctl[kLsProf + 3], (long long)ctl[kLsProf + 4],
                         (long long)ctl[kLsProf + 5]);
        // the runs (3 x nruns); the pairs are in the level buffers once the copy stream drained
        PoolBuf hb = take_host_buf(g, 24 * (size_t)std::max<int64_t>(nruns, 1));
        out.bufs.push_back(hb);
        int64_t* hr = (int64_t*)hb.p;
        if (nruns) HGX_HIP(hipMemcpyAsync(hr, a.runs, sizeof(int64_t) * 3 * (size_t)nruns, hipMemcpyDeviceToHost, st));
        spin_sync(st);
        seq_mark("level kernels done");
        // the copies run on: later work on this stream (the scratch buffers' next users) waits for them, the
        // readers wait per segment (Seg::ready), the result's free waits for all of them
        if (!cevs.empty()) HGX_HIP(hipStreamWaitEvent(st, cevs.back(), 0));
        // a run [b, e) of pairs -> its segments in the level buffer (levels are consecutive ranges of
        // [0, total); a packed level's run may cross rank parts: a segment per part)
        auto run_segs = [&](int64_t b, int64_t e, int32_t dist, std::vector<Seg>& out_segs) {
            size_t L = 0;
            while (L + 1 < lbufs.size() && lbufs[L + 1].out0 <= b) ++L;
            const LevelBuf& lb = lbufs[L];
            if (!lb.packed) {
                const int32_t* pl = (const int32_t*)lb.b.p + 2 * (b - lb.out0);
                Seg sg{pl, pl + 1, nullptr, e - b, dist, 2};
                sg.ready = lb.ready;
                out_segs.push_back(sg);
                return;
            }
            const int64_t rb = b - lb.out0, re = e - lb.out0;
            const char* h_atom = (const char*)lb.b.p;
            for (const LevelPart& pt : lb.parts) {
                const int64_t lo = std::max(rb, pt.b), hi = std::min(re, pt.e);
                if (hi <= lo) continue;
                Seg sg{pt.link, (const int32_t*)(h_atom + (size_t)lb.ab * lo), nullptr, hi - lo, dist, 0};
                sg.ab = lb.ab;
                sg.flags = pt.flags;
                sg.bb = pt.bb;
                sg.pi = lo - pt.b;
                sg.ready = pt.ready;
                out_segs.push_back(sg);
            }
        };
        // runs partition [0, total) in pair order; each seed's runs in distance order are its pairs
        std::vector<int64_t> ord((size_t)nruns);
        for (int64_t k = 0; k < nruns; ++k) ord[k] = k;
        std::sort(ord.begin(), ord.end(), [&](int64_t x, int64_t y) { return hr[3 * x + 2] < hr[3 * y + 2]; });
        // the runs must tile [0, total) exactly (one per seed and level with pairs)
        for (int64_t k = 0; k < nruns; ++k) {
            const int64_t b = hr[3 * ord[k] + 2], e = k + 1 < nruns ? hr[3 * ord[k + 1] + 2] : total;
            const int64_t sd = hr[3 * ord[k] + 1];
            if ((k == 0 && b != 0) || e <= b || sd < 0 || sd >= nb)
                fail(HGX_E_DEVICE, "hgx_bfs_sequence: level engine runs inconsistent (run " + std::to_string(k) + " of " +
                                       std::to_string(nruns) + ": start " + std::to_string(b) + " end " +
                                       std::to_string(e) + " seed " + std::to_string(sd) + " distance " +
                                       std::to_string(hr[3 * ord[k]]) + ", pairs " + std::to_string(total) + ")");
        }
        if (nruns == 0 && total != 0)
            fail(HGX_E_DEVICE, "hgx_bfs_sequence: level engine pairs without runs (" + std::to_string(total) + ")");
        std::vector<std::vector<std::pair<int64_t, int64_t>>> per((size_t)nb);   // (distance, run)
        for (int64_t k = 0; k < nruns; ++k) per[(size_t)hr[3 * ord[k] + 1]].push_back({hr[3 * ord[k]], k});
        for (int32_t s = 0; s < nb; ++s) {
            std::sort(per[s].begin(), per[s].end());
            for (auto& dk : per[s]) {
                const int64_t k = dk.second, b = hr[3 * ord[k] + 2];
                const int64_t e = k + 1 < nruns ? hr[3 * ord[k + 1] + 2] : total;
                run_segs(b, e, (int32_t)dk.first, out.segs[(size_t)(seed0 + s)]);
                out.deepest = std::max(out.deepest, (int32_t)dk.first);
            }
        }
        return true;
    }
}

// The level-synchronous engine over any number of seeds: chunks of <= 1024 seeds; a chunk whose level
// keys do not fit 32 bits is split in halves (its item space shrinks with its seeds), and a single seed
// that still does not fit runs on the round-1 key-array engine (seq_levels: 64-bit keys, a rocPRIM sort
// a level).
void seq_levels_all(hgx_graph* g, const int32_t* seeds, int32_t n_seeds, int32_t maxd, const hgx_algen_opts& o,
                    SeqOut& out, bool v2) {
    if (!v2) {
        seq_levels(g, seeds, n_seeds, maxd, o, out);
        return;
    }
    out.segs.assign((size_t)n_seeds, {});
    const int64_t A = std::max<int64_t>(g->A, 1);
    int64_t B = std::max<int64_t>(1, std::min<int64_t>(n_seeds, 1024));
    // the chunk's examined + frontier rows: 16 bytes per atom and 64 seeds
    while (B > 64 && 16 * A * ((B + 63) / 64) > g->seq_budget_bytes / 2) B = (B + 1) / 2;
    std::vector<std::pair<int64_t, int32_t>> work;   // (first seed, seeds), processed in seed order
    for (int64_t c0 = n_seeds - (n_seeds - 1) % B - 1; n_seeds > 0 && c0 >= 0; c0 -= B)
        work.push_back({c0, (int32_t)std::min<int64_t>(B, n_seeds - c0)});
    while (!work.empty()) {
        const auto [c0, nb] = work.back();
        work.pop_back();
        if (seq_levels2_chunk(g, seeds + c0, nb, maxd, o, out, c0)) continue;
        if (nb > 1) {   // the second half after the first
            const int32_t h = nb / 2;
            work.push_back({c0 + h, nb - h});
            work.push_back({c0, h});
            continue;
        }
        SeqOut one;
        seq_levels(g, seeds + c0, 1, maxd, o, one);
        out.traversed += one.traversed;
        out.deepest = std::max(out.deepest, one.deepest);
        out.segs[(size_t)c0] = std::move(one.segs[0]);
        for (auto& b : one.bufs) out.bufs.push_back(b);
        one.bufs.clear();
    }
}


// ---- the multi-workgroup stage, host side ----


// Whether the grid fits: every workgroup must be resident at once (the barrier waits for all), at most
// 2 per CU and one CU slot left for other streams' kernels.
int co_threads() {
    static const int v = ab_int("HGX_CO_THREADS", 0) == 512 ? 512 : kCoThreads;
    return v;
}


bool co_fits(hgx_graph* g) {
    if (g->co_ok < 0) {
        int per_cu = 0, cus = 0;
        const int nt = co_threads();
        if (nt == 512) HGX_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, hgx_bfs_coop<512>, 512, 0));
        else HGX_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, hgx_bfs_coop<kCoThreads>, kCoThreads, 0));
        HGX_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, g->device));
        const int64_t blocks = (int64_t)std::min(per_cu - 1, 2) * cus;
        static const int cap_env = ab_int("HGX_CO_BLOCKS", 0);   // A/B builds
        const int64_t cap = cap_env >= kCoMinBlocks ? std::min(cap_env, kCoMaxBlocks) : kCoBlocks;
        g->co_ok = blocks >= kCoMinBlocks ? (int32_t)std::min<int64_t>(blocks, cap) : 0;
    }
    return g->co_ok > 0;
}

// One launch of the grid stage: its scratch, pair list and mapped readout, returned to the graph's
// pools with it unless the result took the pairs.
struct CoRun {
    hgx_graph* g;
    SeqScratch sc;
    CoArgs a{};
    int2* pairs = nullptr;
    int64_t pcap = 0;
    PoolBuf hb{nullptr, 0};
    int64_t* hm = nullptr;                  // the mapped readout (CoArgs::hmeta)
    size_t m_seg = 0, m_sel = 0, m_lev = 0;  // its pairs-per-segment, batch-index and level-count parts
    size_t m_blk = 0;                        //   and the blocks' algorithmic bytes
    explicit CoRun(hgx_graph* gg) : g(gg), sc{gg, {}} {}
    CoRun(const CoRun&) = delete;
    CoRun& operator=(const CoRun&) = delete;
    ~CoRun() {
        if (pairs) g->release(pairs, sizeof(int2) * (size_t)pcap);
        if (hb.p) {
            std::lock_guard<std::mutex> lk(g->seq_mu);
            g->seq_hbufs.push_back(hb);
        }
    }
};

// Buffers and arguments of a launch over k seeds (k = -1: the workgroup stage's hand-over, up to kcap
// seeds); the control words are cleared on the stream.
void co_setup(hgx_graph* g, CoRun& r, int32_t k, int32_t kcap, int32_t max_depth, const hgx_algen_opts& o) {
    hipStream_t st = g->stream;
    const int mode = seq_mode(o);
    const int64_t vwords = g->A / 64 + 1;
    if (g->co_vis_seeds < kcap) {   // zero-invariant bitmaps, grown to the seed count
        if (g->co_vis) HGX_HIP(hipFree(g->co_vis));
        g->co_vis = nullptr;
        g->co_vis_seeds = 0;
        const int64_t want = std::max<int64_t>(kcap, 8);
        HGX_HIP(hipMalloc(&g->co_vis, sizeof(u64) * (size_t)(want * vwords)));
        HGX_HIP(hipMemsetAsync(g->co_vis, 0, sizeof(u64) * (size_t)(want * vwords), st));
        g->co_vis_seeds = want;
    }
    if (g->co_pcap == 0) g->co_pcap = (int64_t)1 << 22;
    if (g->co_fr == 0) g->co_fr = (int64_t)1 << 21;
    const int64_t fr_seg = g->co_fr / kCoSegs;   // work items per segment and level
    r.pcap = g->co_pcap;
    int4* fr = (int4*)r.sc.take(sizeof(int4) * 3 * kCoSegs * (size_t)fr_seg);
    r.pairs = (int2*)g->alloc(sizeof(int2) * (size_t)r.pcap);
    const size_t ctl_words = kCoCtlWords + 2 * (size_t)kcap;
    const size_t ctl_bytes = sizeof(u64) * ctl_words + 2 * sizeof(int32_t) * (size_t)kcap;
    u64* ctl = (u64*)r.sc.take(ctl_bytes);
    int32_t* sel_idx = (int32_t*)(ctl + ctl_words);
    HGX_HIP(hipMemsetAsync(ctl, 0, ctl_bytes, st));
    r.m_seg = 4 + 2 * (size_t)kcap;
    r.m_sel = r.m_seg + kCoSegs;
    r.m_lev = r.m_sel + (size_t)kcap;
    r.m_blk = r.m_lev + (size_t)(kcap + 2) * kCoMaxLevels;
    r.hb = take_host_buf(g, sizeof(int64_t) * (r.m_blk + kCoMaxBlocks));
    r.hm = (int64_t*)r.hb.p;
    r.hm[0] = -1;   // written once, at the normal exit of block 0
    r.hm[1] = 0;
    r.hm[2] = k;
    r.hm[3] = 0;    // set by any block that timed out on a grid barrier
    void* hmd = nullptr;
    HGX_HIP(hipHostGetDevicePointer(&hmd, r.hm, 0));
    CoArgs& a = r.a;
    a.k = k;
    a.kcap = kcap;
    a.sel_idx = sel_idx;
    a.seeds = sel_idx + kcap;
    a.inc_off = g->inc_off;
    a.inc_row = g->inc_row;
    a.inc_type = g->inc_type;
    a.yf = mode != sSym ? g->inc_yf : nullptr;
    stage_items(g, mode, o, a);
    a.tgt_off = g->tgt_off;
    a.tgt_idx = g->tgt_idx;
    a.want_type = o.link_type;
    a.min_arity = o.return_source ? 1 : 2;
    a.mode = mode;
    a.maxd = max_depth < 0 ? INT32_MAX : max_depth;
    static const int chunk_env = ab_int("HGX_CO_CHUNK", 0);
    a.chunk = chunk_env > 0 ? std::min(chunk_env, 1 << 20) : kCoChunk;   // entries < 2^23 (co_item)
    static const int bg_env = ab_int("HGX_CO_BARGROUPS", 0);   // A/B builds
    a.bgroups = bg_env > 0 ? std::min(bg_env, kCoBarGroups) : 1;
    static const bool lite_off = ab_int("HGX_CO_LITE", 1) == 0;   // A/B builds
    a.lite = lite_off ? 0 : 1;
    a.vwords = vwords;
    a.vis = g->co_vis;
    a.fr = fr;
    a.fr_seg = fr_seg;
    a.ctl = ctl;
    a.cur = ctl + kCoCtlWords;
    a.trav = ctl + kCoCtlWords + kcap;
    a.pairs = r.pairs;
    a.pseg = r.pcap / kCoSegs;
    a.hmeta = (int64_t*)hmd;
    a.lvl_end = (int64_t*)hmd + r.m_lev;
    a.lvl_trace = a.lvl_end + (size_t)kcap * kCoMaxLevels;
    a.blk_bytes = (int64_t*)hmd + r.m_blk;
    // HGX_OPT_CO_TIMEOUT (per graph, read per launch): tests force the timeout path with a few ticks
    a.timeout = g->co_timeout > 0 ? (u64)g->co_timeout : kCoTimeout;
}

// A launch finished cleanly: block 0 left the level loop normally with both status words clear, and no
// block timed out on a barrier.
bool co_clean(const CoRun& r) { return r.hm[0] == 0 && r.hm[3] == 0; }

void co_launch(hgx_graph* g, CoRun& r) {
    if (co_threads() == 512) hgx_bfs_coop<512><<<(unsigned)g->co_ok, 512, 0, g->stream>>>(r.a);
    else hgx_bfs_coop<kCoThreads><<<(unsigned)g->co_ok, kCoThreads, 0, g->stream>>>(r.a);
    HGX_CHECK_LAUNCH();
}

// A finished launch (status 0) over the seeds sidx (its seed j = batch index sidx[j]) -> out; the
// result takes the pair list.
void co_collect(hgx_graph* g, CoRun& r, const std::vector<int32_t>& sidx, BlockSet& out) {
    const int32_t k = (int32_t)sidx.size();
    const int64_t* hm = r.hm;
    const int32_t nlev = (int32_t)hm[1];   // level counts per seed from the per-level atom counts
    static const bool trace = trace_env("HGX_CO_TRACE");
    if (trace) {   // per level: microseconds since the first level, work items
        const int64_t* tr = hm + r.m_lev + (size_t)r.a.kcap * kCoMaxLevels;
        std::fprintf(stderr, "[hgx coop] k=%d levels=%d:", k, nlev);
        for (int32_t d = 0; d < nlev; ++d)
            std::fprintf(stderr, " %.1f/%lld", (tr[2 * d] - tr[0]) / 100.0, (long long)tr[2 * d + 1]);
        std::fprintf(stderr, "\n");
    }
    out.co_pairs = r.pairs;
    out.co_bytes = sizeof(int2) * (size_t)r.pcap;
    out.co_pseg = r.a.pseg;
    r.pairs = nullptr;
    out.co_segn.assign(hm + r.m_seg, hm + r.m_seg + kCoSegs);
    out.co_n = 0;
    for (int64_t c : out.co_segn) out.co_n += c;
    out.co_idx = sidx;
    out.co_lcnt.assign((size_t)k, {});
    out.co_atoms.assign((size_t)k, {});
    for (int32_t j = 0; j < k; ++j) {
        const int64_t* le = hm + r.m_lev + (int64_t)j * kCoMaxLevels;
        std::vector<int32_t>& lc = out.co_lcnt[j];
        int64_t prev = 0;
        for (int32_t d = 0; d < nlev; ++d) {
            lc.push_back((int32_t)(le[d] - prev));
            prev = le[d];
        }
        while (!lc.empty() && lc.back() == 0) lc.pop_back();
        const int32_t i = sidx[j];
        out.pairs[i] = (int32_t)hm[4 + 2 * j];
        out.levels[i] = (int32_t)lc.size();
        out.lcnt[i] = lc.data();
        out.atoms[i] = nullptr;   // block_materialize
        out.traversed += (double)hm[5 + 2 * j];
    }
    out.expanded = std::max(out.expanded, nlev);
    double bytes = 0;
    for (int b = 0; b < g->co_ok; ++b) bytes += (double)hm[r.m_blk + b];
    out.co_bytes_alg = bytes + 16.0 * (double)out.co_n;   // + the pairs and the bitmap words cleared
}

// A launch that did not finish: the bitmaps may hold bits of atoms no pair records, so they are
// cleared whole; true when only capacities were short (the pair list grown to what was found, a
// level's work items doubled: run again).  A segment's share of a level depends on which blocks find
// its atoms, so a level near the capacity overflows one segment on some runs and not on others.
bool co_failed(hgx_graph* g, CoRun& r, bool may_grow) {
    const int64_t vwords = g->A / 64 + 1;
    HGX_HIP(hipMemsetAsync(g->co_vis, 0, sizeof(u64) * (size_t)(g->co_vis_seeds * vwords), g->stream));
    if (r.hm[3] != 0) ++g->co_timeouts;   // a barrier timed out: the rows engine takes the seeds
    static const bool trace = trace_env("HGX_CO_TRACE");
    if (trace)
        std::fprintf(stderr, "[hgx coop] k=%d status=%lld timeout=%lld\n", r.a.k, (long long)r.hm[0], (long long)r.hm[3]);
    const int64_t st = r.hm[0];
    if (st <= 0 || (st & ~3ll) != 0 || r.hm[3] != 0 || !may_grow) return false;
    if (st & 2) {
        int64_t most = 0;
        for (int q = 0; q < kCoSegs; ++q) most = std::max(most, r.hm[r.m_seg + q]);
        g->co_pcap = std::max<int64_t>(2 * r.pcap, kCoSegs * (most + most / 4 + 64));
    }
    if (st & 1) {
        constexpr int64_t kFrMost = (int64_t)1 << 24;   // 768 MiB of work items over the three slots
        if (g->co_fr >= kFrMost) return false;
        g->co_fr = std::min(2 * g->co_fr, kFrMost);
    }
    return true;
}

float ev_ms(hgx_graph* g, hipEvent_t a, hipEvent_t b) {
    float ms = 0;
    HGX_HIP(hipEventElapsedTime(&ms, a, b));
    return ms;
}

// The multi-workgroup stage over the seeds sidx (indices into seeds); true when they finished there
// (false: a capacity or the grid did not fit, and the rows engine takes them).
bool bfs_coop(hgx_graph* g, const int32_t* seeds, const std::vector<int32_t>& sidx, int32_t max_depth,
              const hgx_algen_opts& o, BlockSet& out) {
    hipStream_t st = g->stream;
    const int32_t k = (int32_t)sidx.size();
    if (k == 0 || k > kMaxCoSeeds || !co_fits(g)) return false;
    for (int attempt = 0; attempt < 3; ++attempt) {
        CoRun r(g);
        co_setup(g, r, k, k, max_depth, o);
        int32_t* hs = (int32_t*)g->pinned_buf(sizeof(int32_t) * (size_t)k);
        for (int32_t j = 0; j < k; ++j) hs[j] = seeds[sidx[j]];
        HGX_HIP(hipMemcpyAsync(const_cast<int32_t*>(r.a.seeds), hs, sizeof(int32_t) * (size_t)k,
                               hipMemcpyHostToDevice, st));
        hipEvent_t ev[2] = {nullptr, nullptr};
        if (g->timing) {
            ev[0] = ev_take(g);
            ev[1] = ev_take(g);
            HGX_HIP(hipEventRecord(ev[0], st));
        }
        co_launch(g, r);
        if (ev[1]) HGX_HIP(hipEventRecord(ev[1], st));
        spin_sync(st);
        if (ev[1]) {
            out.co_ms += ev_ms(g, ev[0], ev[1]);
            ev_give(g, ev[0]);
            ev_give(g, ev[1]);
        }
        if (co_clean(r)) {
            co_collect(g, r, sidx, out);
            return true;
        }
        if (!co_failed(g, r, attempt < 2)) return false;
    }
    return false;
}

// ---- the order-exact multi-workgroup stage, host side ----

// The grid stage's persistent tables (hgx_graph::sc_tab): hash keys and values (all-ones = empty), the word
// counts / degree sums and the key counts (zero).
constexpr int kScHashBits = 19;
constexpr size_t kScTabBytes = sizeof(u64) * (2 * ((size_t)1 << kScHashBits) + 4 * kScWords) + sizeof(uint32_t) * (size_t)kScKeyCap;
void sc_tab_reset(hgx_graph* g) {
    const size_t hb = sizeof(u64) * 2 * ((size_t)1 << kScHashBits);
    HGX_HIP(hipMemsetAsync(g->sc_tab, 0xFF, hb, g->stream));
    HGX_HIP(hipMemsetAsync((char*)g->sc_tab + hb, 0, kScTabBytes - hb, g->stream));
}

int sc_fits(hgx_graph* g) {   // its grid (0: does not fit); the same residency rule as co_fits
    if (g->sc_ok < 0) {
        int per_cu = 0, cus = 0;
        HGX_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, hgx_seq_coop<256>, 256, 0));
        HGX_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, g->device));
        const int64_t blocks = (int64_t)std::min(per_cu - 1, 2) * cus;
        static const int cap_env = ab_int("HGX_SC_BLOCKS", 0);   // A/B builds
        const int64_t cap = cap_env >= kCoMinBlocks ? std::min(cap_env, kCoMaxBlocks) : kCoBlocks;
        g->sc_ok = blocks >= kCoMinBlocks ? (int32_t)std::min<int64_t>(blocks, cap) : 0;
    }
    return g->sc_ok;
}

constexpr int32_t kSeqChainMin = 64;   // seeds of a call from which the grid stage is chained (batches)

// One launch of the order-exact grid stage: arguments, scratch and the mapped readout (ScRun::prepare),
// the launch, and the collection of its result into SeqOut.  The seeds are the launch arguments' (a.k > 0)
// or, chained behind the workgroup engine's launches (round 6), the list that engine fills with the seeds it
// hands back (a.k == -1: the kernel reads the list's length and seeds at its start, and no host round trip
// separates the two stages).
struct ScRun {
    hgx_graph* g;
    SeqScratch w;
    ScArgs a{};
    int nblk = 0;
    bool trace = false;
    PoolBuf hb{}, pb{};
    bool keep_pb = false;
    int32_t* hl = nullptr;
    int32_t* ha = nullptr;
    int64_t* hc = nullptr;
    int64_t* hm = nullptr;
    hipEvent_t ev[2] = {nullptr, nullptr};
    int2* chain_buf = nullptr;      // (chained) the workgroup engine's list and its length
    uint32_t* chain_cnt = nullptr;
    explicit ScRun(hgx_graph* gg) : g(gg), w{gg, {}} {}
    ~ScRun() {
        if (ev[0]) ev_give(g, ev[0]);
        if (ev[1]) ev_give(g, ev[1]);
        std::lock_guard<std::mutex> lk(g->seq_mu);
        if (hb.p) g->seq_hbufs.push_back(hb);
        if (pb.p && !keep_pb) g->seq_hbufs.push_back(pb);
    }
    // chain: the seeds come from the workgroup engine's list (a.chain / a.chain_n, zeroed here)
    void prepare(const YieldAdj* ya, int32_t maxd, bool chain) {
        hipStream_t st = g->stream;
        const int64_t vwords = g->A / 64 + 1;
        if (g->co_vis_seeds < kMaxCoSeeds) {   // the grid stages' zero-invariant bitmaps (shared with hgx_bfs_coop)
            if (g->co_vis) HGX_HIP(hipFree(g->co_vis));
            g->co_vis = nullptr;
            g->co_vis_seeds = 0;
            HGX_HIP(hipMalloc(&g->co_vis, sizeof(u64) * (size_t)(kMaxCoSeeds * vwords)));
            HGX_HIP(hipMemsetAsync(g->co_vis, 0, sizeof(u64) * (size_t)(kMaxCoSeeds * vwords), st));
            g->co_vis_seeds = kMaxCoSeeds;
        }
        if (!g->sc_tab) {   // the stage's tables, empty between calls (a clean launch leaves them so)
            HGX_HIP(hipMalloc(&g->sc_tab, kScTabBytes));
            sc_tab_reset(g);
        }
        a.k = chain ? -1 : 0;
        a.A = g->A;
        a.inc_off = g->inc_off;
        a.y_off = ya->off;
        a.a_tgt = ya->tgt;
        a.a_lnk = ya->lnk;
        a.maxd = maxd;
        a.vwords = vwords;
        a.vis = g->co_vis;
        a.hbits = kScHashBits;                      // 512K slots: a level holds <= kScKeyCap discoveries
        a.hmask = ((int64_t)1 << a.hbits) - 1;
        a.hkey = g->sc_tab;
        a.hval = a.hkey + ((size_t)1 << kScHashBits);
        a.wcnt = a.hval + ((size_t)1 << kScHashBits);   // [2 parities] counts, then [2 parities] degree sums
        a.wdeg = a.wcnt + 2 * kScWords;
        a.kcnt = (uint32_t*)(a.wcnt + 4 * kScWords);
        a.krec = (int4*)w.take(sizeof(int4) * (size_t)kScKeyCap);
        a.kdeg = (uint32_t*)w.take(sizeof(uint32_t) * (size_t)kScKeyCap);
        a.iseg = (int64_t)1 << 14;
        a.items = (int4*)w.take(sizeof(int4) * 2 * kCoSegs * (size_t)a.iseg);
        a.pcap = std::max<int64_t>(g->sc_pcap, (int64_t)1 << 20);
        a.out_link = (int32_t*)w.take(sizeof(int32_t) * 3 * (size_t)a.pcap);
        a.out_atom = a.out_link + a.pcap;
        a.out_seed = a.out_atom + a.pcap;
        a.ctl = (u64*)w.take(sizeof(u64) * (size_t)kScCtlWords);
        // the counters, status words and (chained) the list length in word kScChain -> 0; the level counts are
        // zeroed by each level's P1
        HGX_HIP(hipMemsetAsync(a.ctl, 0, sizeof(u64) * (size_t)kScLcnt, st));
        if (chain) {   // the workgroup engine's list: (seed index, seed atom) [kMaxCoSeeds]; its length in the ctl words
            chain_buf = (int2*)w.take(sizeof(int2) * kMaxCoSeeds);
            chain_cnt = (uint32_t*)(a.ctl + kScChain);
            a.chain = chain_buf;
            a.chain_n = chain_cnt;
        }
        nblk = g->sc_ok;
        trace = trace_env("HGX_CO_TRACE");
        // mapped: [0, 8) status, levels, pairs, timed out, -, seeds | bytes [nblk] | traversed [nblk] | the chained
        // seeds' indices [kMaxCoSeeds] | trace
        hb = take_host_buf(g, sizeof(int64_t) * (8 + 2 * (size_t)nblk + kMaxCoSeeds + (trace ? 3 * (size_t)kCoMaxLevels : 0)));
        hm = (int64_t*)hb.p;
        hm[0] = -1;
        hm[1] = hm[2] = hm[3] = hm[5] = 0;
        void* hmd = nullptr;
        HGX_HIP(hipHostGetDevicePointer(&hmd, hm, 0));
        a.hmeta = (int64_t*)hmd;
        a.blk_bytes = (int64_t*)hmd + 8;
        a.blk_trav = a.blk_bytes + nblk;
        a.chain_idx = a.blk_trav + nblk;
        a.trace = trace ? a.chain_idx + kMaxCoSeeds : nullptr;
        // the result, written by the kernel's end into mapped memory: links [pcap] | atoms [pcap] | level counts
        pb = take_host_buf(g, 8 * (size_t)a.pcap + 8 * (size_t)kCoMaxLevels * 64);
        hl = (int32_t*)pb.p;
        ha = hl + a.pcap;
        hc = (int64_t*)(ha + a.pcap);
        void* pd = nullptr;
        HGX_HIP(hipHostGetDevicePointer(&pd, pb.p, 0));
        a.h_link = (int32_t*)pd;
        a.h_atom = a.h_link + a.pcap;
        a.h_lcnt = (int64_t*)(a.h_atom + a.pcap);
        a.timeout = g->co_timeout > 0 ? (u64)g->co_timeout : kCoTimeout;   // HGX_OPT_CO_TIMEOUT (tests)
    }
    void launch() {
        hipStream_t st = g->stream;
        if (g->timing) {
            ev[0] = ev_take(g);
            ev[1] = ev_take(g);
            HGX_HIP(hipEventRecord(ev[0], st));
        }
        hgx_seq_coop<256><<<(unsigned)nblk, 256, 0, st>>>(a);
        HGX_CHECK_LAUNCH();
        if (ev[1]) HGX_HIP(hipEventRecord(ev[1], st));
        seq_mark("grid stage enqueued");
    }
    // After the launch finished: the k seeds' results (seed j of the launch -> out.segs[sidx[j]]).  1: done;
    // 0: not clean (the bitmaps and tables reset; the caller runs the seeds elsewhere); 2: only the pairs
    // outgrew their buffer (the capacity grown on the graph: run once more)
    int collect(int32_t k, const std::vector<int32_t>& sidx, SeqOut& out, double* ms) {
        hipStream_t st = g->stream;
        if (ev[1]) {
            *ms += ev_ms(g, ev[0], ev[1]);
            ev_give(g, ev[0]);
            ev_give(g, ev[1]);
            ev[0] = ev[1] = nullptr;
        }
        const bool clean = hm[0] == 0 && hm[3] == 0;
        if (trace) {   // per level: P1 (expand + barrier) and P2 (emit) in microseconds of block 0's clock (100 MHz)
            std::fprintf(stderr, "[hgx seq coop] k=%d status=%lld timeout=%lld levels=%lld pairs=%lld; us P1/P2:", k,
                         (long long)hm[0], (long long)hm[3], (long long)hm[1], (long long)hm[2]);
            const int64_t* tr = hm + 8 + 2 * (size_t)nblk + kMaxCoSeeds;
            for (int64_t d = 0; d < hm[1] && d < kCoMaxLevels; ++d)
                std::fprintf(stderr, " %.1f/%.1f", (tr[3 * d + 1] - tr[3 * d]) * 0.01, (tr[3 * d + 2] - tr[3 * d + 1]) * 0.01);
            std::fprintf(stderr, "\n");
        }
        if (!clean) {   // the bitmaps may hold bits no pair records, the tables entries: cleared whole
            if (hm[3] != 0) ++g->co_timeouts;
            HGX_HIP(hipMemsetAsync(g->co_vis, 0, sizeof(u64) * (size_t)(g->co_vis_seeds * (g->A / 64 + 1)), st));
            sc_tab_reset(g);
            if (hm[0] == 2 && hm[3] == 0) {   // only the pairs outgrew their buffer
                g->sc_pcap = a.pcap * 4;
                return 2;
            }
            return 0;
        }
        const int32_t nlev = (int32_t)hm[1];
        const int64_t total = hm[2];
        if (total > a.pcap || nlev > kCoMaxLevels) fail(HGX_E_DEVICE, "hgx_bfs_sequence: grid stage sizes inconsistent");
        keep_pb = true;
        out.bufs.push_back(pb);
        // level-major, seed-major inside a level: seed j's pairs of level d follow the earlier seeds' ones
        int64_t o0 = 0;
        for (int32_t d = 0; d < nlev; ++d) {
            int64_t o = o0;
            for (int32_t j = 0; j < k; ++j) {
                const int64_t c = hc[64 * (size_t)d + j];
                if (c > 0) out.segs[(size_t)sidx[j]].push_back({hl + o, ha + o, nullptr, c, d + 1});
                if (c > 0) out.deepest = std::max(out.deepest, d + 1);
                o += c;
            }
            o0 = o;
        }
        if (o0 != total) fail(HGX_E_DEVICE, "hgx_bfs_sequence: grid stage pair counts inconsistent");
        for (int b = 0; b < nblk; ++b) {
            out.bytes += (double)hm[8 + b];
            out.traversed += (double)hm[8 + nblk + b];
        }
        return 1;
    }
};

// The stage over the seeds sidx of `seeds` (<= kMaxCoSeeds, generator with a yield adjacency): true and
// out.segs[j] / traversed / deepest filled for seed j of sidx when it finished; false (bitmaps cleared)
// when a capacity or the grid did not fit -- the caller runs the level engine.
bool seq_coop(hgx_graph* g, const int32_t* seeds, const std::vector<int32_t>& sidx, int32_t maxd,
              const hgx_algen_opts& o, SeqOut& out, double* ms) {
    const int mode = seq_mode(o);
    const YieldAdj* ya = stage_yield_adj(g, mode, o);
    const int32_t k = (int32_t)sidx.size();
    if (!ya || k == 0 || k > kMaxCoSeeds || !sc_fits(g)) return false;
    static const bool off = ab_int("HGX_SEQ_COOP", 1) == 0;   // A/B builds
    if (off) return false;
    for (int attempt = 0; attempt < 2; ++attempt) {
        ScRun r(g);
        r.prepare(ya, maxd, false);
        r.a.k = k;
        for (int32_t j = 0; j < k; ++j) r.a.seeds[j] = seeds[sidx[j]];
        r.launch();
        spin_sync(g->stream);
        seq_mark("grid stage done");
        const int res = r.collect(k, sidx, out, ms);
        if (res == 1) return true;
        if (res == 0 || attempt == 1) return false;
    }
    return false;
}

}  // namespace

void bfs_block(hgx_graph* g, const int32_t* seeds, int32_t n_seeds, int32_t max_depth, const hgx_algen_opts& o,
               BlockSet& out) {
    hipStream_t st = g->stream;
    const int64_t timeouts0 = g->co_timeouts;
    struct Fallbacks {   // the call's grid launches that fell back (counted by co_failed)
        hgx_graph* g;
        int64_t t0;
        BlockSet& out;
        ~Fallbacks() { out.co_fallbacks = (int32_t)(g->co_timeouts - t0); }
    } fb{g, timeouts0, out};
    const int mode = seq_mode(o);
    if (mode != sSym) ensure_inc_yield(g);
    out.seeds.assign(seeds, seeds + n_seeds);
    out.atoms.assign((size_t)n_seeds, nullptr);
    out.lcnt.assign((size_t)n_seeds, nullptr);
    out.pairs.assign((size_t)n_seeds, -1);
    out.levels.assign((size_t)n_seeds, 0);
    BbArgs a{};
    a.inc_off = g->inc_off;
    a.inc_row = g->inc_row;
    a.inc_type = g->inc_type;
    a.yf = mode != sSym ? g->inc_yf : nullptr;
    a.tgt_off = g->tgt_off;
    a.tgt_idx = g->tgt_idx;
    a.want_type = o.link_type;
    a.min_arity = o.return_source ? 1 : 2;
    a.mode = mode;
    a.maxd = max_depth < 0 ? INT32_MAX : max_depth;
    stage_items(g, mode, o, a);
    const size_t per_seed = (size_t)kBbPairs * 8 + 32;
    // The grid stage goes on the stream right behind the workgroup launches and reads their overflow
    // list itself: one wait for both (HGX_CO_CHAIN=0, for A/B: a host round trip in between).
    static const bool chain_env = ab_int("HGX_CO_CHAIN", 1) != 0;
    std::unique_ptr<CoRun> cr;
    if (g->bfs_block == 1 && chain_env && n_seeds > 0 && co_fits(g)) {
        cr.reset(new CoRun(g));
        co_setup(g, *cr, -1, kMaxCoSeeds, max_depth, o);
        a.sel_n = cr->a.ctl + kCoSel;
        a.sel_idx = const_cast<int32_t*>(cr->a.sel_idx);
        a.sel_seed = const_cast<int32_t*>(cr->a.seeds);
        a.sel_cap = kMaxCoSeeds;
    }
    int32_t* dseeds = nullptr;
    size_t dseeds_n = 0;
    if (n_seeds > kSbInline) {
        dseeds_n = sizeof(int32_t) * (size_t)n_seeds;
        dseeds = (int32_t*)g->alloc(dseeds_n);
        int32_t* hs = (int32_t*)g->pinned_buf(dseeds_n);
        std::memcpy(hs, seeds, dseeds_n);
        HGX_HIP(hipMemcpyAsync(dseeds, hs, dseeds_n, hipMemcpyHostToDevice, st));
    }
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
    if (g->timing) {
        for (auto& e : ev) e = ev_take(g);
        HGX_HIP(hipEventRecord(ev[0], st));
    }
    struct Chunk {
        int64_t c0, nb;
        char* h;
    };
    std::vector<Chunk> chunks;
    // HGX_OPT_BFS_BLOCK 2 (tests): every seed straight to the multi-workgroup stage
    for (int64_t c0 = 0; c0 < (g->bfs_block == 2 ? 0 : n_seeds); c0 += kBbChunk) {
        const int64_t nb = std::min<int64_t>(kBbChunk, n_seeds - c0);
        PoolBuf hb = take_host_buf(g, per_seed * (size_t)nb);
        out.bufs.push_back(hb);
        void* dv = nullptr;
        HGX_HIP(hipHostGetDevicePointer(&dv, hb.p, 0));
        char* d = (char*)dv;
        // layout: meta [4 nb] int64 | atoms [nb * kBbPairs] | level counts [nb * kBbPairs]
        a.n = (int32_t)nb;
        a.base = (int32_t)c0;
        a.meta = (int64_t*)d;
        a.out_atom = (int32_t*)(d + 32 * nb);
        a.out_cnt = a.out_atom + nb * kBbPairs;
        if (nb <= kSbInline) {   // the kernel reads the inline seeds whenever n <= kSbInline
            for (int64_t i = 0; i < nb; ++i) a.seed_inline[i] = seeds[c0 + i];
            a.seeds = nullptr;
        } else {
            a.seeds = dseeds + c0;
        }
        hgx_bfs_block<<<(unsigned)nb, kBbThreads, 0, st>>>(a);
        HGX_CHECK_LAUNCH();
        chunks.push_back({c0, nb, (char*)hb.p});
    }
    if (ev[1]) HGX_HIP(hipEventRecord(ev[1], st));
    if (cr) {
        co_launch(g, *cr);
        if (ev[2]) HGX_HIP(hipEventRecord(ev[2], st));
    }
    spin_sync(st);
    int64_t nsel = cr ? cr->hm[2] : 0;   // seeds the chained grid stage took (> kMaxCoSeeds: none run)
    if (ev[1]) {
        out.ms = ev_ms(g, ev[0], ev[1]);
        if (cr && nsel > 0 && nsel <= kMaxCoSeeds) out.co_ms += ev_ms(g, ev[1], ev[2]);
        for (auto& e : ev) ev_give(g, e);
    }
    if (dseeds) g->release(dseeds, dseeds_n);
    for (auto& c : chunks) {
        const int64_t* meta = (const int64_t*)c.h;
        const int32_t* at = (const int32_t*)(c.h + 32 * c.nb);
        const int32_t* lc = at + c.nb * kBbPairs;
        for (int64_t i = 0; i < c.nb; ++i) {
            const int64_t si = c.c0 + i;
            out.bytes += (double)meta[4 * i + 2];
            if (meta[4 * i] < 0) {
                out.rerun.push_back((int32_t)si);
                continue;
            }
            out.pairs[si] = (int32_t)meta[4 * i];
            out.levels[si] = (int32_t)(meta[4 * i + 3] & 0xFFFFFFFF);
            out.expanded = std::max(out.expanded, (int32_t)(meta[4 * i + 3] >> 32));
            out.traversed += (double)meta[4 * i + 1];
            out.atoms[si] = at + i * kBbPairs;
            out.lcnt[si] = lc + i * kBbPairs;
        }
    }
    if (g->bfs_block == 2)
        for (int32_t i = 0; i < n_seeds; ++i) out.rerun.push_back(i);
    if (cr) {
        if (nsel != (int64_t)out.rerun.size())
            throw std::runtime_error("hgx_bfs_batch: the grid stage took " + std::to_string(nsel) + " of " +
                                     std::to_string(out.rerun.size()) + " handed-over seeds");
        if (nsel == 0 || nsel > kMaxCoSeeds) return;   // none, or more than fit: the rows engine
        std::vector<int32_t> sidx(cr->hm + cr->m_sel, cr->hm + cr->m_sel + nsel);   // the slots' order
        if (co_clean(*cr)) {
            co_collect(g, *cr, sidx, out);
            out.n_coop = (int32_t)nsel;
            out.rerun.clear();
            return;
        }
        const bool again = co_failed(g, *cr, true);
        cr.reset();
        if (!again) return;
    }
    // the few seeds that outgrew a workgroup: one multi-workgroup launch, else the rows engine
    if (!out.rerun.empty() && out.rerun.size() <= (size_t)kMaxCoSeeds && bfs_coop(g, seeds, out.rerun, max_depth, o, out)) {
        out.n_coop = (int32_t)out.rerun.size();
        out.rerun.clear();
    }
}

void free_yield_lists(hgx_graph* g) {
    std::lock_guard<std::mutex> lk(g->ylist_mu);
    if (g->pin_j && !g->base) (void)hipFree(g->pin_j);   // the level engine's pin index (the incidence changed)
    g->pin_j = nullptr;
    if (!g->base) {   // and its pull records
        if (g->pull_rec) (void)hipFree(g->pull_rec);
        if (g->pull_meta) (void)hipFree(g->pull_meta);
    }
    g->pull_rec = nullptr;
    g->pull_meta = nullptr;
    g->pull_rec_state = 0;
    if (!g->base && g->fc_rec) (void)hipFree(g->fc_rec);   // the frontier-code pull's records
    if (!g->base && g->fc_hubs) (void)hipFree(g->fc_hubs);
    g->fc_rec = nullptr;
    g->fc_hubs = nullptr;
    g->fc_nhubs = 0;
    g->fc_rec_state = 0;
    for (YieldList& y : g->ylists) {
        (void)hipFree(y.off);
        (void)hipFree(y.row);
    }
    g->ylists.clear();
    for (YieldAdj& y : g->yadjs) {
        if (y.off) (void)hipFree(y.off);
        if (y.tgt) (void)hipFree(y.tgt);
        if (y.lnk) (void)hipFree(y.lnk);
    }
    g->yadjs.clear();
}

const YieldAdj* yield_adj(hgx_graph* g, int mode, int32_t type, int32_t min_arity, bool rev) {
    if (mode == sSym && type < 0) return nullptr;   // every co-target of every entry: too large to keep
    hgx_graph* root = g->base ? g->base : g;         // built once on the snapshot, read by its contexts
    std::lock_guard<std::mutex> lk(root->ylist_mu);
    for (const YieldAdj& y : root->yadjs)
        if (y.mode == mode && y.type == type && y.min_arity == min_arity && y.rev == (int32_t)rev)
            return y.off ? &y : nullptr;
    if (root->yadjs.size() >= kMaxYieldLists) return nullptr;
    if (mode != sSym) ensure_inc_yield(g);
    hipStream_t st = g->stream;
    const int64_t A = g->A;
    YaArgs a{};
    a.A = A;
    a.inc_off = g->inc_off;
    a.inc_row = g->inc_row;
    a.inc_type = g->inc_type;
    a.yf = mode != sSym ? g->inc_yf : nullptr;
    a.tgt_off = g->tgt_off;
    a.tgt_idx = g->tgt_idx;
    a.link_atom = g->link_atom;
    a.mode = mode;
    a.rev = rev ? 1 : 0;
    a.type = type;
    a.min_arity = min_arity;
    YieldAdj y{mode, type, min_arity, (int32_t)rev, nullptr, nullptr, nullptr, 0};
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((A + 3) / 4, 16384));
    int64_t* off = nullptr;
    HGX_HIP(hipMalloc(&off, sizeof(int64_t) * (size_t)(A + 1)));
    a.cnt = (int64_t*)g->alloc(sizeof(int64_t) * (size_t)(A + 1));
    hgx_ya_count<<<grid, 256, 0, st>>>(a);
    HGX_CHECK_LAUNCH();
    size_t tb = 0;
    HGX_HIP(rocprim::exclusive_scan(nullptr, tb, a.cnt, off, (int64_t)0, (size_t)A + 1, rocprim::plus<int64_t>(), st));
    void* tmp = g->alloc(tb);
    HGX_HIP(rocprim::exclusive_scan(tmp, tb, a.cnt, off, (int64_t)0, (size_t)A + 1, rocprim::plus<int64_t>(), st));
    HGX_HIP(hipMemcpyAsync(&y.n, off + A, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    HGX_HIP(hipStreamSynchronize(st));
    g->release(tmp, tb);
    g->release(a.cnt, sizeof(int64_t) * (size_t)(A + 1));
    if (y.n * 8 > kYieldAdjBudget) {   // remembered as refused: the yield list serves instead
        HGX_HIP(hipFree(off));
        root->yadjs.push_back(y);
        return nullptr;
    }
    y.off = off;
    HGX_HIP(hipMalloc(&y.tgt, sizeof(int32_t) * (size_t)std::max<int64_t>(y.n, 1)));
    HGX_HIP(hipMalloc(&y.lnk, sizeof(int32_t) * (size_t)std::max<int64_t>(y.n, 1)));
    a.off = y.off;
    a.tgt = y.tgt;
    a.lnk = y.lnk;
    hgx_ya_fill<<<grid, 256, 0, st>>>(a);
    HGX_CHECK_LAUNCH();
    HGX_HIP(hipStreamSynchronize(st));
    root->yadjs.push_back(y);
    return &root->yadjs.back();
}

const YieldList* yield_list(hgx_graph* g, int mode, int32_t type) {
    if (mode == sSym && type < 0) return nullptr;   // every entry: the incidence itself
    hgx_graph* root = g->base ? g->base : g;         // built once on the snapshot, read by its contexts
    std::lock_guard<std::mutex> lk(root->ylist_mu);
    for (const YieldList& y : root->ylists)
        if (y.mode == mode && y.type == type) return &y;
    if (root->ylists.size() >= kMaxYieldLists) return nullptr;   // the streamed flags instead
    if (mode != sSym) ensure_inc_yield(g);
    hipStream_t st = g->stream;
    const int64_t A = g->A;
    YieldList y{mode, type, nullptr, nullptr, 0};
    HGX_HIP(hipMalloc(&y.off, sizeof(int64_t) * (size_t)(A + 1)));
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((A + 3) / 4, 16384));
    const uint8_t* yf = mode != sSym ? g->inc_yf : nullptr;
    int64_t* cnt = (int64_t*)g->alloc(sizeof(int64_t) * (size_t)(A + 1));
    hgx_yl_count<<<grid, 256, 0, st>>>(A, g->inc_off, g->inc_type, yf, mode, type, cnt);
    HGX_CHECK_LAUNCH();
    size_t tb = 0;
    HGX_HIP(rocprim::exclusive_scan(nullptr, tb, cnt, y.off, (int64_t)0, (size_t)A + 1, rocprim::plus<int64_t>(), st));
    void* tmp = g->alloc(tb);
    HGX_HIP(rocprim::exclusive_scan(tmp, tb, cnt, y.off, (int64_t)0, (size_t)A + 1, rocprim::plus<int64_t>(), st));
    HGX_HIP(hipMemcpyAsync(&y.n, y.off + A, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    HGX_HIP(hipStreamSynchronize(st));
    g->release(tmp, tb);
    g->release(cnt, sizeof(int64_t) * (size_t)(A + 1));
    HGX_HIP(hipMalloc(&y.row, sizeof(int32_t) * (size_t)std::max<int64_t>(y.n, 1)));
    hgx_yl_fill<<<grid, 256, 0, st>>>(A, g->inc_off, g->inc_row, g->inc_type, yf, mode, type, y.off, y.row);
    HGX_CHECK_LAUNCH();
    HGX_HIP(hipStreamSynchronize(st));
    root->ylists.push_back(y);
    return &root->ylists.back();
}

void block_materialize(hgx_graph* g, BlockSet& b) {
    if (b.co_host || b.co_idx.empty()) return;
    std::vector<int2> h((size_t)b.co_n);
    size_t o = 0;
    for (size_t q = 0; q < b.co_segn.size(); ++q) {   // each segment's pairs
        const size_t n = (size_t)b.co_segn[q];
        if (n) HGX_HIP(hipMemcpyAsync(h.data() + o, (const int2*)b.co_pairs + q * (size_t)b.co_pseg, sizeof(int2) * n,
                                      hipMemcpyDeviceToHost, g->stream));
        o += n;
    }
    HGX_HIP(hipStreamSynchronize(g->stream));
    const size_t k = b.co_idx.size();
    std::vector<std::vector<int64_t>> pos(k);
    for (size_t j = 0; j < k; ++j) {
        int64_t o = 0;
        for (int32_t c : b.co_lcnt[j]) {
            pos[j].push_back(o);
            o += c;
        }
        b.co_atoms[j].assign((size_t)o, -1);
    }
    for (const int2& pr : h) {
        const size_t j = (size_t)(pr.y & 0xFF);
        const int32_t lev = pr.y >> 8;   // >= 1
        b.co_atoms[j][(size_t)pos[j][lev - 1]++] = pr.x;
    }
    for (size_t j = 0; j < k; ++j) b.atoms[b.co_idx[j]] = b.co_atoms[j].data();
    b.co_host = true;
}

void block_release(hgx_graph* g, BlockSet& b) {
    if (b.co_pairs) g->release(b.co_pairs, b.co_bytes);
    b.co_pairs = nullptr;
    std::lock_guard<std::mutex> lk(g->seq_mu);
    for (auto& x : b.bufs) g->seq_hbufs.push_back(x);
    b.bufs.clear();
}

}  // namespace hgx

using namespace hgx;

// Per seed, where its pairs live: a region of a mapped buffer the workgroup engine wrote, or one
// segment per level of the level-synchronous run's mapped buffers.  The result keeps a reference on
// its graph so the mapped buffers go back to the graph's pool when it is freed.
struct hgx_seq_result {
    int32_t n_seeds = 0;
    int32_t n_levels = 0;           // 1 + deepest distance returned by any seed
    std::vector<int64_t> off;       // [n_seeds + 1]
    std::vector<Seg> blk;           // [n_seeds] the workgroup engine's region (n < 0: level engine)
    std::vector<PoolBuf> hbufs;     // mapped buffers of the workgroup launches (owned until free)
    SeqOut lev;                     // the level-synchronous engine's seeds (indexed by rerun order)
    std::vector<int32_t> lev_of;    // [n_seeds] index into lev.segs, or -1
    hgx_graph* g = nullptr;
    mutable double ms_total = 0;
    double traversed = 0;
    double ms_block = 0, bytes_block = 0;   // the workgroup engine's launches: device ms, algorithmic bytes
    mutable double ms_level = 0;            // the level-synchronous engine: device ms (timing on) ...
    // timing events of a call whose pair copies were still running when it returned (read on first use).
    // settle() runs from the const stats readers and the destructor, possibly from several threads at once
    // (hgx.h: every entry point is thread-safe): the mutex makes the event read + destroy happen once.
    mutable hipEvent_t lz_ev0 = nullptr, lz_ev1 = nullptr, lz_el0 = nullptr, lz_el1 = nullptr;
    mutable std::mutex lz_mu;
    void settle() const {
        std::lock_guard<std::mutex> lk(lz_mu);
        float ms = 0;
        if (lz_el1 && hipEventSynchronize(lz_el1) == hipSuccess && hipEventElapsedTime(&ms, lz_el0, lz_el1) == hipSuccess)
            ms_level = ms;
        if (lz_ev1 && hipEventSynchronize(lz_ev1) == hipSuccess && hipEventElapsedTime(&ms, lz_ev0, lz_ev1) == hipSuccess)
            ms_total = ms;
        for (hipEvent_t* e : {&lz_ev0, &lz_ev1, &lz_el0, &lz_el1})
            if (*e) {
                (void)hipEventDestroy(*e);
                *e = nullptr;
            }
    }
    double ms_coop = 0, bytes_coop = 0;     // the order-exact grid stage (hgx_seq_coop): device ms, algorithmic bytes
    int32_t n_coop = 0;                     //   and the seeds it finished
    int32_t n_block = 0, n_level = 0;       // seeds finished by each engine
    ~hgx_seq_result() {
        if (!g) return;
        settle();
        for (hipEvent_t e : lev.evs) {   // the level buffers' copies must have landed before they are reused
            (void)hipEventSynchronize(e);
            (void)hipEventDestroy(e);
        }
        lev.evs.clear();
        {
            std::lock_guard<std::mutex> lk(g->seq_mu);
            for (auto& b : hbufs) g->seq_hbufs.push_back(b);
            for (auto& b : lev.bufs) g->seq_hbufs.push_back(b);
        }
        hbufs.clear();
        lev.bufs.clear();
        graph_release(g);
    }
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
    SeqTrace trace;
    g_seq_trace = trace.on ? &trace : nullptr;
    struct TraceOff {
        ~TraceOff() { g_seq_trace = nullptr; }
    } trace_off;
    HGX_HIP(hipSetDevice(g->device));
    hipStream_t st = g->stream;
    const int32_t maxd = max_depth < 0 ? INT32_MAX : max_depth;
    const int mode = seq_mode(o);

    hgx_seq_result* r = new hgx_seq_result();
    struct Guard {
        hgx_seq_result* r;
        ~Guard() { delete r; }
    } guard{r};
    r->g = g;
    g->refs.fetch_add(1);
    r->n_seeds = n_seeds;
    r->blk.assign((size_t)n_seeds, Seg{nullptr, nullptr, nullptr, -1, 0});
    r->lev_of.assign((size_t)n_seeds, -1);
    std::vector<int64_t> cnt((size_t)n_seeds, 0);
    seq_maxes(g);
    if (mode != sSym) ensure_inc_yield(g);

    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    if (g->timing) {
        ev0 = ev_take(g);
        ev1 = ev_take(g);
        HGX_HIP(hipEventRecord(ev0, st));
    }
    seq_mark("call set up");
    std::vector<int32_t> rerun;   // seed indices for the level-synchronous engine
    int32_t deepest = 0;
    std::unique_ptr<ScRun> chained;   // the grid stage chained behind the workgroup launches
    if (g->seq_engine == 0 && n_seeds > 0) {
        const int kbits = bitlen(g->max_arity > 1 ? (u64)(g->max_arity - 1) : 0);
        SbArgs a{};
        a.inc_off = g->inc_off;
        a.inc_row = g->inc_row;
        a.inc_type = g->inc_type;
        a.yf = mode != sSym ? g->inc_yf : nullptr;
        const YieldAdj* ya = stage_yield_adj(g, mode, o);
        if (ya) {
            a.y_off = ya->off;
            a.a_tgt = ya->tgt;
            a.a_lnk = ya->lnk;
        } else if (const YieldList* yl = stage_yield_list(g, mode, o.link_type)) {
            a.y_off = yl->off;
            a.y_row = yl->row;
        }
        a.tgt_off = g->tgt_off;
        a.tgt_idx = g->tgt_idx;
        a.link_atom = g->link_atom;
        a.want_type = o.link_type;
        a.min_arity = o.return_source ? 1 : 2;
        a.mode = mode;
        a.rev = o.reverse_order ? 1 : 0;
        a.kbits = ya ? 0 : kbits;   // an adjacency pair's index is its whole stream position
        a.maxd = maxd;
        a.t_limit = std::min<int64_t>(INT32_MAX - 1, (int64_t)(0xFFFFFFFFull >> a.kbits));
        // batches chain the grid stage behind the workgroup launches (no host round trip between the stages);
        // a single traversal (the drop-in's next() shape) keeps its latency without the extra launch
        static const bool chain_off = ab_int("HGX_SEQ_CHAIN", 1) == 0 || ab_int("HGX_SEQ_COOP", 1) == 0;   // A/B builds
        if (!chain_off && ya && n_seeds >= kSeqChainMin && sc_fits(g)) {
            chained.reset(new ScRun(g));
            chained->prepare(ya, maxd, true);
            a.chain = chained->chain_buf;
            a.chain_n = chained->chain_cnt;
        }
        const size_t per_seed = (size_t)kSbPairs * 12 + 24;
        int32_t* dseeds = nullptr;
        size_t dseeds_n = 0;
        if (n_seeds > kSbInline) {
            dseeds_n = sizeof(int32_t) * (size_t)n_seeds;
            dseeds = (int32_t*)g->alloc(dseeds_n);
            int32_t* hs = (int32_t*)g->pinned_buf(dseeds_n);
            std::memcpy(hs, seeds, dseeds_n);
            HGX_HIP(hipMemcpyAsync(dseeds, hs, dseeds_n, hipMemcpyHostToDevice, st));
        }
        struct Chunk {
            int64_t c0, nb;
            char* h;
        };
        std::vector<Chunk> chunks;
        static const bool clk_trace = trace_env("HGX_SB_CLOCK");   // per-seed start / end ticks to stderr
        int64_t* clk = nullptr;
        if (clk_trace) HGX_HIP(hipHostMalloc((void**)&clk, sizeof(int64_t) * 2 * (size_t)n_seeds, hipHostMallocMapped));
        for (int64_t c0 = 0; c0 < n_seeds; c0 += kSbChunk) {
            const int64_t nb = std::min<int64_t>(kSbChunk, n_seeds - c0);
            PoolBuf hb = take_host_buf(g, per_seed * (size_t)nb);
            r->hbufs.push_back(hb);
            char* h = (char*)hb.p;
            void* dv = nullptr;
            HGX_HIP(hipHostGetDevicePointer(&dv, h, 0));
            char* d = (char*)dv;
            // layout: meta [3 nb] int64 | link [nb * kSbPairs] | atom [..] | dist [..]
            a.n = (int32_t)nb;
            a.c0 = (int32_t)c0;
            a.meta = (int64_t*)d;
            a.out_link = (int32_t*)(d + 24 * nb);
            a.out_atom = a.out_link + nb * kSbPairs;
            a.out_dist = a.out_atom + nb * kSbPairs;
            if (nb <= kSbInline) {   // the kernel reads the inline seeds whenever n <= kSbInline
                for (int64_t i = 0; i < nb; ++i) a.seed_inline[i] = seeds[c0 + i];
                a.seeds = nullptr;
            } else {
                a.seeds = dseeds + c0;
            }
            if (clk) {
                void* dc = nullptr;
                HGX_HIP(hipHostGetDevicePointer(&dc, clk + 2 * c0, 0));
                a.clk = (int64_t*)dc;
            }
            hgx_seq_block<<<(unsigned)nb, kSbThreads, 0, st>>>(a);
            HGX_CHECK_LAUNCH();
            chunks.push_back({c0, nb, h});
        }
        hipEvent_t evb = nullptr;
        if (g->timing) {
            evb = ev_take(g);
            HGX_HIP(hipEventRecord(evb, st));
        }
        seq_mark("workgroup stage enqueued");
        if (chained) chained->launch();
        spin_sync(st);
        seq_mark("workgroup stage done");
        if (evb) {
            float ms = 0;
            HGX_HIP(hipEventElapsedTime(&ms, ev0, evb));
            r->ms_block = ms;
            ev_give(g, evb);
        }
        if (dseeds) g->release(dseeds, dseeds_n);
        if (clk) {   // per seed: start after the first start, duration (us), pairs, depth; the 12 last to end
            int64_t t0 = INT64_MAX;
            for (int32_t i = 0; i < n_seeds; ++i) t0 = std::min(t0, clk[2 * i]);
            std::vector<int32_t> ord((size_t)n_seeds);
            for (int32_t i = 0; i < n_seeds; ++i) ord[i] = i;
            std::sort(ord.begin(), ord.end(), [&](int32_t x, int32_t y) { return clk[2 * x + 1] > clk[2 * y + 1]; });
            double sum = 0;
            for (int32_t i = 0; i < n_seeds; ++i) sum += (clk[2 * i + 1] - clk[2 * i]) * 0.01;
            std::fprintf(stderr, "[hgx sb clock] seeds=%d mean_us=%.1f end_us=%.1f; last to end (seed: start/dur us, pairs, depth):",
                         n_seeds, sum / std::max(1, n_seeds), (clk[2 * ord[0] + 1] - t0) * 0.01);
            for (int32_t k = 0; k < std::min<int32_t>(12, n_seeds); ++k) {
                const int32_t i = ord[k];
                const Chunk& c = chunks[(size_t)(i / kSbChunk)];
                const int64_t j = i - c.c0;
                const int64_t np = ((const int64_t*)c.h)[3 * j];
                const int32_t* ds = (const int32_t*)(c.h + 24 * c.nb) + 2 * c.nb * kSbPairs;
                std::fprintf(stderr, " %d: %.1f/%.1f %lld %d;", i, (clk[2 * i] - t0) * 0.01, (clk[2 * i + 1] - clk[2 * i]) * 0.01,
                             (long long)np, np > 0 ? ds[j * kSbPairs + np - 1] : 0);
            }
            std::fprintf(stderr, "\n");
            (void)hipHostFree(clk);
        }
        for (auto& c : chunks) {
            const int64_t* meta = (const int64_t*)c.h;
            const int32_t* lk_ = (const int32_t*)(c.h + 24 * c.nb);
            const int32_t* at = lk_ + c.nb * kSbPairs;
            const int32_t* ds = at + c.nb * kSbPairs;
            for (int64_t i = 0; i < c.nb; ++i) {
                const int64_t np = meta[3 * i];
                const int64_t si = c.c0 + i;
                r->bytes_block += (double)meta[3 * i + 2];
                if (np < 0) {
                    rerun.push_back((int32_t)si);
                    continue;
                }
                cnt[si] = np;
                r->traversed += (double)meta[3 * i + 1];
                r->blk[si] = {lk_ + i * kSbPairs, at + i * kSbPairs, ds + i * kSbPairs, np, 0};
                if (np > 0) deepest = std::max(deepest, ds[i * kSbPairs + np - 1]);
            }
        }
    } else {
        for (int32_t i = 0; i < n_seeds; ++i) rerun.push_back(i);
    }
    r->n_level = (int32_t)rerun.size();
    r->n_block = n_seeds - r->n_level;
    if (!rerun.empty()) {
        std::vector<int32_t> rs(rerun.size());
        for (size_t k = 0; k < rerun.size(); ++k) rs[k] = seeds[rerun[k]];
        hipEvent_t el0 = nullptr, el1 = nullptr;
        if (g->timing) {
            el0 = ev_take(g);
            el1 = ev_take(g);
            HGX_HIP(hipEventRecord(el0, st));
        }
        bool done = false;
        if (chained) {   // the chained grid stage took exactly these seeds (its list, in arrival order)
            const int64_t kk = chained->hm[5];
            if (kk == (int64_t)rerun.size() && kk <= kMaxCoSeeds) {
                std::vector<int32_t> pos((size_t)kk);
                for (int64_t j = 0; j < kk; ++j) {   // list entry j -> its position in rerun (ascending)
                    const int64_t idx = chained->hm[8 + 2 * (size_t)chained->nblk + j];
                    const auto it = std::lower_bound(rerun.begin(), rerun.end(), (int32_t)idx);
                    if (it == rerun.end() || *it != (int32_t)idx) fail(HGX_E_DEVICE, "hgx_bfs_sequence: chained seed list inconsistent");
                    pos[j] = (int32_t)(it - rerun.begin());
                }
                SeqOut co;
                co.segs.assign(rs.size(), {});
                done = chained->collect((int32_t)kk, pos, co, &r->ms_coop) == 1;
                if (done) {
                    r->lev.segs = std::move(co.segs);
                    r->lev.bufs = std::move(co.bufs);
                    r->lev.traversed = co.traversed;
                    r->lev.deepest = co.deepest;
                    r->bytes_coop = co.bytes;
                    r->n_coop = (int32_t)rs.size();
                }
            } else if (chained->hm[0] != 0 || chained->hm[3] != 0) {   // did not run them: state back to empty
                SeqOut co;
                (void)chained->collect(0, {}, co, &r->ms_coop);
            }
            chained.reset();
        }
        if (!done && g->seq_engine == 0 && rs.size() <= (size_t)kMaxCoSeeds) {   // the grid stage first (one launch)
            r->lev.segs.assign(rs.size(), {});
            std::vector<int32_t> sidx(rs.size());
            for (size_t q = 0; q < rs.size(); ++q) sidx[q] = (int32_t)q;
            SeqOut co;
            co.segs.assign(rs.size(), {});
            done = seq_coop(g, rs.data(), sidx, maxd, o, co, &r->ms_coop);
            if (done) {
                r->lev.segs = std::move(co.segs);
                r->lev.bufs = std::move(co.bufs);
                r->lev.traversed = co.traversed;
                r->lev.deepest = co.deepest;
                r->bytes_coop = co.bytes;
                r->n_coop = (int32_t)rs.size();
            } else {
                std::lock_guard<std::mutex> lk(g->seq_mu);
                for (auto& b : co.bufs) g->seq_hbufs.push_back(b);
            }
        }
        if (!done) seq_levels_all(g, rs.data(), (int32_t)rs.size(), maxd, o, r->lev, g->seq_engine != 1);
        if (el0 && !r->lev.evs.empty()) {   // the pair copies are still running: timed on first use
            HGX_HIP(hipEventRecord(el1, st));
            r->lz_el0 = el0;
            r->lz_el1 = el1;
        } else if (el0) {
            HGX_HIP(hipEventRecord(el1, st));
            HGX_HIP(hipEventSynchronize(el1));
            float ms = 0;
            HGX_HIP(hipEventElapsedTime(&ms, el0, el1));
            r->ms_level = ms;
            ev_give(g, el0);
            ev_give(g, el1);
        }
        r->traversed += r->lev.traversed;
        deepest = std::max(deepest, r->lev.deepest);
        for (size_t k = 0; k < rerun.size(); ++k) {
            int64_t n = 0;
            for (const Seg& sg : r->lev.segs[k]) n += sg.n;
            cnt[rerun[k]] = n;
            r->lev_of[rerun[k]] = (int32_t)k;
        }
    }
    if (g->timing && !r->lev.evs.empty()) {
        HGX_HIP(hipEventRecord(ev1, st));
        r->lz_ev0 = ev0;
        r->lz_ev1 = ev1;
    } else if (g->timing) {
        HGX_HIP(hipEventRecord(ev1, st));
        HGX_HIP(hipEventSynchronize(ev1));
        seq_mark("timing event done");
        float ms = 0;
        HGX_HIP(hipEventElapsedTime(&ms, ev0, ev1));
        r->ms_total = ms;
        ev_give(g, ev0);
        ev_give(g, ev1);
    }
    r->off.assign((size_t)n_seeds + 1, 0);
    for (int32_t i = 0; i < n_seeds; ++i) r->off[i + 1] = r->off[i] + cnt[i];
    r->n_levels = deepest + 1;
    seq_mark("call done");
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
    // the copy jobs: one per segment, split into pieces of <= 4M pairs; large results are copied by
    // several host threads (config 2's drop-in call returns 258M pairs: 3 GB of caller arrays whose
    // pages are first touched here)
    struct Job {
        int64_t b;
        const Seg* s;
        int64_t lo, n;
    };
    std::vector<Job> jobs;
    constexpr int64_t kPiece = (int64_t)1 << 22;
    auto add = [&](int64_t b, const Seg& s) {
        for (int64_t lo = 0; lo < s.n; lo += kPiece) jobs.push_back({b, &s, lo, std::min(kPiece, s.n - lo)});
    };
    for (int32_t i = 0; i < r->n_seeds; ++i) {
        int64_t b = r->off[i];
        if (r->lev_of[i] < 0) {
            add(b, r->blk[i]);
            continue;
        }
        for (const Seg& s : r->lev.segs[(size_t)r->lev_of[i]]) {
            add(b, s);
            b += s.n;
        }
    }
    // large caller arrays are usually fresh (their pages first touched by the copy below): ask for
    // transparent huge pages on their 2 MB-aligned interior, 512x fewer page faults where the kernel's THP
    // mode is "madvise" (a hint: no effect under "never", already the case under "always")
    static const bool thp = ab_int("HGX_READOUT_THP", 1) != 0;
    if (thp && r->off.back() >= ((int64_t)1 << 24)) {
        auto hint = [](void* p, size_t bytes) {
            if (!p) return;
            const uintptr_t b = ((uintptr_t)p + (2u << 20) - 1) & ~(uintptr_t)((2u << 20) - 1);
            const uintptr_t e = ((uintptr_t)p + bytes) & ~(uintptr_t)((2u << 20) - 1);
            if (e > b) (void)madvise((void*)b, e - b, MADV_HUGEPAGE);
        };
        const size_t nb = sizeof(int32_t) * (size_t)r->off.back();
        hint(links, nb);
        hint(atoms, nb);
        hint(dists, nb);
    }
    std::atomic<bool> copy_failed{false};
    auto run = [&](const Job& j) {
        const Seg& s = *j.s;
        if (s.ready && hipEventSynchronize(s.ready) != hipSuccess) {   // its copy may still be running
            copy_failed = true;
            return;
        }
        const int64_t o = j.b + j.lo;
        copy_pairs(s, j.lo, j.n, links ? links + o : nullptr, atoms ? atoms + o : nullptr);
        if (dists) {
            if (s.dist) std::memcpy(dists + o, s.dist + j.lo, sizeof(int32_t) * j.n);
            else std::fill(dists + o, dists + o + j.n, s.dist_c);
        }
    };
    host_parallel((int64_t)jobs.size(), r->off.back() >= ((int64_t)1 << 24), [&](int64_t k) { run(jobs[(size_t)k]); });
    if (copy_failed) fail(HGX_E_DEVICE, "hgx_seq_result_pairs: a pair copy failed");
    HGX_API_END
}

int hgx_seq_result_pairs_range(const hgx_seq_result* r, int64_t first, int64_t n, int32_t* links, int32_t* atoms,
                               int32_t* dists, int64_t* n_out) {
    HGX_API_BEGIN
    if (!r || first < 0 || n < 0) fail(HGX_E_INVALID, "hgx_seq_result_pairs_range: bad argument");
    const int64_t total = r->off.back();
    const int64_t hi = std::min(total, first + std::min(n, total));
    if (n_out) *n_out = std::max<int64_t>(hi - first, 0);
    // copy the overlap of every segment with [first, hi)
    auto put = [&](int64_t b, const Seg& s) {
        const int64_t lo_ = std::max(b, first), hi_ = std::min(b + s.n, hi);
        if (hi_ <= lo_) return;
        const int64_t k = hi_ - lo_, so = lo_ - b, o = lo_ - first;
        if (s.ready) HGX_HIP(hipEventSynchronize(s.ready));
        copy_pairs(s, so, k, links ? links + o : nullptr, atoms ? atoms + o : nullptr);
        if (dists) {
            if (s.dist) std::memcpy(dists + o, s.dist + so, sizeof(int32_t) * k);
            else std::fill(dists + o, dists + o + k, s.dist_c);
        }
    };
    if (hi > first) {
        // the first seed whose pairs reach past `first`
        int32_t i0 = (int32_t)(std::upper_bound(r->off.begin(), r->off.end(), first) - r->off.begin()) - 1;
        for (int32_t i = std::max(i0, 0); i < r->n_seeds && r->off[i] < hi; ++i) {
            int64_t b = r->off[i];
            if (r->lev_of[i] < 0) {
                put(b, r->blk[i]);
                continue;
            }
            for (const Seg& sg : r->lev.segs[(size_t)r->lev_of[i]]) {
                put(b, sg);
                b += sg.n;
            }
        }
    }
    HGX_API_END
}

int hgx_seq_result_stats(const hgx_seq_result* r, double* ms_total, double* traversed_edges) {
    HGX_API_BEGIN
    if (!r) fail(HGX_E_INVALID, "null result");
    r->settle();
    if (ms_total) *ms_total = r->ms_total;
    if (traversed_edges) *traversed_edges = r->traversed;
    HGX_API_END
}

int hgx_seq_result_engine_stats(const hgx_seq_result* r, int32_t* n_block, int32_t* n_level, double* ms_block,
                                 double* bytes_block) {
    HGX_API_BEGIN
    if (!r) fail(HGX_E_INVALID, "null result");
    if (n_block) *n_block = r->n_block;
    if (n_level) *n_level = r->n_level;
    if (ms_block) *ms_block = r->ms_block;
    if (bytes_block) *bytes_block = r->bytes_block;
    HGX_API_END
}

int hgx_seq_result_grid_stats(const hgx_seq_result* r, int32_t* n_seeds, double* ms, double* bytes) {
    HGX_API_BEGIN
    if (!r) fail(HGX_E_INVALID, "null result");
    if (n_seeds) *n_seeds = r->n_coop;
    if (ms) *ms = r->ms_coop;
    if (bytes) *bytes = r->bytes_coop;
    HGX_API_END
}

int hgx_seq_result_level_stats(const hgx_seq_result* r, double* ms_level, double* bytes_level, int64_t* pull_levels) {
    HGX_API_BEGIN
    if (!r) fail(HGX_E_INVALID, "null result");
    r->settle();
    if (ms_level) *ms_level = r->ms_level;
    if (bytes_level) *bytes_level = r->lev.bytes;
    if (pull_levels) *pull_levels = r->lev.pull_levels;
    HGX_API_END
}

void hgx_seq_result_free(hgx_seq_result* r) { delete r; }

}  // extern "C"
