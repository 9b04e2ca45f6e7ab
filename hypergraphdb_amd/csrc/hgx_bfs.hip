// hgx_bfs.hip -- batched multi-source breadth-first traversal over the bipartite CSR.
//
// Replaces HGBreadthFirstTraversal (C/algorithms/HGBreadthFirstTraversal.java:29-164) driven by
// DefaultALGenerator (C/algorithms/DefaultALGenerator.java:73-593) for S <= 1024 start atoms at
// once.  The per-depth visited sets V_d (the atoms next() returns at distance d) are computed
// level-synchronously with one bit per start atom:
//
//   lvl_d[v]  : S-bit row, bit s set <=> v is returned at distance d by traversal s
//   vis[v]    : OR of lvl_0..lvl_d (the reference's 'examined' map, per traversal)
//   lf[L]     : S-bit row of link L = OR of lvl_d over L's targets              (link gather)
//   lvl_d+1[t]: (OR over L in inc(t) of lf[L]) & ~vis[t]                         (atom pull)
//
// In the default generator mode (returnPreceeding = returnSucceeding = true) the neighbours of v
// are every co-target of every incident link except v itself (DefaultALGenerator.java:149-203),
// which is exactly lf/pull above; v itself is removed by ~vis because v is visited for every bit
// of its own frontier row.  Ordered modes (succeeding-only / reverse, used by hg.subsumed /
// hg.subsumes, C/query/cond2qry/ToQueryMap.java:282-370) use the position rule of DESIGN.md 3.2
// inside the pull instead of lf.  Rows are only read behind per-level activity bitmaps, so a
// sparse level costs the CSR scan, not the full mask traffic.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstring>
#include <map>

#include "hgx_internal.h"

namespace hgx {

typedef unsigned long long u64;
typedef u64 u64x2 __attribute__((ext_vector_type(2)));

enum Mode { kSym = 0, kAfterFirst = 1, kBeforeFirst = 2, kBeforeLast = 3, kAfterLast = 4 };

// Mirrors pyref.mode_of (validated exhaustively against the DefaultALGenerator restatement).
static int mode_of(const hgx_algen_opts& o) {
    bool P = o.return_preceding, S = o.return_succeeding, R = o.reverse_order, RS = o.return_source;
    if (!R) {
        if (!P) return kAfterFirst;
        if (!S && !RS) return kBeforeFirst;
        return kSym;
    }
    if (!P) return kBeforeLast;
    if (!S && !RS) return kAfterLast;
    return kSym;
}

// W words of 64 bits per row; each lane of a G-lane group holds WPL words (16 B loads for W >= 2).
template <int W> struct Lay {
    static constexpr int WPL = W >= 2 ? 2 : 1;
    static constexpr int G = W / WPL;
};

template <int WPL> struct Vec;
template <> struct Vec<1> {
    typedef u64 T;
    static __device__ __forceinline__ T zero() { return 0ull; }
    static __device__ __forceinline__ bool nz(T x) { return x != 0ull; }
    static __device__ __forceinline__ T ld(const u64* p) { return *p; }
    static __device__ __forceinline__ void st(u64* p, T x) { *p = x; }
    static __device__ __forceinline__ int pop(T x) { return __popcll(x); }
};
template <> struct Vec<2> {
    typedef u64x2 T;
    static __device__ __forceinline__ T zero() { return u64x2{0ull, 0ull}; }
    static __device__ __forceinline__ bool nz(T x) { return (x.x | x.y) != 0ull; }
    static __device__ __forceinline__ T ld(const u64* p) { return *reinterpret_cast<const u64x2*>(p); }
    static __device__ __forceinline__ void st(u64* p, T x) { *reinterpret_cast<u64x2*>(p) = x; }
    static __device__ __forceinline__ int pop(T x) { return __popcll(x.x) + __popcll(x.y); }
};

__device__ __forceinline__ bool bit(const uint32_t* __restrict__ bm, int64_t i) {
    return (bm[i >> 5] >> (i & 31)) & 1u;
}
__device__ __forceinline__ void set_bit(uint32_t* bm, int64_t i) { atomicOr(&bm[i >> 5], 1u << (i & 31)); }

// true if predicate holds on any lane of this lane's G-lane group (groups are G-aligned in the wave).
template <int G> __device__ __forceinline__ bool group_any(bool p) {
    if constexpr (G == 1) {
        return p;
    } else {
        u64 b = __ballot(p);
        int base = (threadIdx.x & 63) & ~(G - 1);
        return ((b >> base) & ((1ull << G) - 1ull)) != 0ull;
    }
}

// per-level counters (device), used for the early stop and for the byte accounting
enum Ctr {
    cActiveLinks = 0,   // links whose lf row is nonzero                      (link gather)
    cActivePins,        // (link, target) pairs whose target row was gathered (link gather)
    cIncLight,          // incidence entries with an active link, light atoms (atom pull)
    cAccLight,          // light atoms with a nonzero pull result (vis read)
    cNewLight,          // light atoms with a new bit (lvl + vis written)
    cIncHeavy,          // incidence entries with an active link, heavy chunks
    cAccHub,            // heavy atoms with a nonzero pull result
    cNewHub,            // heavy atoms with a new bit
    cNewAtoms,          // all new atoms of the level (early stop)
    cNum = 10
};

__device__ __forceinline__ void wave_add(u64* ctr, u64 v) {
    // one atomic per wave: sum over lanes via DPP-free shuffles
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(ctr, v);
}

// ---------------------------------------------------------------------------------------------
// Link gather: lf[L] = OR_{v in targets(L), fa_d(v)} lvl_d[v]; la(L) set iff any target active.
// One G-lane group per link row, grid-stride.  WRITE_LF = false in the ordered modes.
// ---------------------------------------------------------------------------------------------
template <int W, bool WRITE_LF>
__global__ void __launch_bounds__(256) hgx_link_gather(int64_t M, const int64_t* __restrict__ tgt_off,
                                                       const int32_t* __restrict__ tgt_idx,
                                                       const int32_t* __restrict__ link_type, int32_t want_type,
                                                       const uint32_t* __restrict__ fa,
                                                       const u64* __restrict__ lvl, u64* __restrict__ lf,
                                                       uint32_t* __restrict__ la, u64* __restrict__ ctr) {
    constexpr int WPL = Lay<W>::WPL, G = Lay<W>::G;
    typedef Vec<WPL> V;
    const int sub = threadIdx.x & (G - 1);
    const int64_t grp = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / G;
    const int64_t ngrp = ((int64_t)gridDim.x * blockDim.x) / G;
    u64 n_links = 0, n_pins = 0;
    for (int64_t L = grp; L < M; L += ngrp) {
        if (want_type >= 0 && link_type[L] != want_type) continue;
        const int64_t b = tgt_off[L], e = tgt_off[L + 1];
        typename V::T acc = V::zero();
        int nact = 0;
        int64_t p = b;
        for (; p + 4 <= e; p += 4) {
            int32_t v0 = tgt_idx[p], v1 = tgt_idx[p + 1], v2 = tgt_idx[p + 2], v3 = tgt_idx[p + 3];
            bool a0 = bit(fa, v0), a1 = bit(fa, v1), a2 = bit(fa, v2), a3 = bit(fa, v3);
            if (a0) acc |= V::ld(lvl + (int64_t)v0 * W + sub * WPL);
            if (a1) acc |= V::ld(lvl + (int64_t)v1 * W + sub * WPL);
            if (a2) acc |= V::ld(lvl + (int64_t)v2 * W + sub * WPL);
            if (a3) acc |= V::ld(lvl + (int64_t)v3 * W + sub * WPL);
            nact += (int)a0 + (int)a1 + (int)a2 + (int)a3;
        }
        for (; p < e; ++p) {
            int32_t v = tgt_idx[p];
            if (bit(fa, v)) {
                acc |= V::ld(lvl + (int64_t)v * W + sub * WPL);
                ++nact;
            }
        }
        if (nact) {
            if (WRITE_LF) V::st(lf + L * W + sub * WPL, acc);
            if (sub == 0) {
                set_bit(la, L);
                ++n_links;
                n_pins += nact;
            }
        }
    }
    wave_add(ctr + cActiveLinks, n_links);
    wave_add(ctr + cActivePins, n_pins);
}

// Ordered modes: the frontier rows of the co-targets of t in link row Lr that may yield t.
template <int W, int MODE>
__device__ __forceinline__ typename Vec<Lay<W>::WPL>::T pull_ordered(int32_t t, int64_t b, int64_t e,
                                                                      const int32_t* __restrict__ tgt_idx,
                                                                      const uint32_t* __restrict__ fa,
                                                                      const u64* __restrict__ lvl, int sub) {
    constexpr int WPL = Lay<W>::WPL;
    typedef Vec<WPL> V;
    typename V::T acc = V::zero();
    const int n = (int)(e - b);
    int ft = -1, lt = -1;
    for (int i = 0; i < n; ++i)
        if (tgt_idx[b + i] == t) {
            if (ft < 0) ft = i;
            lt = i;
        }
    for (int i = 0; i < n; ++i) {
        int32_t v = tgt_idx[b + i];
        if (v == t || !bit(fa, v)) continue;
        int fv = -1, lv = -1;
        for (int j = 0; j < n; ++j)
            if (tgt_idx[b + j] == v) {
                if (fv < 0) fv = j;
                lv = j;
            }
        if (fv != i) continue;   // evaluate each distinct co-target once
        bool ok;
        if constexpr (MODE == kAfterFirst) ok = lt > fv;        // yields positions after first(v)
        else if constexpr (MODE == kBeforeFirst) ok = ft < fv;  // positions before first(v)
        else if constexpr (MODE == kBeforeLast) ok = ft < lv;   // reverse: before last(v)
        else ok = lt > lv;                                      // reverse, !succeeding: after last(v)
        if (ok) acc |= V::ld(lvl + (int64_t)v * W + sub * WPL);
    }
    return acc;
}

// Accumulate the pull of incidence entries [b, e) of atom t.
template <int W, int MODE>
__device__ __forceinline__ typename Vec<Lay<W>::WPL>::T pull_range(
    int32_t t, int64_t b, int64_t e, const int32_t* __restrict__ inc_row, const uint32_t* __restrict__ la,
    const u64* __restrict__ lf, const int64_t* __restrict__ tgt_off, const int32_t* __restrict__ tgt_idx,
    const uint32_t* __restrict__ fa, const u64* __restrict__ lvl, int sub, u64& n_inc) {
    constexpr int WPL = Lay<W>::WPL;
    typedef Vec<WPL> V;
    typename V::T acc = V::zero();
    int64_t i = b;
    if constexpr (MODE == kSym) {
        for (; i + 8 <= e; i += 8) {
            int32_t L[8];
            bool act[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) L[k] = inc_row[i + k];
#pragma unroll
            for (int k = 0; k < 8; ++k) act[k] = bit(la, L[k]);
#pragma unroll
            for (int k = 0; k < 8; ++k)
                if (act[k]) {
                    acc |= V::ld(lf + (int64_t)L[k] * W + sub * WPL);
                    ++n_inc;
                }
        }
        for (; i < e; ++i) {
            int32_t L = inc_row[i];
            if (bit(la, L)) {
                acc |= V::ld(lf + (int64_t)L * W + sub * WPL);
                ++n_inc;
            }
        }
    } else {
        for (; i < e; ++i) {
            int32_t L = inc_row[i];
            if (bit(la, L)) {
                acc |= pull_ordered<W, MODE>(t, tgt_off[L], tgt_off[L + 1], tgt_idx, fa, lvl, sub);
                ++n_inc;
            }
        }
    }
    return acc;
}

// new = acc & ~vis[t]; write lvl_next/vis/fa_next/ever (owner of t only).
template <int W>
__device__ __forceinline__ void finalize(int64_t t, typename Vec<Lay<W>::WPL>::T acc, int sub,
                                         u64* __restrict__ vis, uint32_t* __restrict__ ever,
                                         u64* __restrict__ lvl_next, uint32_t* __restrict__ fa_next,
                                         u64& n_acc, u64& n_new) {
    constexpr int WPL = Lay<W>::WPL, G = Lay<W>::G;
    typedef Vec<WPL> V;
    if (!group_any<G>(V::nz(acc))) return;
    const bool ev = bit(ever, t);
    typename V::T old = ev ? V::ld(vis + t * W + sub * WPL) : V::zero();
    typename V::T nw = acc & ~old;
    if (sub == 0) ++n_acc;
    if (!group_any<G>(V::nz(nw))) return;
    V::st(lvl_next + t * W + sub * WPL, nw);
    V::st(vis + t * W + sub * WPL, old | nw);
    if (sub == 0) {
        set_bit(fa_next, t);
        if (!ev) set_bit(ever, t);
        ++n_new;
    }
}

// Atom pull for light atoms (deg <= kHeavyDegree): one G-lane group per atom.
template <int W, int MODE>
__global__ void __launch_bounds__(256) hgx_atom_pull(int64_t A, const int64_t* __restrict__ inc_off,
                                                     const int32_t* __restrict__ inc_row,
                                                     const uint32_t* __restrict__ la, const u64* __restrict__ lf,
                                                     const int64_t* __restrict__ tgt_off,
                                                     const int32_t* __restrict__ tgt_idx,
                                                     const uint32_t* __restrict__ fa, const u64* __restrict__ lvl,
                                                     u64* __restrict__ vis, uint32_t* __restrict__ ever,
                                                     u64* __restrict__ lvl_next, uint32_t* __restrict__ fa_next,
                                                     u64* __restrict__ ctr) {
    constexpr int G = Lay<W>::G;
    const int sub = threadIdx.x & (G - 1);
    const int64_t grp = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / G;
    const int64_t ngrp = ((int64_t)gridDim.x * blockDim.x) / G;
    u64 n_inc = 0, n_acc = 0, n_new = 0;
    for (int64_t t = grp; t < A; t += ngrp) {
        const int64_t b = inc_off[t], e = inc_off[t + 1];
        if (e == b || e - b > kHeavyDegree) continue;
        auto acc = pull_range<W, MODE>((int32_t)t, b, e, inc_row, la, lf, tgt_off, tgt_idx, fa, lvl, sub, n_inc);
        finalize<W>(t, acc, sub, vis, ever, lvl_next, fa_next, n_acc, n_new);
    }
    if (sub != 0) n_inc = 0;
    wave_add(ctr + cIncLight, n_inc);
    wave_add(ctr + cAccLight, n_acc);
    wave_add(ctr + cNewLight, n_new);
    wave_add(ctr + cNewAtoms, n_new);
}

// Heavy atoms: one workgroup per chunk of <= kChunkEntries incidence entries; groups OR their
// share, the block reduces through LDS and ORs the chunk result into hubacc[slot].
template <int W, int MODE>
__global__ void __launch_bounds__(256) hgx_atom_pull_heavy(const HeavyChunk* __restrict__ chunks,
                                                           const int32_t* __restrict__ inc_row,
                                                           const uint32_t* __restrict__ la,
                                                           const u64* __restrict__ lf,
                                                           const int64_t* __restrict__ tgt_off,
                                                           const int32_t* __restrict__ tgt_idx,
                                                           const uint32_t* __restrict__ fa,
                                                           const u64* __restrict__ lvl, u64* __restrict__ hubacc,
                                                           u64* __restrict__ ctr) {
    constexpr int WPL = Lay<W>::WPL, G = Lay<W>::G;
    constexpr int NG = 256 / G;
    typedef Vec<WPL> V;
    __shared__ u64 red[NG * W];
    const HeavyChunk c = chunks[blockIdx.x];
    const int sub = threadIdx.x & (G - 1);
    const int gi = threadIdx.x / G;
    const int64_t n = c.end - c.beg;
    const int64_t per = (n + NG - 1) / NG;
    const int64_t b = c.beg + gi * per;
    const int64_t e = b + per < c.end ? b + per : c.end;
    u64 n_inc = 0;
    typename V::T acc = V::zero();
    if (b < e) acc = pull_range<W, MODE>(c.atom, b, e, inc_row, la, lf, tgt_off, tgt_idx, fa, lvl, sub, n_inc);
    V::st(red + gi * W + sub * WPL, acc);
    __syncthreads();
    for (int j = threadIdx.x; j < W; j += 256) {
        u64 r = 0;
        for (int k = 0; k < NG; ++k) r |= red[k * W + j];
        if (r) atomicOr(hubacc + (int64_t)c.slot * W + j, r);
    }
    if (sub != 0) n_inc = 0;
    wave_add(ctr + cIncHeavy, n_inc);
}

template <int W>
__global__ void __launch_bounds__(256) hgx_hub_finalize(int64_t H, const int32_t* __restrict__ heavy_atom,
                                                        u64* __restrict__ hubacc, u64* __restrict__ vis,
                                                        uint32_t* __restrict__ ever, u64* __restrict__ lvl_next,
                                                        uint32_t* __restrict__ fa_next, u64* __restrict__ ctr) {
    constexpr int WPL = Lay<W>::WPL, G = Lay<W>::G;
    typedef Vec<WPL> V;
    const int sub = threadIdx.x & (G - 1);
    const int64_t grp = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / G;
    const int64_t ngrp = ((int64_t)gridDim.x * blockDim.x) / G;
    u64 n_acc = 0, n_new = 0;
    for (int64_t h = grp; h < H; h += ngrp) {
        typename V::T acc = V::ld(hubacc + h * W + sub * WPL);
        V::st(hubacc + h * W + sub * WPL, V::zero());
        finalize<W>(heavy_atom[h], acc, sub, vis, ever, lvl_next, fa_next, n_acc, n_new);
    }
    wave_add(ctr + cAccHub, n_acc);
    wave_add(ctr + cNewHub, n_new);
    wave_add(ctr + cNewAtoms, n_new);
}

// Level 0: seed rows.  rows[i*W ..] is the mask row of unique seed atom atoms[i].
template <int W>
__global__ void hgx_seed(int32_t n, const int32_t* __restrict__ atoms, const u64* __restrict__ rows,
                         u64* __restrict__ lvl0, u64* __restrict__ vis, uint32_t* __restrict__ fa0,
                         uint32_t* __restrict__ ever) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n * W) return;
    int k = i / W, w = i % W;
    int64_t a = atoms[k];
    u64 r = rows[(int64_t)k * W + w];
    lvl0[a * W + w] = r;
    vis[a * W + w] = r;
    if (w == 0) {
        set_bit(fa0, a);
        set_bit(ever, a);
    }
}

// ---------------------------------------------------------------------------------------------
// Result extraction / accounting (not on the timed path)
// ---------------------------------------------------------------------------------------------

// Bit-sliced per-source counts of one level: counts[w*64 + b] += |{v : bit b of lvl[v][w]}|.
// Also traversed += sum_v popcount(lvl[v]) * deg(v) (the hyperedge TEPS numerator).
template <int W>
__global__ void __launch_bounds__(256) hgx_level_count(int64_t A, const uint32_t* __restrict__ fa,
                                                       const u64* __restrict__ lvl,
                                                       const int64_t* __restrict__ inc_off,
                                                       u64* __restrict__ counts, u64* __restrict__ traversed) {
    constexpr int K = 22;   // planes: < 4M atoms per thread (grid chosen by the host)
    __shared__ unsigned int lc[W * 64];
    for (int j = threadIdx.x; j < W * 64; j += 256) lc[j] = 0;
    __syncthreads();
    const int w = threadIdx.x % W;
    const int slot = threadIdx.x / W;
    const int per_block = 256 / W;
    u64 c[K];
#pragma unroll
    for (int k = 0; k < K; ++k) c[k] = 0;
    u64 trav = 0;
    for (int64_t v = blockIdx.x * (int64_t)per_block + slot; v < A; v += (int64_t)gridDim.x * per_block) {
        if (!bit(fa, v)) continue;
        u64 x = lvl[v * W + w];
        trav += (u64)__popcll(x) * (u64)(inc_off[v + 1] - inc_off[v]);
        u64 carry = x;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            u64 tk = c[k] & carry;
            c[k] ^= carry;
            carry = tk;
        }
    }
    for (int b = 0; b < 64; ++b) {
        unsigned int n = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) n |= (unsigned int)((c[k] >> b) & 1ull) << k;
        if (n) atomicAdd(&lc[w * 64 + b], n);
    }
    wave_add(traversed, trav);
    __syncthreads();
    for (int j = threadIdx.x; j < W * 64; j += 256)
        if (lc[j]) atomicAdd(&counts[j], (u64)lc[j]);
}

// Compaction of {v : fa(v) && bit s of lvl[v]} in ascending order.  Pass 1 (write = false)
// counts per block; pass 2 writes at the block's exclusive offset.  Each block owns the
// contiguous atom range [blk*span, (blk+1)*span).
__global__ void __launch_bounds__(256) hgx_extract(int64_t A, int64_t span, int W, int s,
                                                   const uint32_t* __restrict__ fa, const u64* __restrict__ lvl,
                                                   const int64_t* __restrict__ blk_off, int64_t* __restrict__ blk_cnt,
                                                   int32_t* __restrict__ out, int64_t cap, bool write) {
    __shared__ int64_t wave_tot[4];
    __shared__ int64_t run;
    if (threadIdx.x == 0) run = write ? blk_off[blockIdx.x] : 0;
    __syncthreads();
    const int64_t lo = blockIdx.x * span, hi = lo + span < A ? lo + span : A;
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int64_t base = lo; base < hi; base += 256) {
        int64_t v = base + threadIdx.x;
        bool hit = v < hi && bit(fa, v) && ((lvl[v * W + (s >> 6)] >> (s & 63)) & 1ull);
        u64 m = __ballot(hit);
        int before = __popcll(m & ((1ull << lane) - 1ull));
        if (lane == 0) wave_tot[wid] = __popcll(m);
        __syncthreads();
        int64_t wbase = run;
        for (int k = 0; k < wid; ++k) wbase += wave_tot[k];
        if (write && hit) {
            int64_t pos = wbase + before;
            if (pos < cap) out[pos] = (int32_t)v;
        }
        __syncthreads();
        if (threadIdx.x == 0) run += wave_tot[0] + wave_tot[1] + wave_tot[2] + wave_tot[3];
        __syncthreads();
    }
    if (!write && threadIdx.x == 0) blk_cnt[blockIdx.x] = run;
}

// |U_d|, sum deg(v), P_d = sum_{v in U_d} sum_{L in inc v} arity(L)  
__global__ void __launch_bounds__(256) hgx_level_survey(int64_t A, const uint32_t* __restrict__ fa,
                                                        const int64_t* __restrict__ inc_off,
                                                        const int32_t* __restrict__ inc_row,
                                                        const int64_t* __restrict__ tgt_off, u64* __restrict__ out) {
    u64 nu = 0, sd = 0, pd = 0;
    for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < A; v += (int64_t)gridDim.x * blockDim.x) {
        if (!bit(fa, v)) continue;
        ++nu;
        const int64_t b = inc_off[v], e = inc_off[v + 1];
        sd += (u64)(e - b);
        for (int64_t i = b; i < e; ++i) {
            int32_t L = inc_row[i];
            pd += (u64)(tgt_off[L + 1] - tgt_off[L]);
        }
    }
    wave_add(out + 0, nu);
    wave_add(out + 1, sd);
    wave_add(out + 2, pd);
}

__global__ void hgx_depth_probe(int32_t nlev, const uint32_t* const* __restrict__ fa,
                                const u64* const* __restrict__ lvl, int W, int s, int64_t atom,
                                int32_t* __restrict__ out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    int32_t d = -1;
    for (int k = 0; k < nlev && d < 0; ++k)
        if (bit(fa[k], atom) && ((lvl[k][atom * W + (s >> 6)] >> (s & 63)) & 1ull)) d = k;
    *out = d;
}

}  // namespace hgx

using namespace hgx;

// ---------------------------------------------------------------------------------------------
// Host orchestration
// ---------------------------------------------------------------------------------------------

struct BfsBatch {
    int32_t seed0 = 0, S = 0, W = 0;
    int32_t n_expanded = 0;       // levels whose frontier was expanded (advance() iterated)
    std::vector<u64*> lvl;        // per level, A*W words (rows valid where fa bit set)
    std::vector<uint32_t*> fa;    // per level, A bits
    std::vector<int64_t> counts;  // [S * n_levels] after hgx_bfs_result_counts
};

struct hgx_bfs_result {
    hgx_graph* g = nullptr;
    int32_t n_seeds = 0, n_levels = 0;
    std::vector<BfsBatch> batches;
    hgx_bfs_stats stats{};
    bool counts_ready = false;
    bool typed = false;
    std::vector<int64_t> counts;   // [n_seeds * n_levels]
    size_t row_bytes(const BfsBatch& b) const { return sizeof(u64) * (size_t)g->A * b.W; }
    size_t bm_bytes() const { return sizeof(uint32_t) * (size_t)(g->A / 32 + 2); }
};

namespace {

struct Events {
    hipEvent_t a = nullptr, b = nullptr;
};

// Launch helper that brackets a kernel with events when timing is on.
struct Timer {
    hgx_graph* g;
    std::vector<std::pair<int, Events>> rec;   // (kind, events)
    Events begin_all{}, end_all{};
    bool on;
    explicit Timer(hgx_graph* gg) : g(gg), on(gg->timing) {
        if (on) {
            HGX_HIP(hipEventCreate(&begin_all.a));
            HGX_HIP(hipEventCreate(&end_all.a));
        }
    }
    ~Timer() {
        for (auto& r : rec) {
            (void)hipEventDestroy(r.second.a);
            (void)hipEventDestroy(r.second.b);
        }
        if (begin_all.a) (void)hipEventDestroy(begin_all.a);
        if (end_all.a) (void)hipEventDestroy(end_all.a);
    }
    Events start(int kind) {
        Events e{};
        if (!on) return e;
        HGX_HIP(hipEventCreate(&e.a));
        HGX_HIP(hipEventCreate(&e.b));
        HGX_HIP(hipEventRecord(e.a, g->stream));
        rec.push_back({kind, e});
        return e;
    }
    void stop(const Events& e) {
        if (on) HGX_HIP(hipEventRecord(e.b, g->stream));
    }
    double total(int kind) {
        double t = 0;
        for (auto& r : rec)
            if (r.first == kind) {
                float ms = 0;
                HGX_HIP(hipEventElapsedTime(&ms, r.second.a, r.second.b));
                t += ms;
            }
        return t;
    }
};

enum { kKindGather = HGX_K_LINK_GATHER, kKindPull = HGX_K_ATOM_PULL, kKindHeavy = HGX_K_PULL_HEAVY,
       kKindHub = HGX_K_HUB_FINALIZE };

template <int W, int MODE>
void run_levels(hgx_graph* g, hgx_bfs_result* res, BfsBatch& bt, int32_t max_depth, int32_t want_type,
                const std::vector<int32_t>& seed_atoms, const std::vector<u64>& seed_rows, Timer& tm,
                std::vector<std::vector<u64>>& level_ctr) {
    hipStream_t s = g->stream;
    const int64_t A = g->A, M = g->M;
    const size_t row_bytes = sizeof(u64) * (size_t)A * W;
    const size_t bm_bytes = res->bm_bytes();
    const size_t la_bytes = sizeof(uint32_t) * (size_t)(M / 32 + 2);

    u64* vis = (u64*)g->alloc(row_bytes);
    u64* lf = (MODE == kSym) ? (u64*)g->alloc(sizeof(u64) * (size_t)std::max<int64_t>(M, 1) * W) : nullptr;
    u64* hubacc = (u64*)g->alloc(sizeof(u64) * (size_t)std::max<int64_t>(g->n_heavy, 1) * W);
    uint32_t* ever = (uint32_t*)g->alloc(bm_bytes);
    uint32_t* la = (uint32_t*)g->alloc(la_bytes);
    const int max_levels_cap = 4096;
    u64* ctr = (u64*)g->alloc(sizeof(u64) * cNum * max_levels_cap);
    int32_t* d_atoms = (int32_t*)g->alloc(sizeof(int32_t) * seed_atoms.size());
    u64* d_rows = (u64*)g->alloc(sizeof(u64) * seed_rows.size());
    u64* h_new = (u64*)g->pinned_buf(sizeof(u64) * cNum);

    HGX_HIP(hipMemsetAsync(ever, 0, bm_bytes, s));
    HGX_HIP(hipMemsetAsync(hubacc, 0, sizeof(u64) * (size_t)std::max<int64_t>(g->n_heavy, 1) * W, s));
    HGX_HIP(hipMemsetAsync(ctr, 0, sizeof(u64) * cNum * max_levels_cap, s));
    HGX_HIP(hipMemcpyAsync(d_atoms, seed_atoms.data(), sizeof(int32_t) * seed_atoms.size(), hipMemcpyHostToDevice, s));
    HGX_HIP(hipMemcpyAsync(d_rows, seed_rows.data(), sizeof(u64) * seed_rows.size(), hipMemcpyHostToDevice, s));

    bt.lvl.push_back((u64*)g->alloc(row_bytes));
    bt.fa.push_back((uint32_t*)g->alloc(bm_bytes));
    HGX_HIP(hipMemsetAsync(bt.fa[0], 0, bm_bytes, s));
    {
        int n = (int)seed_atoms.size();
        hgx_seed<W><<<grid_for((int64_t)n * W, 256, 1 << 20), 256, 0, s>>>(n, d_atoms, d_rows, bt.lvl[0], vis,
                                                                           bt.fa[0], ever);
        HGX_CHECK_LAUNCH();
    }

    const int block = 256;
    const int gather_grid = grid_for(M * Lay<W>::G, block, 256 * 16);
    const int pull_grid = grid_for(A * Lay<W>::G, block, 256 * 16);
    const int hub_grid = grid_for(std::max<int64_t>(g->n_heavy, 1) * Lay<W>::G, block, 256 * 16);
    const int32_t maxd = max_depth < 0 ? INT32_MAX : max_depth;

    for (int32_t d = 0; d < maxd && d < max_levels_cap - 1; ++d) {
        u64* lvl = bt.lvl[d];
        uint32_t* fa = bt.fa[d];
        u64* lvl_next = (u64*)g->alloc(row_bytes);
        uint32_t* fa_next = (uint32_t*)g->alloc(bm_bytes);
        u64* c = ctr + (size_t)d * cNum;
        HGX_HIP(hipMemsetAsync(la, 0, la_bytes, s));
        HGX_HIP(hipMemsetAsync(fa_next, 0, bm_bytes, s));

        Events e1 = tm.start(kKindGather);
        hgx_link_gather<W, MODE == kSym><<<gather_grid, block, 0, s>>>(M, g->tgt_off, g->tgt_idx, g->link_type,
                                                                      want_type, fa, lvl, lf, la, c);
        HGX_CHECK_LAUNCH();
        tm.stop(e1);
        Events e2 = tm.start(kKindPull);
        hgx_atom_pull<W, MODE><<<pull_grid, block, 0, s>>>(A, g->inc_off, g->inc_row, la, lf, g->tgt_off,
                                                           g->tgt_idx, fa, lvl, vis, ever, lvl_next, fa_next, c);
        HGX_CHECK_LAUNCH();
        tm.stop(e2);
        if (g->n_chunks > 0) {
            Events e3 = tm.start(kKindHeavy);
            hgx_atom_pull_heavy<W, MODE><<<(unsigned)g->n_chunks, block, 0, s>>>(
                g->chunks, g->inc_row, la, lf, g->tgt_off, g->tgt_idx, fa, lvl, hubacc, c);
            HGX_CHECK_LAUNCH();
            tm.stop(e3);
            Events e4 = tm.start(kKindHub);
            hgx_hub_finalize<W><<<hub_grid, block, 0, s>>>(g->n_heavy, g->heavy_atom, hubacc, vis, ever, lvl_next,
                                                           fa_next, c);
            HGX_CHECK_LAUNCH();
            tm.stop(e4);
        }
        HGX_HIP(hipMemcpyAsync(h_new, c, sizeof(u64) * cNum, hipMemcpyDeviceToHost, s));
        HGX_HIP(hipStreamSynchronize(s));
        level_ctr.push_back(std::vector<u64>(h_new, h_new + cNum));
        if (h_new[cNewAtoms] == 0) {
            g->release(lvl_next, row_bytes);
            g->release(fa_next, bm_bytes);
            break;
        }
        bt.lvl.push_back(lvl_next);
        bt.fa.push_back(fa_next);
    }
    g->release(vis, row_bytes);
    if (lf) g->release(lf, sizeof(u64) * (size_t)std::max<int64_t>(M, 1) * W);
    g->release(hubacc, sizeof(u64) * (size_t)std::max<int64_t>(g->n_heavy, 1) * W);
    g->release(ever, bm_bytes);
    g->release(la, la_bytes);
    g->release(ctr, sizeof(u64) * cNum * max_levels_cap);
    g->release(d_atoms, sizeof(int32_t) * seed_atoms.size());
    g->release(d_rows, sizeof(u64) * seed_rows.size());
}

template <int W>
void run_mode(int mode, hgx_graph* g, hgx_bfs_result* res, BfsBatch& bt, int32_t max_depth, int32_t want_type,
              const std::vector<int32_t>& sa, const std::vector<u64>& sr, Timer& tm,
              std::vector<std::vector<u64>>& lc) {
    switch (mode) {
        case kSym: run_levels<W, kSym>(g, res, bt, max_depth, want_type, sa, sr, tm, lc); break;
        case kAfterFirst: run_levels<W, kAfterFirst>(g, res, bt, max_depth, want_type, sa, sr, tm, lc); break;
        case kBeforeFirst: run_levels<W, kBeforeFirst>(g, res, bt, max_depth, want_type, sa, sr, tm, lc); break;
        case kBeforeLast: run_levels<W, kBeforeLast>(g, res, bt, max_depth, want_type, sa, sr, tm, lc); break;
        default: run_levels<W, kAfterLast>(g, res, bt, max_depth, want_type, sa, sr, tm, lc); break;
    }
}

int words_for(int S) {
    int w = (S + 63) / 64;
    int W = 1;
    while (W < w) W <<= 1;
    return W;
}

template <int W>
void count_level(hgx_graph* g, const uint32_t* fa, const u64* lvl, u64* counts, u64* trav) {
    const int per_block = 256 / W;
    int64_t blocks = ceil_div(g->A, per_block);
    // keep atoms per thread < 2^22 (bit-sliced planes)
    int grid = (int)std::min<int64_t>(blocks, 8192);
    hgx_level_count<W><<<std::max(grid, 1), 256, 0, g->stream>>>(g->A, fa, lvl, g->inc_off, counts, trav);
    HGX_CHECK_LAUNCH();
}

void count_level_dispatch(int W, hgx_graph* g, const uint32_t* fa, const u64* lvl, u64* counts, u64* trav) {
    switch (W) {
        case 1: count_level<1>(g, fa, lvl, counts, trav); break;
        case 2: count_level<2>(g, fa, lvl, counts, trav); break;
        case 4: count_level<4>(g, fa, lvl, counts, trav); break;
        case 8: count_level<8>(g, fa, lvl, counts, trav); break;
        default: count_level<16>(g, fa, lvl, counts, trav); break;
    }
}

// Fill res->counts and the TEPS numerator (first call only).
void ensure_counts(hgx_bfs_result* r) {
    if (r->counts_ready) return;
    hgx_graph* g = r->g;
    HGX_HIP(hipSetDevice(g->device));
    r->counts.assign((size_t)r->n_seeds * r->n_levels, 0);
    double trav_total = 0;
    u64* dc = (u64*)g->alloc(sizeof(u64) * (1024 + 1));
    std::vector<u64> hc(1025);
    for (auto& bt : r->batches) {
        int nl = (int)bt.lvl.size();
        for (int d = 0; d < nl; ++d) {
            HGX_HIP(hipMemsetAsync(dc, 0, sizeof(u64) * 1025, g->stream));
            count_level_dispatch(bt.W, g, bt.fa[d], bt.lvl[d], dc, dc + 1024);
            HGX_HIP(hipMemcpyAsync(hc.data(), dc, sizeof(u64) * 1025, hipMemcpyDeviceToHost, g->stream));
            HGX_HIP(hipStreamSynchronize(g->stream));
            for (int s = 0; s < bt.S; ++s) r->counts[(size_t)(bt.seed0 + s) * r->n_levels + d] = (int64_t)hc[s];
            // expanded levels are those below the last level that was expanded
            if (d < bt.n_expanded) {
                trav_total += (double)hc[1024];
                // SURVEY.md 8(d) push-model bytes from the union frontier of this level
                HGX_HIP(hipMemsetAsync(dc, 0, sizeof(u64) * 4, g->stream));
                hgx_level_survey<<<grid_for(g->A, 256, 8192), 256, 0, g->stream>>>(g->A, bt.fa[d], g->inc_off,
                                                                                    g->inc_row, g->tgt_off, dc);
                HGX_CHECK_LAUNCH();
                u64 sv[3];
                HGX_HIP(hipMemcpyAsync(sv, dc, sizeof(sv), hipMemcpyDeviceToHost, g->stream));
                HGX_HIP(hipStreamSynchronize(g->stream));
                const double U = (double)sv[0], sdeg = (double)sv[1], Pd = (double)sv[2];
                const double typed = r->typed ? 1.0 : 0.0;
                const double mask = (double)((bt.S + 7) / 8);
                r->stats.bytes_survey += 16.0 * U + 4.0 * sdeg + (16.0 + 4.0 * typed) * sdeg + 4.0 * Pd +
                                         mask * (U + 2.0 * Pd);
                if (d < 64) r->stats.union_frontier[d] += (int64_t)sv[0];
            }
        }
    }
    g->release(dc, sizeof(u64) * 1025);
    r->stats.traversed_edges = trav_total;
    r->counts_ready = true;
}

}  // namespace

extern "C" {

int hgx_bfs_batch(hgx_graph* g, const int32_t* seeds, int32_t n_seeds, int32_t max_depth,
                  const hgx_algen_opts* opts, hgx_bfs_result** out) {
    HGX_API_BEGIN
    if (!g || !out || n_seeds < 0 || (n_seeds > 0 && !seeds)) fail(HGX_E_INVALID, "hgx_bfs_batch: bad argument");
    *out = nullptr;
    hgx_algen_opts o = opts ? *opts : hgx_algen_opts{HGX_NO_TYPE, 1, 1, 0, 0};
    for (int32_t i = 0; i < n_seeds; ++i)
        if (seeds[i] < 0 || seeds[i] >= g->A) fail(HGX_E_INVALID, "hgx_bfs_batch: seed out of range");
    if (max_depth < -1) fail(HGX_E_INVALID, "hgx_bfs_batch: bad max_depth");
    std::lock_guard<std::mutex> lk(g->mu);
    HGX_HIP(hipSetDevice(g->device));
    const int mode = mode_of(o);

    hgx_bfs_result* r = new hgx_bfs_result();
    struct Guard {
        hgx_bfs_result* r;
        ~Guard() { if (r) hgx_bfs_result_free(r); }
    } guard{r};
    r->g = g;
    g->refs.fetch_add(1);
    r->n_seeds = n_seeds;
    r->typed = o.link_type >= 0;

    Timer tm(g);
    if (tm.on) HGX_HIP(hipEventRecord(tm.begin_all.a, g->stream));
    std::vector<std::vector<u64>> level_ctr;
    int max_expanded = 0;
    for (int32_t s0 = 0; s0 < n_seeds; s0 += 1024) {
        BfsBatch bt;
        bt.seed0 = s0;
        bt.S = std::min<int32_t>(1024, n_seeds - s0);
        bt.W = words_for(bt.S);
        // unique seed atoms (ascending) and their rows
        std::map<int32_t, std::vector<u64>> rows;
        for (int32_t i = 0; i < bt.S; ++i) {
            auto& row = rows[seeds[s0 + i]];
            if (row.empty()) row.assign(bt.W, 0ull);
            row[i >> 6] |= 1ull << (i & 63);
        }
        std::vector<int32_t> sa;
        std::vector<u64> sr;
        for (auto& kv : rows) {
            sa.push_back(kv.first);
            sr.insert(sr.end(), kv.second.begin(), kv.second.end());
        }
        size_t before = level_ctr.size();
        switch (bt.W) {
            case 1: run_mode<1>(mode, g, r, bt, max_depth, o.link_type, sa, sr, tm, level_ctr); break;
            case 2: run_mode<2>(mode, g, r, bt, max_depth, o.link_type, sa, sr, tm, level_ctr); break;
            case 4: run_mode<4>(mode, g, r, bt, max_depth, o.link_type, sa, sr, tm, level_ctr); break;
            case 8: run_mode<8>(mode, g, r, bt, max_depth, o.link_type, sa, sr, tm, level_ctr); break;
            default: run_mode<16>(mode, g, r, bt, max_depth, o.link_type, sa, sr, tm, level_ctr); break;
        }
        // accounting for this batch (levels expanded = level_ctr entries added)
        const int64_t A = g->A, M = g->M, P = g->P, I = g->I;
        (void)I;
        const double rowb = 8.0 * bt.W;
        const bool typed = o.link_type >= 0;
        int nexp = (int)(level_ctr.size() - before);
        bt.n_expanded = nexp;
        max_expanded = std::max(max_expanded, nexp);
        const double I_light = (double)(I - g->I_heavy), I_heavy = (double)g->I_heavy;
        for (int d = 0; d < nexp; ++d) {
            const auto& c = level_ctr[before + d];
            // hgx_link_gather: tgt_off + tgt_idx (+ link_type) + frontier bitmap + gathered rows + lf/la writes
            r->stats.bytes_kernel[HGX_K_LINK_GATHER] +=
                8.0 * (M + 1) + 4.0 * P + (typed ? 4.0 * M : 0.0) + A / 8.0 + rowb * c[cActivePins] +
                (mode == kSym ? rowb * c[cActiveLinks] : 0.0) + M / 8.0;
            // hgx_atom_pull: inc_off + light inc_row + la bitmap + pulled rows + vis reads + lvl/vis writes
            //                + ever/fa_next bitmaps
            r->stats.bytes_kernel[HGX_K_ATOM_PULL] += 8.0 * (A + 1) + 4.0 * I_light + M / 8.0 +
                                                      rowb * c[cIncLight] + rowb * c[cAccLight] +
                                                      2.0 * rowb * c[cNewLight] + A / 4.0;
            if (g->n_chunks > 0) {
                r->stats.bytes_kernel[HGX_K_PULL_HEAVY] += 24.0 * g->n_chunks + 4.0 * I_heavy + rowb * c[cIncHeavy] +
                                                           rowb * g->n_chunks;
                r->stats.bytes_kernel[HGX_K_HUB_FINALIZE] += 4.0 * g->n_heavy + 2.0 * rowb * g->n_heavy +
                                                             rowb * c[cAccHub] + 2.0 * rowb * c[cNewHub];
                r->stats.launches[HGX_K_PULL_HEAVY] += 1;
                r->stats.launches[HGX_K_HUB_FINALIZE] += 1;
            }
            r->stats.launches[HGX_K_LINK_GATHER] += 1;
            r->stats.launches[HGX_K_ATOM_PULL] += 1;
        }
        r->batches.push_back(std::move(bt));
    }
    if (tm.on) HGX_HIP(hipEventRecord(tm.end_all.a, g->stream));
    HGX_HIP(hipStreamSynchronize(g->stream));
    int nl = 1;
    for (auto& bt : r->batches) nl = std::max(nl, (int)bt.lvl.size());
    r->n_levels = nl;
    r->stats.n_levels_expanded = max_expanded;
    r->stats.n_batches = (int32_t)r->batches.size();
    if (tm.on) {
        float ms = 0;
        HGX_HIP(hipEventElapsedTime(&ms, tm.begin_all.a, tm.end_all.a));
        r->stats.ms_total = ms;
        for (int k = 0; k < HGX_K_COUNT; ++k) r->stats.ms_kernel[k] = tm.total(k);
    }
    guard.r = nullptr;
    *out = r;
    HGX_API_END
}

int hgx_bfs_result_info(const hgx_bfs_result* r, int32_t* n_seeds, int32_t* n_levels) {
    HGX_API_BEGIN
    if (!r) fail(HGX_E_INVALID, "null result");
    if (n_seeds) *n_seeds = r->n_seeds;
    if (n_levels) *n_levels = r->n_levels;
    HGX_API_END
}

int hgx_bfs_result_counts(hgx_bfs_result* r, int64_t* counts) {
    HGX_API_BEGIN
    if (!r || !counts) fail(HGX_E_INVALID, "hgx_bfs_result_counts: bad argument");
    std::lock_guard<std::mutex> lk(r->g->mu);
    ensure_counts(r);
    std::memcpy(counts, r->counts.data(), sizeof(int64_t) * r->counts.size());
    HGX_API_END
}

int hgx_bfs_result_visited(hgx_bfs_result* r, int32_t seed_index, int32_t depth, int32_t* out, int64_t cap,
                           int64_t* n_out) {
    HGX_API_BEGIN
    if (!r || !n_out || (cap > 0 && !out)) fail(HGX_E_INVALID, "hgx_bfs_result_visited: bad argument");
    if (seed_index < 0 || seed_index >= r->n_seeds) fail(HGX_E_NOTFOUND, "no such seed index");
    if (depth < 0) fail(HGX_E_NOTFOUND, "no such depth");
    hgx_graph* g = r->g;
    std::lock_guard<std::mutex> lk(g->mu);
    HGX_HIP(hipSetDevice(g->device));
    const BfsBatch& bt = r->batches[seed_index / 1024];
    const int s = seed_index % 1024;
    *n_out = 0;
    if (depth >= (int32_t)bt.lvl.size()) return HGX_OK;
    const int nblk = (int)std::min<int64_t>(2048, std::max<int64_t>(1, ceil_div(g->A, 4096)));
    const int64_t span = ceil_div(std::max<int64_t>(g->A, 1), nblk);
    int64_t* dcnt = (int64_t*)g->alloc(sizeof(int64_t) * nblk * 2);
    int64_t* doff = dcnt + nblk;
    hgx_extract<<<nblk, 256, 0, g->stream>>>(g->A, span, bt.W, s, bt.fa[depth], bt.lvl[depth], doff, dcnt, nullptr,
                                              0, false);
    HGX_CHECK_LAUNCH();
    std::vector<int64_t> hc(nblk), ho(nblk);
    HGX_HIP(hipMemcpyAsync(hc.data(), dcnt, sizeof(int64_t) * nblk, hipMemcpyDeviceToHost, g->stream));
    HGX_HIP(hipStreamSynchronize(g->stream));
    int64_t tot = 0;
    for (int i = 0; i < nblk; ++i) {
        ho[i] = tot;
        tot += hc[i];
    }
    *n_out = tot;
    int64_t k = std::min(tot, cap);
    if (k > 0) {
        int32_t* dout = (int32_t*)g->alloc(sizeof(int32_t) * k);
        HGX_HIP(hipMemcpyAsync(doff, ho.data(), sizeof(int64_t) * nblk, hipMemcpyHostToDevice, g->stream));
        hgx_extract<<<nblk, 256, 0, g->stream>>>(g->A, span, bt.W, s, bt.fa[depth], bt.lvl[depth], doff, dcnt, dout,
                                                  k, true);
        HGX_CHECK_LAUNCH();
        HGX_HIP(hipMemcpyAsync(out, dout, sizeof(int32_t) * k, hipMemcpyDeviceToHost, g->stream));
        HGX_HIP(hipStreamSynchronize(g->stream));
        g->release(dout, sizeof(int32_t) * k);
    }
    g->release(dcnt, sizeof(int64_t) * nblk * 2);
    HGX_API_END
}

int hgx_bfs_result_depth_of(hgx_bfs_result* r, int32_t seed_index, int32_t atom, int32_t* depth_out) {
    HGX_API_BEGIN
    if (!r || !depth_out) fail(HGX_E_INVALID, "hgx_bfs_result_depth_of: bad argument");
    if (seed_index < 0 || seed_index >= r->n_seeds) fail(HGX_E_NOTFOUND, "no such seed index");
    hgx_graph* g = r->g;
    if (atom < 0 || atom >= g->A) fail(HGX_E_INVALID, "atom id out of range");
    std::lock_guard<std::mutex> lk(g->mu);
    HGX_HIP(hipSetDevice(g->device));
    const BfsBatch& bt = r->batches[seed_index / 1024];
    const int nl = (int)bt.lvl.size();
    void** tab = (void**)g->alloc(sizeof(void*) * 2 * nl + sizeof(int32_t) * 4);
    std::vector<void*> h(2 * nl);
    for (int k = 0; k < nl; ++k) {
        h[k] = bt.fa[k];
        h[nl + k] = bt.lvl[k];
    }
    int32_t* dres = (int32_t*)(tab + 2 * nl);
    HGX_HIP(hipMemcpyAsync(tab, h.data(), sizeof(void*) * 2 * nl, hipMemcpyHostToDevice, g->stream));
    hgx_depth_probe<<<1, 64, 0, g->stream>>>(nl, (const uint32_t* const*)tab, (const u64* const*)(tab + nl), bt.W,
                                             seed_index % 1024, atom, dres);
    HGX_CHECK_LAUNCH();
    HGX_HIP(hipMemcpyAsync(depth_out, dres, sizeof(int32_t), hipMemcpyDeviceToHost, g->stream));
    HGX_HIP(hipStreamSynchronize(g->stream));
    g->release(tab, sizeof(void*) * 2 * nl + sizeof(int32_t) * 4);
    HGX_API_END
}

int hgx_bfs_result_stats(hgx_bfs_result* r, int32_t with_accounting, hgx_bfs_stats* st) {
    HGX_API_BEGIN
    if (!r || !st) fail(HGX_E_INVALID, "hgx_bfs_result_stats: bad argument");
    std::lock_guard<std::mutex> lk(r->g->mu);
    if (with_accounting) ensure_counts(r);
    *st = r->stats;
    HGX_API_END
}

void hgx_bfs_result_free(hgx_bfs_result* r) {
    if (!r) return;
    hgx_graph* g = r->g;
    if (g) {
        std::lock_guard<std::mutex> lk(g->mu);
        (void)hipSetDevice(g->device);
        for (auto& bt : r->batches) {
            for (auto p : bt.lvl) g->release(p, r->row_bytes(bt));
            for (auto p : bt.fa) g->release(p, r->bm_bytes());
        }
    }
    delete r;
    if (g) graph_release(g);
}

}  // extern "C"
