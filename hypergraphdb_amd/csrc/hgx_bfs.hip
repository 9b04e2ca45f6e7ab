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
// inside the pull instead of lf.
//
// Work avoidance (all exact):
//   * rows are only read behind per-level activity bitmaps (fa: atom frontier, la: link active),
//     so a sparse level costs the CSR scan, not the mask traffic;
//   * an atom visited by every traversal ('full') is never pulled again, and a link whose targets
//     are all full is never gathered;
//   * a pull stops as soon as acc | vis covers every traversal, a gather as soon as acc does.
// Bitmaps are 64-bit words owned by one wavefront each (a wave processes 64 consecutive rows), so
// they are written with plain stores -- no per-row atomics.

#include <algorithm>
#include <cstring>
#include <map>
#include <memory>

#include <cstdio>
#include <cstdlib>

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
    static constexpr int PER_WAVE = 64 / G;   // rows handled by one wave per iteration
};

template <int WPL> struct Vec;
template <> struct Vec<1> {
    typedef u64 T;
    static __device__ __forceinline__ T zero() { return 0ull; }
    static __device__ __forceinline__ bool nz(T x) { return x != 0ull; }
    static __device__ __forceinline__ bool eq(T x, T y) { return x == y; }
    static __device__ __forceinline__ T ld(const u64* p) { return *p; }
    static __device__ __forceinline__ void st(u64* p, T x) { *p = x; }
    static __device__ __forceinline__ void st_nt(u64* p, T x) { __builtin_nontemporal_store(x, p); }
};
template <> struct Vec<2> {
    typedef u64x2 T;
    static __device__ __forceinline__ T zero() { return u64x2{0ull, 0ull}; }
    static __device__ __forceinline__ bool nz(T x) { return (x.x | x.y) != 0ull; }
    static __device__ __forceinline__ bool eq(T x, T y) { return x.x == y.x && x.y == y.y; }
    static __device__ __forceinline__ T ld(const u64* p) { return *reinterpret_cast<const u64x2*>(p); }
    static __device__ __forceinline__ void st(u64* p, T x) { *reinterpret_cast<u64x2*>(p) = x; }
    static __device__ __forceinline__ void st_nt(u64* p, T x) { __builtin_nontemporal_store(x, reinterpret_cast<u64x2*>(p)); }
};

// Valid-source mask of a row (S need not be a multiple of 64 or a power of two).
struct FullMask {
    u64 w[16];
};

template <int W>
__device__ __forceinline__ typename Vec<Lay<W>::WPL>::T full_part(const FullMask& fm, int sub) {
    if constexpr (Lay<W>::WPL == 1) {
        return fm.w[sub];
    } else {
        return u64x2{fm.w[sub * 2], fm.w[sub * 2 + 1]};
    }
}

__device__ __forceinline__ bool bit(const u64* __restrict__ bm, int64_t i) { return (bm[i >> 6] >> (i & 63)) & 1ull; }
__device__ __forceinline__ void set_bit(u64* bm, int64_t i) { atomicOr(&bm[i >> 6], 1ull << (i & 63)); }

// position of the n-th (0-based) set bit of x (n < popcount(x)): a binary descent over the halves
__device__ __forceinline__ int nth_set_bit(u64 x, int n) {
    int pos = 0;
#pragma unroll
    for (int half = 32; half > 0; half >>= 1) {
        const u64 lo = x & ((1ull << half) - 1ull);
        const int c = __popcll(lo);
        if (n >= c) {
            n -= c;
            x >>= half;
            pos += half;
        } else {
            x = lo;
        }
    }
    return pos;
}

// true if predicate holds on any / every lane of this lane's G-lane group (groups are G-aligned).
template <int G> __device__ __forceinline__ bool group_any(bool p) {
    if constexpr (G == 1) {
        return p;
    } else {
        u64 b = __ballot(p);
        int base = (threadIdx.x & 63) & ~(G - 1);
        return ((b >> base) & ((1ull << G) - 1ull)) != 0ull;
    }
}
template <int G> __device__ __forceinline__ bool group_all(bool p) { return !group_any<G>(!p); }

// Compress a wave ballot whose bit of group g sits at lane g*G into bits [pos0, pos0 + 64/G).
template <int G> __device__ __forceinline__ u64 compress_groups(u64 b, int pos0) {
    if constexpr (G == 1) {
        return b;   // pos0 == 0 (one iteration covers the 64-row tile)
    } else {
        u64 out = 0;
#pragma unroll
        for (int g = 0; g < 64 / G; ++g) out |= ((b >> (g * G)) & 1ull) << (pos0 + g);
        return out;
    }
}

// Bitmap scans: a wave loads 64 consecutive words at once (one per lane) and visits only the
// nonzero ones, so a sparse bitmap costs one coalesced load per 64 words instead of a serial
// word-per-iteration loop.  body(word_index, word) runs wave-uniformly.
template <class F>
__device__ __forceinline__ void for_nonzero_words(const u64* __restrict__ bm, int64_t nwords, F body) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    const int64_t nwave = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t base = wave * 64; base < nwords; base += nwave * 64) {
        const u64 x = base + lane < nwords ? bm[base + lane] : 0ull;
        u64 m = __ballot(x != 0ull);
        while (m) {
            const int k = __ffsll((long long)m) - 1;
            m &= m - 1ull;
            body(base + k, (u64)__shfl(x, k));
        }
    }
}

// For every set bit b of the wave-uniform word xw: op(b, w, payload of lane b) on W lanes
// (w = 0..W-1), 64/W bits at a time.  The shuffle runs on every lane (a lane shuffling from an
// inactive lane reads garbage on CDNA).
template <class F>
__device__ __forceinline__ void rows_of_word(u64 xw, int W, int32_t payload, F op) {
    const int lane = threadIdx.x & 63, R = 64 / W, k = lane / W, wd = lane % W;
    while (xw) {
        u64 y = xw;
        for (int i = 0; i < k && y; ++i) y &= y - 1ull;
        const int b = y ? __ffsll((long long)y) - 1 : -1;
        for (int i = 0; i < R && xw; ++i) xw &= xw - 1ull;
        const int32_t pv = __shfl(payload, b < 0 ? 0 : b);
        if (b >= 0) op(b, wd, pv);
    }
}

// per-level counters (device): early stop + byte accounting
enum Ctr {
    cActiveLinks = 0,   // lf rows written                                   (link gather)
    cActivePins,        // target rows gathered                              (link gather)
    cIncLight,          // lf rows pulled, light atoms                       (atom pull)
    cVisLight,          // vis rows read, light atoms
    cNewLight,          // light atoms with a new bit (lvl + vis written)
    cIncHeavy,          // lf rows pulled, heavy chunks
    cAccHub,            // heavy atoms finalised with a nonzero pull
    cNewHub,            // heavy atoms with a new bit
    cNewAtoms,          // all new atoms of the level (early stop)
    cDirRows,           // ordered modes: target rows re-read in the pull
    cNewDeg,            // sum of |inc(v)| over the new atoms (next level's push volume)
    cNewFull,           // atoms that became visited by every traversal
    cCand,              // frontier-push candidates finalised
    cNewDegNF,          // sum of |inc(v)| over the new atoms not yet visited by every traversal
    cNfRows,            // frontier rows read by the non-full pull
    cScanned,           // incidence entries scanned by the frontier push (type + yield flag)
    cNum = 16
};

__device__ __forceinline__ void wave_add(u64* ctr, u64 v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(ctr, v);
}

// Level counters are kept in kCtrShards replicas on lines of their own (one device-scope atomic
// word saturates at ~90 adds/us; thousands of waves add to every counter each level).  Counter c
// of shard k lives at base[k * kCtrStride + c]; the host sums the shards.
constexpr int kCtrShards = 16, kCtrStride = 16, kCtrBlock = kCtrShards * kCtrStride;
constexpr int kHostSlot = 32;   // u64 words of one level's counters in mapped host memory (cNum + sequence)
// Internal per-level flag (above the HGX_OPT_BFS_FLAGS bits): dense level with every lf row written.
constexpr int kAllRows = 1 << 16;
// Cache-policy A/B bits of HGX_OPT_BFS_FLAGS for the tile-staged dense kernels (gather2 / pull2).
// None moved config 2 beyond noise (17.66 / 17.63 / 17.68 / 17.65 / 17.63 ms for none / 12 / 13 /
// 14 / all three, profiles/r01i_ab_nt.log): the streamed columns and the written rows do not evict
// the hub rows the Infinity Cache serves, so the default keeps the plain policy.
constexpr int kNtIdx = 1 << 12;    // nontemporal loads of the streamed CSR columns (offsets, ids)
constexpr int kNtLf = 1 << 13;     // nontemporal stores of the gather's lf rows
constexpr int kNtOut = 1 << 14;    // nontemporal stores of the pull's lvl_next / vis rows
// Heavy (hub) pull of the symmetric mode with two incidence chunks of a group in flight at once and
// no la probe, in all-rows levels before the full-visited skip turns on (HGX_OPT_BFS_FLAGS bit 15,
// A/B only, off by default).  Config 2: level 1 8.89 -> 8.60 ms but level 2 6.81 -> 7.04 ms (hub
// pulls there exit early after a few chunks and the one-chunk pull_range exits sooner); with the
// probe kept both levels were slower; neither the `ever` bit nor the full-skip state of the level
// separates the two cases (profiles/r01i_ab_heavy*.log), so the default keeps pull_range.
constexpr int kHeavyMlp2 = 1 << 15;
constexpr int kGatherO5 = 1 << 10;   // diagnostic: the dense gather built at 5 waves/SIMD (spills)

template <typename T>
__device__ __forceinline__ T ld_col(const T* p, bool nt) {
    return nt ? __builtin_nontemporal_load(p) : *p;
}
template <typename V>
__device__ __forceinline__ void st_row(u64* p, typename V::T x, bool nt) {
    if (nt) V::st_nt(p, x);
    else V::st(p, x);
}
static_assert(cNum <= kCtrStride, "counter block");
__device__ __forceinline__ void wave_add_sh(u64* ctr, u64 v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    const int shard = (int)((blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) & (kCtrShards - 1));
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(ctr + shard * kCtrStride, v);
}

// Block-wide sum of v added into shard (blockIdx.x % kStatShards) of counter c: stats[shard *
// kStatStride + c].  Every thread of the block calls it.  One device atomic per block spread over 16
// lines: thousands of waves adding into one word serialise at ~90 adds/us (a 4096-wave kernel spent
// ~90 us there per counter).
constexpr int kStatShards = 16, kStatStride = 16;
__device__ __forceinline__ void block_add_sh(u64* stats, int c, u64 v) {
    __shared__ u64 part[16];
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    const int wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) part[wv] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        u64 t = 0;
        for (int w = 0; w < nw; ++w) t += part[w];
        if (t) atomicAdd(stats + (blockIdx.x % kStatShards) * kStatStride + c, t);
    }
}

// ---------------------------------------------------------------------------------------------
// Link gather: lf[L] = OR_{v in targets(L), fa_d(v)} lvl_d[v]; la(L) set iff the row was written.
// A wave owns 64 consecutive link rows (one la word); a G-lane group handles one row at a time.
// WRITE_LF = false in the ordered modes (only la is needed there).
// ---------------------------------------------------------------------------------------------
template <int W, bool WRITE_LF>
__global__ void __launch_bounds__(256) hgx_link_gather(int64_t M, const int64_t* __restrict__ tgt_off,
                                                       const int32_t* __restrict__ tgt_idx,
                                                       const int32_t* __restrict__ link_type, int32_t want_type,
                                                       const u64* __restrict__ fa, const u64* __restrict__ full,
                                                       const u64* __restrict__ lvl, u64* __restrict__ lf,
                                                       u64* __restrict__ la, u64* __restrict__ ctr, FullMask fm,
                                                       int flags, const u64* __restrict__ lcand,
                                                       u64* __restrict__ cand) {
    constexpr int WPL = Lay<W>::WPL, G = Lay<W>::G, PW = Lay<W>::PER_WAVE;
    const bool early = flags & 1, skip_full = flags & 4;
    typedef Vec<WPL> V;
    const int lane = threadIdx.x & 63, g = lane / G, sub = lane & (G - 1);
    const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    const int64_t nwave = ((int64_t)gridDim.x * blockDim.x) >> 6;
    const typename V::T FULL = full_part<W>(fm, sub);
    u64 n_links = 0, n_pins = 0;
    for (int64_t tile = wave; tile * 64 < M; tile += nwave) {
        u64 word = 0;
        // sparse levels: only links incident to a frontier atom (lcand) can be active
        const u64 lc = lcand ? lcand[tile] : ~0ull;
        if (lc == 0) {
            if (lane == 0) la[tile] = 0;
            continue;
        }
        for (int j = 0; j < G; ++j) {
            const int64_t L = tile * 64 + j * PW + g;
            bool act = false;
            if (L < M && ((lc >> (j * PW + g)) & 1ull) && (want_type < 0 || link_type[L] == want_type)) {
                const int64_t b = tgt_off[L], e = tgt_off[L + 1];
                typename V::T acc = V::zero();
                int nact = 0;
                bool all_full = true;
                if constexpr (G >= 4) {
                    // lane `sub` loads target p+sub and checks its own bitmap bits; the group then
                    // gathers the active rows (16 B per lane) via ballot + shuffle.  The full bits of
                    // all targets are known before any row is loaded: a link whose targets are all
                    // visited by every traversal costs no row traffic.
                    const int base = lane & ~(G - 1);
                    const u64 gmask = (1ull << G) - 1ull;
                    bool any_not_full = !skip_full;
                    if (e - b > G && skip_full) {          // long rows: full bits first
                        for (int64_t p = b; p < e && !any_not_full; p += G) {
                            const int64_t q = p + sub;
                            const int32_t myv = q < e ? tgt_idx[q] : -1;
                            any_not_full |= ((__ballot(myv >= 0 && !bit(full, myv)) >> base) & gmask) != 0ull;
                        }
                    }
                    for (int64_t p = b; p < e; p += G) {
                        const int64_t q = p + sub;
                        const int32_t myv = q < e ? tgt_idx[q] : -1;
                        if (e - b <= G && skip_full)
                            any_not_full = ((__ballot(myv >= 0 && !bit(full, myv)) >> base) & gmask) != 0ull;
                        if (!any_not_full) break;           // every target full: nobody pulls this row
                        const bool mya = myv >= 0 && bit(fa, myv);
                        const unsigned ga = (unsigned)((__ballot(mya) >> base) & gmask);
                        typename V::T r[G];
#pragma unroll
                        for (int k = 0; k < G; ++k) {
                            const int32_t vk = __shfl(myv, base + k);
                            r[k] = ((ga >> k) & 1u) ? V::ld(lvl + (int64_t)vk * W + sub * WPL) : V::zero();
                        }
#pragma unroll
                        for (int k = 0; k < G; ++k) acc |= r[k];
                        nact += __popc(ga);
                        if (early && p + G < e && group_all<G>(V::eq(acc, FULL))) break;
                    }
                    all_full = !any_not_full;
                } else {
                    for (int64_t p = b; p < e; p += 4) {
                        int32_t v[4];
                        bool a[4];
#pragma unroll
                        for (int k = 0; k < 4; ++k) v[k] = p + k < e ? tgt_idx[p + k] : -1;
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            a[k] = v[k] >= 0 && bit(fa, v[k]);
                            if (skip_full) all_full &= v[k] < 0 || bit(full, v[k]);
                        }
#pragma unroll
                        for (int k = 0; k < 4; ++k)
                            if (a[k]) acc |= V::ld(lvl + (int64_t)v[k] * W + sub * WPL);
                        nact += (int)a[0] + (int)a[1] + (int)a[2] + (int)a[3];
                        if (early && p + 4 < e && group_all<G>(V::eq(acc, FULL))) {   // every traversal present
                            all_full = false;
                            break;
                        }
                    }
                }
                act = nact > 0 && !(skip_full && all_full);   // all targets full: nobody pulls this row
                if (act && cand) {   // sparse levels: the targets of an active link are the pull candidates
                    for (int64_t p = b + sub; p < e; p += G) {
                        const int32_t v = tgt_idx[p];
                        atomicOr(&cand[v >> 6], 1ull << (v & 63));
                    }
                }
                if (act) {
                    if (WRITE_LF) V::st(lf + L * W + sub * WPL, acc);
                    if (sub == 0) {
                        ++n_links;
                        n_pins += nact;
                    }
                }
            }
            word |= compress_groups<G>(__ballot(act), j * PW);
        }
        if (lane == 0) la[tile] = word;
    }
    wave_add_sh(ctr + cActiveLinks, n_links);
    wave_add_sh(ctr + cActivePins, n_pins);
}

// Ordered modes: the frontier rows of the co-targets of t in one link row that may yield t.
template <int W, int MODE>
__device__ __forceinline__ typename Vec<Lay<W>::WPL>::T pull_ordered(int32_t t, int64_t b, int64_t e,
                                                                      const int32_t* __restrict__ tgt_idx,
                                                                      const u64* __restrict__ fa,
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

// Pull incidence entries [b, e) of atom t into acc, stopping once acc | old covers FULL.
// `old` is loaded lazily from vis (only when the first active link is met and t has a vis row).
template <int W, int MODE>
__device__ __forceinline__ void pull_range(int32_t t, int64_t b, int64_t e, const int32_t* __restrict__ inc_row,
                                           const u64* __restrict__ la, const u64* __restrict__ lf,
                                           const int64_t* __restrict__ tgt_off, const int32_t* __restrict__ tgt_idx,
                                           const u64* __restrict__ fa, const u64* __restrict__ lvl,
                                           const u64* __restrict__ vis_row, bool have_vis,
                                           typename Vec<Lay<W>::WPL>::T FULL, int sub,
                                           typename Vec<Lay<W>::WPL>::T& acc, typename Vec<Lay<W>::WPL>::T& old,
                                           bool& have_old, u64& n_inc, u64& n_vis, bool early) {
    constexpr int WPL = Lay<W>::WPL, G = Lay<W>::G;
    typedef Vec<WPL> V;
    if constexpr (G >= 4 && MODE == kSym) {
        // lane `sub` loads entry i+sub and tests its la bit; the group then pulls the active lf rows
        const int base = (threadIdx.x & 63) & ~(G - 1);
        for (int64_t i = b; i < e; i += G) {
            const int64_t q = i + sub;
            const int32_t myL = q < e ? inc_row[q] : -1;
            const bool mya = myL >= 0 && bit(la, myL);
            const unsigned ga = (unsigned)((__ballot(mya) >> base) & ((1ull << G) - 1ull));
            typename V::T r[G];
#pragma unroll
            for (int k = 0; k < G; ++k) {
                const int32_t Lk = __shfl(myL, base + k);
                r[k] = ((ga >> k) & 1u) ? V::ld(lf + (int64_t)Lk * W + sub * WPL) : V::zero();
            }
#pragma unroll
            for (int k = 0; k < G; ++k) acc |= r[k];
            n_inc += __popc(ga);
            if (!early) continue;
            if (!have_old && group_any<G>(V::nz(acc))) {
                if (have_vis) {
                    old = V::ld(vis_row + sub * WPL);
                    ++n_vis;
                }
                have_old = true;
            }
            if (have_old && i + G < e && group_all<G>(V::eq(acc | old, FULL))) break;
        }
    } else {
        for (int64_t i = b; i < e; i += 8) {
            int32_t L[8];
            bool act[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) L[k] = i + k < e ? inc_row[i + k] : -1;
#pragma unroll
            for (int k = 0; k < 8; ++k) act[k] = L[k] >= 0 && bit(la, L[k]);
            if constexpr (MODE == kSym) {
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    if (act[k]) {
                        acc |= V::ld(lf + (int64_t)L[k] * W + sub * WPL);
                        ++n_inc;
                    }
            } else {
                for (int k = 0; k < 8; ++k)
                    if (act[k]) {
                        acc |= pull_ordered<W, MODE>(t, tgt_off[L[k]], tgt_off[L[k] + 1], tgt_idx, fa, lvl, sub);
                        ++n_inc;
                    }
            }
            if (!early) continue;
            if (!have_old && group_any<G>(V::nz(acc))) {
                if (have_vis) {
                    old = V::ld(vis_row + sub * WPL);
                    ++n_vis;
                }
                have_old = true;
            }
            if (have_old && i + 8 < e && group_all<G>(V::eq(acc | old, FULL))) break;
        }
    }
    if (!have_old && group_any<G>(V::nz(acc))) {   // no early exit: vis read once at the end
        if (have_vis) {
            old = V::ld(vis_row + sub * WPL);
            ++n_vis;
        }
        have_old = true;
    }
}

// Atom pull for light atoms (deg <= kHeavyDegree).  A wave owns 64 consecutive atoms (one word of
// fa_next / ever / full); a G-lane group handles one atom at a time.  Heavy atoms are skipped here
// (hgx_atom_pull_heavy + hgx_hub_finalize run afterwards and OR their bits in).
template <int W, int MODE>
__global__ void __launch_bounds__(256) hgx_atom_pull(int64_t A, const int64_t* __restrict__ inc_off,
                                                     const int32_t* __restrict__ inc_row,
                                                     const u64* __restrict__ la, const u64* __restrict__ lf,
                                                     const int64_t* __restrict__ tgt_off,
                                                     const int32_t* __restrict__ tgt_idx,
                                                     const u64* __restrict__ fa, const u64* __restrict__ lvl,
                                                     u64* __restrict__ vis, u64* __restrict__ ever,
                                                     u64* __restrict__ full, u64* __restrict__ lvl_next,
                                                     u64* __restrict__ fa_next, u64* __restrict__ ctr, FullMask fm,
                                                     int flags, const u64* __restrict__ cand) {
    constexpr int WPL = Lay<W>::WPL, G = Lay<W>::G, PW = Lay<W>::PER_WAVE;
    const bool early = flags & 2, skip_full = flags & 4;
    typedef Vec<WPL> V;
    const int lane = threadIdx.x & 63, g = lane / G, sub = lane & (G - 1);
    const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    const int64_t nwave = ((int64_t)gridDim.x * blockDim.x) >> 6;
    const typename V::T FULL = full_part<W>(fm, sub);
    u64 n_inc = 0, n_vis = 0, n_new = 0, n_newdeg = 0, n_newdeg_nf = 0, n_full = 0;
    for (int64_t tile = wave; tile * 64 < A; tile += nwave) {
        // sparse levels: only targets of active links (cand) can gain a bit
        const u64 cw = cand ? cand[tile] : ~0ull;
        if (cw == 0) {
            if (lane == 0) fa_next[tile] = 0;
            continue;
        }
        const u64 ever_w = ever[tile], full_w = full[tile];
        u64 new_w = 0, fullnew_w = 0;
        for (int j = 0; j < G; ++j) {
            const int pos = j * PW + g;
            const int64_t t = tile * 64 + pos;
            bool isnew = false, becomes_full = false;
            if (t < A && ((cw >> pos) & 1ull) && !(skip_full && ((full_w >> pos) & 1ull))) {
                const int64_t b = inc_off[t], e = inc_off[t + 1];
                if (e > b && e - b <= kHeavyDegree) {
                    const bool ev = (ever_w >> pos) & 1ull;
                    typename V::T acc = V::zero(), old = V::zero();
                    bool have_old = false;
                    pull_range<W, MODE>((int32_t)t, b, e, inc_row, la, lf, tgt_off, tgt_idx, fa, lvl, vis + t * W,
                                        ev, FULL, sub, acc, old, have_old, n_inc, n_vis, early);
                    const typename V::T nw = acc & ~old;
                    if (group_any<G>(V::nz(nw))) {
                        V::st(lvl_next + t * W + sub * WPL, nw);
                        V::st(vis + t * W + sub * WPL, old | nw);
                        isnew = true;
                        becomes_full = group_all<G>(V::eq(old | nw, FULL));
                        if (sub == 0) { const u64 dg_ = (u64)(e - b); n_newdeg += dg_; if (!becomes_full) n_newdeg_nf += dg_; }
                    }
                }
            }
            new_w |= compress_groups<G>(__ballot(isnew), j * PW);
            fullnew_w |= compress_groups<G>(__ballot(becomes_full), j * PW);
        }
        if (lane == 0) {
            fa_next[tile] = new_w;
            if (new_w & ~ever_w) ever[tile] = ever_w | new_w;
            if (fullnew_w) full[tile] = full_w | fullnew_w;
            n_new += __popcll(new_w);
            n_full += __popcll(fullnew_w);
        }
    }
    if (sub != 0) {
        n_inc = 0;
        n_vis = 0;
    }
    wave_add_sh(ctr + cNewFull, n_full);
    wave_add_sh(ctr + cIncLight, n_inc);
    wave_add_sh(ctr + cVisLight, n_vis);
    wave_add_sh(ctr + cNewLight, n_new);
    wave_add_sh(ctr + cNewAtoms, n_new);
    wave_add_sh(ctr + cNewDeg, n_newdeg);
    wave_add_sh(ctr + cNewDegNF, n_newdeg_nf);
}

// ---------------------------------------------------------------------------------------------
// Dense levels, W >= 8 (G >= 4 lanes per row): the same gather / pull as above, restructured for
// memory-level parallelism.  The kernels above walk one row per G-lane group through a chain of
// dependent loads (offsets -> ids -> bitmap probes -> mask rows), one step of the chain in flight
// per group; here a wave first loads the offsets of all 64 rows of its tile (one coalesced load),
// then the ids of every row of the tile, then every probe, then the mask rows -- G independent
// loads in flight per lane at each stage.  Tiles with no work (e.g. the link atoms' zero-degree
// rows) cost one load.
// ---------------------------------------------------------------------------------------------
template <int W, bool WRITE_LF>
__device__ __forceinline__ void gather2_body(int64_t M, const int64_t* __restrict__ tgt_off,
                                             const int32_t* __restrict__ tgt_idx,
                                             const int32_t* __restrict__ link_type, int32_t want_type,
                                             const u64* __restrict__ fa, const u64* __restrict__ full,
                                             const u64* __restrict__ lvl, u64* __restrict__ lf,
                                             u64* __restrict__ la, u64* __restrict__ ctr, FullMask fm, int flags) {
    constexpr int WPL = Lay<W>::WPL, G = Lay<W>::G, PW = Lay<W>::PER_WAVE;
    static_assert(G >= 4, "gather2 needs G >= 4");
    typedef Vec<WPL> V;
    const bool early = flags & 1, skip_full = flags & 4, all_rows = flags & kAllRows;
    const bool nt_idx = flags & kNtIdx, nt_lf = flags & kNtLf;
    const int lane = threadIdx.x & 63, g = lane / G, sub = lane & (G - 1), base = lane & ~(G - 1);
    const u64 gmask = (1ull << G) - 1ull;
    const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    const int64_t nwave = ((int64_t)gridDim.x * blockDim.x) >> 6;
    const typename V::T FULL = full_part<W>(fm, sub);
    u64 n_links = 0, n_pins = 0;
    for (int64_t tile = wave; tile * 64 < M; tile += nwave) {
        const int64_t Lme = tile * 64 + lane;
        int64_t bme = 0;
        int nme = 0;
        if (Lme < M && (want_type < 0 || link_type[Lme] == want_type)) {
            bme = ld_col(tgt_off + Lme, nt_idx);
            nme = (int)(ld_col(tgt_off + Lme + 1, nt_idx) - bme);
        }
        int32_t v[G];
        int n[G];
        int64_t bb[G];
#pragma unroll
        for (int j = 0; j < G; ++j) {
            bb[j] = __shfl(bme, j * PW + g);
            n[j] = __shfl(nme, j * PW + g);
            v[j] = sub < n[j] ? ld_col(tgt_idx + bb[j] + sub, nt_idx) : -1;
        }
        unsigned pa = 0, pnf = 0;
#pragma unroll
        for (int j = 0; j < G; ++j)
            if (v[j] >= 0) {
                if (bit(fa, v[j])) pa |= 1u << j;
                if (!skip_full || !bit(full, v[j])) pnf |= 1u << j;
            }
        u64 word = 0;
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const int64_t L = tile * 64 + j * PW + g;
            unsigned ga = (unsigned)((__ballot((pa >> j) & 1u) >> base) & gmask);
            const bool any_nf0 = ((__ballot((pnf >> j) & 1u) >> base) & gmask) != 0ull;
            typename V::T acc = V::zero();
            int nact = 0;
            bool act = false;
            if (n[j] <= G) {
                if (any_nf0 && ga) {   // group-uniform
                    typename V::T r[G];
#pragma unroll
                    for (int k = 0; k < G; ++k) {
                        const int32_t vk = __shfl(v[j], base + k);
                        r[k] = ((ga >> k) & 1u) ? V::ld(lvl + (int64_t)vk * W + sub * WPL) : V::zero();
                    }
#pragma unroll
                    for (int k = 0; k < G; ++k) acc |= r[k];
                }
                nact = __popc(ga);
                act = nact > 0 && any_nf0;
            } else {   // a row longer than G (rare): full bits first, then the rows with early exit
                const int64_t b = bb[j], e = b + n[j];
                bool any_not_full = !skip_full;
                for (int64_t p = b; p < e && !any_not_full; p += G) {
                    const int64_t q = p + sub;
                    const int32_t myv = q < e ? tgt_idx[q] : -1;
                    any_not_full |= ((__ballot(myv >= 0 && !bit(full, myv)) >> base) & gmask) != 0ull;
                }
                for (int64_t p = b; p < e && any_not_full; p += G) {
                    const int64_t q = p + sub;
                    const int32_t myv = q < e ? tgt_idx[q] : -1;
                    const unsigned g2 = (unsigned)((__ballot(myv >= 0 && bit(fa, myv)) >> base) & gmask);
                    typename V::T r[G];
#pragma unroll
                    for (int k = 0; k < G; ++k) {
                        const int32_t vk = __shfl(myv, base + k);
                        r[k] = ((g2 >> k) & 1u) ? V::ld(lvl + (int64_t)vk * W + sub * WPL) : V::zero();
                    }
#pragma unroll
                    for (int k = 0; k < G; ++k) acc |= r[k];
                    nact += __popc(g2);
                    if (early && p + G < e && group_all<G>(V::eq(acc, FULL))) break;
                }
                act = nact > 0 && any_not_full;
            }
            if (act) {
                if (WRITE_LF) st_row<V>(lf + L * W + sub * WPL, acc, nt_lf);
                if (sub == 0) {
                    ++n_links;
                    n_pins += nact;
                }
            } else if (WRITE_LF && all_rows && L < M) {
                st_row<V>(lf + L * W + sub * WPL, V::zero(), nt_lf);   // the pull reads every row unprobed
            }
            word |= compress_groups<G>(__ballot(act), j * PW);
        }
        if (lane == 0) la[tile] = word;
    }
    wave_add_sh(ctr + cActiveLinks, n_links);
    wave_add_sh(ctr + cActivePins, n_pins);
}

template <int W, bool WRITE_LF>
__global__ void __launch_bounds__(256) hgx_link_gather2(int64_t M, const int64_t* __restrict__ tgt_off,
                                                        const int32_t* __restrict__ tgt_idx,
                                                        const int32_t* __restrict__ link_type, int32_t want_type,
                                                        const u64* __restrict__ fa, const u64* __restrict__ full,
                                                        const u64* __restrict__ lvl, u64* __restrict__ lf,
                                                        u64* __restrict__ la, u64* __restrict__ ctr, FullMask fm,
                                                        int flags) {
    gather2_body<W, WRITE_LF>(M, tgt_off, tgt_idx, link_type, want_type, fa, full, lvl, lf, la, ctr, fm, flags);
}

// Diagnostic only (HGX_OPT_BFS_FLAGS bit 10, A/B): the same gather forced to 5 waves/SIMD, which
// makes the compiler spill ~47 VGPRs per lane to scratch (round 1 saw wrong
// level sizes from such a build; tools/ab_bfs.py compares its per-source results with the default).
template <int W, bool WRITE_LF>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5, 5)))
hgx_link_gather2_o5(int64_t M, const int64_t* __restrict__ tgt_off, const int32_t* __restrict__ tgt_idx,
                    const int32_t* __restrict__ link_type, int32_t want_type, const u64* __restrict__ fa,
                    const u64* __restrict__ full, const u64* __restrict__ lvl, u64* __restrict__ lf,
                    u64* __restrict__ la, u64* __restrict__ ctr, FullMask fm, int flags) {
    gather2_body<W, WRITE_LF>(M, tgt_off, tgt_idx, link_type, want_type, fa, full, lvl, lf, la, ctr, fm, flags);
}

template <int W, int JBX, bool SORT, int KR>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(KR < Lay<W>::G ? 4 : 1, 8))) hgx_atom_pull2(int64_t A, const int64_t* __restrict__ inc_off,
                                                      const int32_t* __restrict__ inc_row,
                                                      const u64* __restrict__ la, const u64* __restrict__ lf,
                                                      u64* __restrict__ vis, u64* __restrict__ ever,
                                                      u64* __restrict__ full, u64* __restrict__ lvl_next,
                                                      u64* __restrict__ fa_next, u64* __restrict__ ctr, FullMask fm,
                                                      int flags, const u64* __restrict__ own) {
    constexpr int WPL = Lay<W>::WPL, G = Lay<W>::G, PW = Lay<W>::PER_WAVE;
    constexpr int JB = G >= 8 ? JBX : G;   // atoms of a group interleaved at once (register budget)
    static_assert(G >= 4, "pull2 needs G >= 4");
    typedef Vec<WPL> V;
    const bool early = flags & 2, skip_full = flags & 4, all_rows = flags & kAllRows;
    const bool nt_idx = flags & kNtIdx, nt_out = flags & kNtOut;
    const int lane = threadIdx.x & 63, g = lane / G, sub = lane & (G - 1), base = lane & ~(G - 1);
    const u64 gmask = (1ull << G) - 1ull;
    const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    const int64_t nwave = ((int64_t)gridDim.x * blockDim.x) >> 6;
    const typename V::T FULL = full_part<W>(fm, sub);
    u64 n_inc = 0, n_vis = 0, n_new = 0, n_newdeg = 0, n_newdeg_nf = 0, n_full = 0;
    for (int64_t tile = wave; tile * 64 < A; tile += nwave) {
        const u64 ever_w = ever[tile], full_w = full[tile];
        // partition part: a ghost's new row is partial and its vis / ever are rewritten by the
        // broadcast of the owner's final row (hgx_x_apply), so the pull writes neither for ghosts
        const u64 own_w = own ? own[tile] : ~0ull;
        const int64_t tme = tile * 64 + lane;
        int64_t bme = 0;
        int dme = 0;
        if (tme < A && !(skip_full && ((full_w >> lane) & 1ull))) {
            bme = ld_col(inc_off + tme, nt_idx);
            const int64_t d = ld_col(inc_off + tme + 1, nt_idx) - bme;
            dme = (d > 0 && d <= kHeavyDegree) ? (int)d : 0;
        }
        if (__ballot(dme > 0) == 0ull) {   // nothing to pull in this tile
            if (lane == 0) fa_next[tile] = 0ull;
            continue;
        }
        // SORT (A/B, bit 11): the atoms of the tile go to the (j0, group) slots in descending degree
        // order, so the JB * PW atoms interleaved together have similar degrees (the wave-uniform chunk
        // loop runs to the largest degree among them; unsorted, power-law degrees leave ~40% of the
        // lane slots idle on config 2).  Bitonic sort of (degree << 6 | lane) over the wave; slot i
        // takes the atom at lane key[i] & 63.  Unsorted, slot i is lane i.
        uint32_t key = ((uint32_t)dme << 6) | (uint32_t)lane;
        if constexpr (SORT) {
#pragma unroll
            for (int k2 = 2; k2 <= 64; k2 <<= 1) {
#pragma unroll
                for (int j2 = k2 >> 1; j2 > 0; j2 >>= 1) {
                    const uint32_t other = (uint32_t)__shfl_xor((int)key, j2);
                    const bool up = ((lane & k2) == 0) == ((lane & j2) == 0);   // keep the larger key here
                    key = up ? max(key, other) : min(key, other);
                }
            }
        }
        u64 new_w = 0, fullnew_w = 0;
        for (int j0 = 0; j0 < G; j0 += JB) {
            int64_t bj[JB];
            int dj[JB], sl[JB], dmax = 0;
            typename V::T acc[JB], old[JB];
            bool hv[JB], done[JB];
#pragma unroll
            for (int jj = 0; jj < JB; ++jj) {
                sl[jj] = SORT ? (int)((uint32_t)__shfl((int)key, (j0 + jj) * PW + g) & 63u) : (j0 + jj) * PW + g;
                bj[jj] = __shfl(bme, sl[jj]);
                dj[jj] = __shfl(dme, sl[jj]);
                acc[jj] = V::zero();
                old[jj] = V::zero();
                hv[jj] = false;
                done[jj] = dj[jj] == 0;
                dmax = max(dmax, dj[jj]);
            }
            for (int off = 32; off > 0; off >>= 1) dmax = max(dmax, __shfl_xor(dmax, off));
            for (int c0 = 0; c0 < dmax; c0 += G) {   // wave-uniform
                int32_t myL[JB];
#pragma unroll
                for (int jj = 0; jj < JB; ++jj)
                    myL[jj] = (!done[jj] && c0 + sub < dj[jj]) ? ld_col(inc_row + bj[jj] + c0 + sub, nt_idx) : -1;
                unsigned pa = 0;
#pragma unroll
                for (int jj = 0; jj < JB; ++jj)
                    if (myL[jj] >= 0 && (all_rows || bit(la, myL[jj]))) pa |= 1u << jj;
#pragma unroll
                for (int jj = 0; jj < JB; ++jj) {
                    const unsigned ga = (unsigned)((__ballot((pa >> jj) & 1u) >> base) & gmask);
                    if (ga) {   // group-uniform
                        // KR of the G rows in flight at once (KR < G: fewer VGPRs, more waves/SIMD)
#pragma unroll
                        for (int k0 = 0; k0 < G; k0 += KR) {
                            typename V::T r[KR];
#pragma unroll
                            for (int k = 0; k < KR; ++k) {
                                const int32_t Lk = __shfl(myL[jj], base + k0 + k);
                                r[k] = ((ga >> (k0 + k)) & 1u) ? V::ld(lf + (int64_t)Lk * W + sub * WPL) : V::zero();
                            }
#pragma unroll
                            for (int k = 0; k < KR; ++k) acc[jj] |= r[k];
                        }
                        n_inc += __popc(ga);
                    }
                    if (done[jj]) continue;   // group-uniform from here on
                    const int64_t t = tile * 64 + sl[jj];
                    if (early) {
                        if (!hv[jj] && group_any<G>(V::nz(acc[jj]))) {
                            if ((ever_w >> sl[jj]) & 1ull) {
                                old[jj] = V::ld(vis + t * W + sub * WPL);
                                ++n_vis;
                            }
                            hv[jj] = true;
                        }
                        if (hv[jj] && c0 + G < dj[jj] && group_all<G>(V::eq(acc[jj] | old[jj], FULL))) done[jj] = true;
                    }
                    if (c0 + G >= dj[jj]) done[jj] = true;
                }
            }
#pragma unroll
            for (int jj = 0; jj < JB; ++jj) {
                const int pos = sl[jj];
                const int64_t t = tile * 64 + pos;
                bool isnew = false, becomes_full = false;
                if (dj[jj] > 0) {   // group-uniform
                    if (!hv[jj] && group_any<G>(V::nz(acc[jj]))) {
                        if ((ever_w >> pos) & 1ull) {
                            old[jj] = V::ld(vis + t * W + sub * WPL);
                            ++n_vis;
                        }
                    }
                    const typename V::T nw = acc[jj] & ~old[jj];
                    if (group_any<G>(V::nz(nw))) {
                        st_row<V>(lvl_next + t * W + sub * WPL, nw, nt_out);
                        if ((own_w >> pos) & 1ull) st_row<V>(vis + t * W + sub * WPL, old[jj] | nw, nt_out);
                        isnew = true;
                        becomes_full = group_all<G>(V::eq(old[jj] | nw, FULL));
                        if (sub == 0) { n_newdeg += (u64)dj[jj]; if (!becomes_full) n_newdeg_nf += (u64)dj[jj]; }
                    }
                }
                if (sub == 0) {   // the atom's own bit (slots are permuted: no ballot compression)
                    new_w |= (u64)isnew << pos;
                    fullnew_w |= (u64)becomes_full << pos;
                }
            }
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            new_w |= (u64)__shfl_xor((long long)new_w, off);
            fullnew_w |= (u64)__shfl_xor((long long)fullnew_w, off);
        }
        if (lane == 0) {
            fa_next[tile] = new_w;
            if (new_w & own_w & ~ever_w) ever[tile] = ever_w | (new_w & own_w);
            if (fullnew_w) full[tile] = full_w | fullnew_w;
            n_new += __popcll(new_w);
            n_full += __popcll(fullnew_w);
        }
    }
    if (sub != 0) {
        n_inc = 0;
        n_vis = 0;
    }
    wave_add_sh(ctr + cNewFull, n_full);
    wave_add_sh(ctr + cIncLight, n_inc);
    wave_add_sh(ctr + cVisLight, n_vis);
    wave_add_sh(ctr + cNewLight, n_new);
    wave_add_sh(ctr + cNewAtoms, n_new);
    wave_add_sh(ctr + cNewDeg, n_newdeg);
    wave_add_sh(ctr + cNewDegNF, n_newdeg_nf);
}

// pull_range for the symmetric mode, G >= 4, restructured for memory-level parallelism: a group
// loads U chunks of G incidence entries at once, probes their la bits together (no probe when every
// lf row was written, kAllRows) and then issues all U*G lf row loads before ORing them.  The early
// exit is tested every U*G entries; ORing rows past the point where acc | old covers FULL changes
// nothing in acc & ~old, so the result is the same as pull_range's.
template <int W, int U>
__device__ __forceinline__ void pull_range_mlp(int64_t b, int64_t e, const int32_t* __restrict__ inc_row,
                                               const u64* __restrict__ la, const u64* __restrict__ lf,
                                               const u64* __restrict__ vis_row, bool have_vis,
                                               typename Vec<Lay<W>::WPL>::T FULL, int sub,
                                               typename Vec<Lay<W>::WPL>::T& acc, typename Vec<Lay<W>::WPL>::T& old,
                                               bool& have_old, u64& n_inc, u64& n_vis, bool early, bool all_rows) {
    constexpr int WPL = Lay<W>::WPL, G = Lay<W>::G;
    static_assert(G >= 4, "pull_range_mlp needs G >= 4");
    typedef Vec<WPL> V;
    const int base = (threadIdx.x & 63) & ~(G - 1);
    for (int64_t i = b; i < e; i += U * G) {
        int32_t myL[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t q = i + u * G + sub;
            myL[u] = q < e ? inc_row[q] : -1;
        }
        unsigned ga[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool mya = myL[u] >= 0 && (all_rows || bit(la, myL[u]));
            ga[u] = (unsigned)((__ballot(mya) >> base) & ((1ull << G) - 1ull));
        }
        typename V::T r[U][G];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int k = 0; k < G; ++k) {
                const int32_t Lk = __shfl(myL[u], base + k);
                r[u][k] = ((ga[u] >> k) & 1u) ? V::ld(lf + (int64_t)Lk * W + sub * WPL) : V::zero();
            }
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
            for (int k = 0; k < G; ++k) acc |= r[u][k];
            n_inc += __popc(ga[u]);
        }
        if (!early) continue;
        if (!have_old && group_any<G>(V::nz(acc))) {
            if (have_vis) {
                old = V::ld(vis_row + sub * WPL);
                ++n_vis;
            }
            have_old = true;
        }
        if (have_old && i + U * G < e && group_all<G>(V::eq(acc | old, FULL))) break;
    }
}

// Heavy atoms: one workgroup per chunk of <= kChunkEntries incidence entries; groups OR their
// share (stopping early once every traversal is covered), the block reduces through LDS and ORs
// the chunk result into hubacc[slot].  Hubs already visited by every traversal exit at once.
template <int W, int MODE>
__global__ void __launch_bounds__(256) hgx_atom_pull_heavy(const HeavyChunk* __restrict__ chunks,
                                                           const int32_t* __restrict__ inc_row,
                                                           const u64* __restrict__ la, const u64* __restrict__ lf,
                                                           const int64_t* __restrict__ tgt_off,
                                                           const int32_t* __restrict__ tgt_idx,
                                                           const u64* __restrict__ fa, const u64* __restrict__ lvl,
                                                           const u64* __restrict__ vis, const u64* __restrict__ ever,
                                                           const u64* __restrict__ full, u64* __restrict__ hubacc,
                                                           u64* __restrict__ ctr, FullMask fm, int flags,
                                                           const u64* __restrict__ cand) {
    constexpr int WPL = Lay<W>::WPL, G = Lay<W>::G;
    constexpr int NG = 256 / G;
    typedef Vec<WPL> V;
    __shared__ u64 red[NG * W];
    const HeavyChunk c = chunks[blockIdx.x];
    if ((flags & 4) && bit(full, c.atom)) return;   // block-uniform
    if (cand && !bit(cand, c.atom)) return;
    const int sub = threadIdx.x & (G - 1);
    const int gi = threadIdx.x / G;
    const int64_t n = c.end - c.beg;
    const int64_t per = (n + NG - 1) / NG;
    const int64_t b = c.beg + gi * per;
    const int64_t e = b + per < c.end ? b + per : c.end;
    const typename V::T FULL = full_part<W>(fm, sub);
    u64 n_inc = 0, n_vis = 0;
    typename V::T acc = V::zero(), old = V::zero();
    bool have_old = false;
    bool done = false;
    if constexpr (G >= 4 && MODE == kSym) {
        if (b < e && (flags & kHeavyMlp2) && (flags & kAllRows) && !(flags & 4)) {   // block-uniform
            pull_range_mlp<W, 2>(b, e, inc_row, la, lf, vis + (int64_t)c.atom * W, bit(ever, c.atom), FULL, sub, acc,
                                 old, have_old, n_inc, n_vis, (flags & 2) != 0, true);
            done = true;
        }
    }
    if (b < e && !done)
        pull_range<W, MODE>(c.atom, b, e, inc_row, la, lf, tgt_off, tgt_idx, fa, lvl, vis + (int64_t)c.atom * W,
                            bit(ever, c.atom), FULL, sub, acc, old, have_old, n_inc, n_vis, (flags & 2) != 0);
    V::st(red + gi * W + sub * WPL, acc);
    __syncthreads();
    for (int j = threadIdx.x; j < W; j += 256) {
        u64 r = 0;
        for (int k = 0; k < NG; ++k) r |= red[k * W + j];
        if (r) atomicOr(hubacc + (int64_t)c.slot * W + j, r);
    }
    if (sub != 0) n_inc = 0;
    wave_add_sh(ctr + cIncHeavy, n_inc);
}

template <int W>
__global__ void __launch_bounds__(256) hgx_hub_finalize(int64_t H, const int32_t* __restrict__ heavy_atom,
                                                        const int64_t* __restrict__ inc_off,
                                                        u64* __restrict__ hubacc, u64* __restrict__ vis,
                                                        u64* __restrict__ ever, u64* __restrict__ full,
                                                        u64* __restrict__ lvl_next, u64* __restrict__ fa_next,
                                                        u64* __restrict__ ctr, FullMask fm) {
    constexpr int WPL = Lay<W>::WPL, G = Lay<W>::G;
    typedef Vec<WPL> V;
    const int sub = threadIdx.x & (G - 1);
    const int64_t grp = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / G;
    const int64_t ngrp = ((int64_t)gridDim.x * blockDim.x) / G;
    const typename V::T FULL = full_part<W>(fm, sub);
    u64 n_acc = 0, n_new = 0, n_newdeg = 0, n_newdeg_nf = 0, n_full = 0;
    for (int64_t h = grp; h < H; h += ngrp) {
        const int64_t t = heavy_atom[h];
        typename V::T acc = V::ld(hubacc + h * W + sub * WPL);
        if (!group_any<G>(V::nz(acc))) continue;
        V::st(hubacc + h * W + sub * WPL, V::zero());
        const bool ev = bit(ever, t);
        typename V::T old = ev ? V::ld(vis + t * W + sub * WPL) : V::zero();
        typename V::T nw = acc & ~old;
        if (sub == 0) ++n_acc;
        if (!group_any<G>(V::nz(nw))) continue;
        V::st(lvl_next + t * W + sub * WPL, nw);
        V::st(vis + t * W + sub * WPL, old | nw);
        const bool becomes_full = group_all<G>(V::eq(old | nw, FULL));
        if (sub == 0) {
            set_bit(fa_next, t);
            if (!ev) set_bit(ever, t);
            if (becomes_full) set_bit(full, t);
            ++n_new;
            n_full += becomes_full;
            { const u64 dg_ = (u64)(inc_off[t + 1] - inc_off[t]); n_newdeg += dg_; if (!becomes_full) n_newdeg_nf += dg_; }
        }
    }
    wave_add_sh(ctr + cNewFull, n_full);
    wave_add_sh(ctr + cAccHub, n_acc);
    wave_add_sh(ctr + cNewHub, n_new);
    wave_add_sh(ctr + cNewAtoms, n_new);
    wave_add_sh(ctr + cNewDeg, n_newdeg);
    wave_add_sh(ctr + cNewDegNF, n_newdeg_nf);
}

// Sparse levels: mark every (typed) link incident to a frontier atom.  One wave per frontier word:
// for each frontier atom of the word, the 64 lanes stride over its incidence row.  Heavy atoms are
// left to hgx_frontier_links_heavy (one workgroup per chunk).
__global__ void __launch_bounds__(256) hgx_frontier_links(int64_t A, const u64* __restrict__ fa,
                                                          const int64_t* __restrict__ inc_off,
                                                          const int32_t* __restrict__ inc_row,
                                                          const int32_t* __restrict__ link_type, int32_t want_type,
                                                          u64* __restrict__ lcand) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    const int64_t nwave = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t w = wave; w * 64 < A; w += nwave) {
        u64 x = fa[w];
        while (x) {
            const int b = __ffsll((long long)x) - 1;
            x &= x - 1;
            const int64_t v = w * 64 + b;
            const int64_t lo = inc_off[v], hi = inc_off[v + 1];
            if (hi - lo > kHeavyDegree) continue;
            for (int64_t i = lo + lane; i < hi; i += 64) {
                const int32_t L = inc_row[i];
                if (want_type < 0 || link_type[L] == want_type) atomicOr(&lcand[L >> 6], 1ull << (L & 63));
            }
        }
    }
}

__global__ void __launch_bounds__(256) hgx_frontier_links_heavy(const HeavyChunk* __restrict__ chunks,
                                                                const u64* __restrict__ fa,
                                                                const int32_t* __restrict__ inc_row,
                                                                const int32_t* __restrict__ link_type,
                                                                int32_t want_type, u64* __restrict__ lcand) {
    const HeavyChunk c = chunks[blockIdx.x];
    if (!bit(fa, c.atom)) return;
    for (int64_t i = c.beg + threadIdx.x; i < c.end; i += 256) {
        const int32_t L = inc_row[i];
        if (want_type < 0 || link_type[L] == want_type) atomicOr(&lcand[L >> 6], 1ull << (L & 63));
    }
}

// ---- sparse levels, default mode: push instead of pull ------------------------------------------
// (1) zero the next-level rows of the candidate atoms, (2) OR every active link's lf row into the
// rows of its targets with 64-bit atomics, (3) finalise the candidates (new = acc & ~vis).

__global__ void __launch_bounds__(256) hgx_push_zero(int64_t A, int W, const u64* __restrict__ cand,
                                                     const u64* __restrict__ full, u64* __restrict__ lvl_next) {
    const int lane = threadIdx.x & 63;
    const int64_t nwords = (A + 63) / 64;
    const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    const int64_t nwave = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t base = wave * 64; base < nwords; base += nwave * 64) {
        const u64 x = base + lane < nwords ? cand[base + lane] & ~full[base + lane] : 0ull;
        u64 m = __ballot(x != 0ull);
        while (m) {
            const int k = __ffsll((long long)m) - 1;
            m &= m - 1ull;
            const int64_t t0 = (base + k) * 64;
            rows_of_word((u64)__shfl(x, k), W, 0, [&](int b, int w, int32_t) { lvl_next[(t0 + b) * W + w] = 0ull; });
        }
    }
}

__global__ void __launch_bounds__(256) hgx_push_rows(int64_t M, int W, const u64* __restrict__ la,
                                                     const int64_t* __restrict__ tgt_off,
                                                     const int32_t* __restrict__ tgt_idx, const u64* __restrict__ lf,
                                                     const u64* __restrict__ full, u64* __restrict__ lvl_next) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    const int64_t nwave = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t w = wave; w * 64 < M; w += nwave) {
        u64 x = la[w];
        while (x) {
            const int64_t L = w * 64 + __ffsll((long long)x) - 1;
            x &= x - 1;
            const int64_t b = tgt_off[L], n = (tgt_off[L + 1] - b) * W;
            for (int64_t j = lane; j < n; j += 64) {
                const int32_t t = tgt_idx[b + j / W];
                const int wd = (int)(j % W);
                const u64 r = lf[L * W + wd];
                if (r && !bit(full, t)) atomicOr(&lvl_next[(int64_t)t * W + wd], r);
            }
        }
    }
}

template <int W>
__global__ void __launch_bounds__(256) hgx_push_finalize(int64_t A, const int64_t* __restrict__ inc_off,
                                                         const u64* __restrict__ cand, u64* __restrict__ vis,
                                                         u64* __restrict__ ever, u64* __restrict__ full,
                                                         u64* __restrict__ lvl_next, u64* __restrict__ fa_next,
                                                         u64* __restrict__ ctr, FullMask fm) {
    constexpr int WPL = Lay<W>::WPL, G = Lay<W>::G, PW = Lay<W>::PER_WAVE;
    typedef Vec<WPL> V;
    const int lane = threadIdx.x & 63, g = lane / G, sub = lane & (G - 1);
    const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    const int64_t nwave = ((int64_t)gridDim.x * blockDim.x) >> 6;
    const int64_t nwords = (A + 63) / 64;
    const typename V::T FULL = full_part<W>(fm, sub);
    u64 n_vis = 0, n_new = 0, n_newdeg = 0, n_newdeg_nf = 0, n_full = 0;
    for (int64_t base = wave * 64; base < nwords; base += nwave * 64) {
        const bool in = base + lane < nwords;
        const u64 myfull = in ? full[base + lane] : 0ull;
        const u64 mycw = in ? cand[base + lane] & ~myfull : 0ull;
        if (in && mycw == 0ull) fa_next[base + lane] = 0ull;   // no candidate: empty frontier word
        u64 m = __ballot(mycw != 0ull);
        while (m) {
            const int kk = __ffsll((long long)m) - 1;
            m &= m - 1ull;
            const int64_t tile = base + kk;
            const u64 cw = __shfl(mycw, kk), full_w = __shfl(myfull, kk);
            const u64 ever_w = ever[tile];
            u64 new_w = 0, fullnew_w = 0;
            for (int j = 0; j < G; ++j) {
                const int pos = j * PW + g;
                const int64_t t = tile * 64 + pos;
                bool isnew = false, becomes_full = false;
                if (t < A && ((cw >> pos) & 1ull)) {
                    const typename V::T acc = V::ld(lvl_next + t * W + sub * WPL);
                    if (group_any<G>(V::nz(acc))) {
                        const bool ev = (ever_w >> pos) & 1ull;
                        const typename V::T old = ev ? V::ld(vis + t * W + sub * WPL) : V::zero();
                        n_vis += ev;
                        const typename V::T nw = acc & ~old;
                        if (group_any<G>(V::nz(nw))) {
                            V::st(lvl_next + t * W + sub * WPL, nw);
                            V::st(vis + t * W + sub * WPL, old | nw);
                            isnew = true;
                            becomes_full = group_all<G>(V::eq(old | nw, FULL));
                            if (sub == 0) { const u64 dg_ = (u64)(inc_off[t + 1] - inc_off[t]); n_newdeg += dg_; if (!becomes_full) n_newdeg_nf += dg_; }
                        }
                    }
                }
                new_w |= compress_groups<G>(__ballot(isnew), j * PW);
                fullnew_w |= compress_groups<G>(__ballot(becomes_full), j * PW);
            }
            if (lane == 0) {
                fa_next[tile] = new_w;
                if (new_w & ~ever_w) ever[tile] = ever_w | new_w;
                if (fullnew_w) full[tile] = full_w | fullnew_w;
                n_new += __popcll(new_w);
                n_full += __popcll(fullnew_w);
            }
        }
    }
    wave_add_sh(ctr + cNewFull, n_full);
    if (sub != 0) n_vis = 0;
    wave_add_sh(ctr + cVisLight, n_vis);
    wave_add_sh(ctr + cNewLight, n_new);
    wave_add_sh(ctr + cNewAtoms, n_new);
    wave_add_sh(ctr + cNewDeg, n_newdeg);
    wave_add_sh(ctr + cNewDegNF, n_newdeg_nf);
}

// ---- sparse levels, ordered modes (hg.subsumed / hg.subsumes): frontier-driven push ------------
// For every frontier atom v and incident (typed) link L, the targets DefaultALGenerator yields from
// v by position (FTargetSetIterator / BTargetSetIterator,
// C/algorithms/DefaultALGenerator.java:121-285) receive v's row.  Pass 0 marks the candidates,
// pass 1 ORs the rows into their (zeroed) next-level rows with 64-bit atomics; hgx_push_finalize
// then applies ~vis.  Work = sum over the frontier of |inc(v)| * arity, independent of |A| -- a
// hub reached as a candidate is never scanned (the pull would scan all of its incidence row).
template <int MODE>
__device__ __forceinline__ bool yields(int pos, int fv, int lv) {
    if constexpr (MODE == kSym) return true;   // every co-target (t != v is checked by the caller)
    else if constexpr (MODE == kAfterFirst) return pos > fv;
    else if constexpr (MODE == kBeforeFirst) return pos < fv;
    else if constexpr (MODE == kBeforeLast) return pos < lv;
    else return pos > lv;   // kAfterLast
}

// Yield flags of incidence entry i = (v, L), bit MODE set <=> DefaultALGenerator in ordered mode
// MODE can yield a target of L from v (a target other than v after / before v's first / last
// position).  A frontier atom's push reads the target row of L only when the bit is
// set: a hub's links where it sits at the far end (e.g. the parent end of its HGSubsumes links in
// hg.subsumes) cost one byte each instead of two dependent row loads.  One wave per atom.
__global__ void __launch_bounds__(256) hgx_inc_yield(int64_t A, const int64_t* __restrict__ inc_off,
                                                     const int32_t* __restrict__ inc_row,
                                                     const int64_t* __restrict__ tgt_off,
                                                     const int32_t* __restrict__ tgt_idx, uint8_t* __restrict__ yf) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    const int64_t nwave = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t v = wave; v < A; v += nwave) {
        const int64_t e = inc_off[v + 1];
        for (int64_t i = inc_off[v] + lane; i < e; i += 64) {
            const int32_t L = inc_row[i];
            const int64_t b = tgt_off[L];
            const int n = (int)(tgt_off[L + 1] - b);
            int fv = -1, lv = -1;
            for (int p = 0; p < n; ++p)
                if (tgt_idx[b + p] == v) {
                    if (fv < 0) fv = p;
                    lv = p;
                }
            bool after_first = false, before_last = false;
            for (int p = 0; p < n; ++p) {
                const bool other = tgt_idx[b + p] != v;
                after_first |= other && p > fv;
                before_last |= other && p < lv;
            }
            unsigned f = 0;
            if (after_first) f |= 1u << kAfterFirst;
            if (fv > 0) f |= 1u << kBeforeFirst;
            if (before_last) f |= 1u << kBeforeLast;
            if (lv >= 0 && lv < n - 1) f |= 1u << kAfterLast;
            yf[i] = (uint8_t)f;
        }
    }
}

// Per-wave LDS scratch of the frontier push: the yielded targets of one position step and the
// nonzero words of the pushing atom's row.
constexpr int kCBuf = 256;   // candidates staged per wave before one list append
constexpr int kEBuf = 256;   // filtered incidence entries staged per wave
// Frontier push load balance: an atom with more than kPushLight incidences is pushed by blocks of
// four waves over kPushChunk-entry chunks (hgx_opush_heavy), the others by one wave each.
constexpr int64_t kPushLight = 512, kPushChunk = 256;

struct OPushLds {
    int32_t tgt[64];
    int32_t widx[16];
    u64 wval[16];
    int32_t cbuf[kCBuf];     // fresh candidates not yet appended to the candidate list
    int32_t ent[kEBuf];      // incidence entries (relative to the range start) that pass type + yield
};

// Append the wave's staged candidates with one atomic (a same-address atomic per ballot serialises
// on the counter when thousands of waves find candidates).  Wave-uniform call, every lane active.
__device__ __forceinline__ void cand_flush(OPushLds& sh, int& cc, int32_t* __restrict__ clist,
                                           u64* __restrict__ n_clist) {
    const int lane = threadIdx.x & 63;
    if (cc == 0) return;
    u64 base = 0;
    if (lane == 0) base = atomicAdd(n_clist, (u64)cc);
    base = __shfl(base, 0);
    for (int i = lane; i < cc; i += 64) clist[base + i] = sh.cbuf[i];
    __builtin_amdgcn_wave_barrier();
    cc = 0;
}

// Links [start, hi) of frontier atom v (wave-uniform), lane l taking start + l, start + l + step, ...
// Each lane reads its link's target row; position by position the wave ballots the yielded
// targets and spreads the (target, nonzero word of v's row) pairs over the lanes: one 64-bit
// atomicOr into the zero-invariant accumulator per pair and word, skipped when the bits are
// already there (hub targets are hit by many pairs).  The first pair to reach a target sets its
// candidate bit and appends it to the candidate list of the finalise.
template <int W, int MODE>
__device__ __forceinline__ void opush_entry(int32_t v, int64_t i, bool have, const int32_t* __restrict__ inc_row,
                                            const int64_t* __restrict__ tgt_off, const int32_t* __restrict__ tgt_idx,
                                            int nnz, OPushLds& sh, const u64* __restrict__ full,
                                            u64* __restrict__ cand, int32_t* __restrict__ clist,
                                            u64* __restrict__ n_clist, u64* __restrict__ acc, u64& n_links,
                                            u64& n_pins, u64& n_pairs, int& cc) {
    const int lane = threadIdx.x & 63;
    const u64 lt = (1ull << lane) - 1ull;
    // A row of <= kRegRow targets is held in registers and so are the full-bitmap words of its
    // eligible targets; longer rows take the loop below.  (Inline target records in incidence order --
    // one load instead of link row, target offsets, targets -- measured no faster on config 5 and were
    // removed in round 5: profiles/r03n_c5.log)
    constexpr int kRegRow = 8;
    int32_t tr[kRegRow];
    int64_t b = 0;
    int n = 0, fv = -1, lv = -1;
    if (have) {
        const int32_t L = inc_row[i];
        b = tgt_off[L];
        n = (int)(tgt_off[L + 1] - b);
    }
    if (have) {
        ++n_links;
        n_pins += (u64)n;
    }
    const bool reg = n <= kRegRow;
#pragma unroll
    for (int k = 0; k < kRegRow; ++k) tr[k] = (reg && k < n) ? tgt_idx[b + k] : -1;
    if (reg) {
#pragma unroll
        for (int k = 0; k < kRegRow; ++k)
            if (tr[k] == v) {
                if (fv < 0) fv = k;
                lv = k;
            }
    } else {
        for (int p = 0; p < n; ++p)
            if (tgt_idx[b + p] == v) {
                if (fv < 0) fv = p;
                lv = p;
            }
    }
    unsigned em = 0;   // eligible register positions
    if (reg) {
        u64 fw[kRegRow];
#pragma unroll
        for (int k = 0; k < kRegRow; ++k) {
            const bool e = tr[k] >= 0 && tr[k] != v && yields<MODE>(k, fv, lv);
            fw[k] = e ? full[tr[k] >> 6] : ~0ull;
        }
#pragma unroll
        for (int k = 0; k < kRegRow; ++k)
            if (!((fw[k] >> (tr[k] & 63)) & 1ull)) em |= 1u << k;
    }
    int nmax = n;
    for (int off = 32; off > 0; off >>= 1) nmax = max(nmax, __shfl_xor(nmax, off));
    for (int p = 0; p < nmax; ++p) {
        int32_t t = -1;
        bool elig;
        if (reg) {
#pragma unroll
            for (int k = 0; k < kRegRow; ++k)
                if (k == p) t = tr[k];
            elig = (em >> p) & 1u;
        } else {
            t = p < n ? tgt_idx[b + p] : -1;
            elig = t >= 0 && t != v && yields<MODE>(p, fv, lv) && !bit(full, t);
        }
        const u64 m = __ballot(elig);
        if (m == 0ull) continue;
        n_pairs += elig;
        if (elig) sh.tgt[__popcll(m & lt)] = t;
        __builtin_amdgcn_wave_barrier();
        const int total = __popcll(m) * nnz;
        for (int q0 = 0; q0 < total; q0 += 64) {   // wave-uniform trip count
            const int q = q0 + lane;
            bool fresh = false;
            int32_t ts = 0;
            if (q < total) {
                const int pr = q / nnz, wi = q - pr * nnz;
                ts = sh.tgt[pr];
                u64* a = acc + (int64_t)ts * W + sh.widx[wi];
                const u64 val = sh.wval[wi];
                if ((*a & val) != val) atomicOr(a, val);
                if (wi == 0) {
                    const u64 cb = 1ull << (ts & 63);
                    if (!(cand[ts >> 6] & cb)) fresh = !(atomicOr(&cand[ts >> 6], cb) & cb);
                }
            }
            const u64 fm = __ballot(fresh);
            if (fm) {   // wave-uniform: stage the fresh candidates in LDS
                const int nf = __popcll(fm);
                if (cc + nf > kCBuf) cand_flush(sh, cc, clist, n_clist);
                if (fresh) sh.cbuf[cc + __popcll(fm & lt)] = ts;
                cc += nf;
                __builtin_amdgcn_wave_barrier();
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// Entries [start, hi) of frontier atom v (wave-uniform), lane l taking start + l, start + l + step, ...
// Stage 1 streams the type column and the yield flags kUnroll chunks at a time (independent loads)
// and compacts the passing entries into an LDS list; stage 2 runs the dependent chain (link row,
// target offsets, target row, full bits, accumulator atomics) only for those, 64 per pass.  A hub's
// links that cannot yield (most of them in hg.subsumes) thus cost streamed bytes, not round trips.
template <int W, int MODE>
__device__ __forceinline__ void opush_links(int32_t v, int64_t start, int64_t hi, int64_t step,
                                            const int32_t* __restrict__ inc_row,
                                            const int32_t* __restrict__ inc_type, int32_t want_type,
                                            const uint8_t* __restrict__ yf,
                                            const int64_t* __restrict__ tgt_off, const int32_t* __restrict__ tgt_idx,
                                            int nnz, OPushLds& sh, const u64* __restrict__ full,
                                            u64* __restrict__ cand, int32_t* __restrict__ clist,
                                            u64* __restrict__ n_clist, u64* __restrict__ acc, u64& n_links,
                                            u64& n_pins, u64& n_pairs, u64& n_scan, int& cc) {
    constexpr int kUnroll = 4;
    const int lane = threadIdx.x & 63;
    const u64 lt = (1ull << lane) - 1ull;
    int ne = 0;   // staged entries (wave-uniform)
    auto drain = [&]() {
        for (int k0 = 0; k0 < ne; k0 += 64) {   // wave-uniform
            const bool have = k0 + lane < ne;
            const int64_t i = have ? start + sh.ent[k0 + lane] : 0;
            opush_entry<W, MODE>(v, i, have, inc_row, tgt_off, tgt_idx, nnz, sh, full, cand, clist, n_clist, acc,
                                 n_links, n_pins, n_pairs, cc);
        }
        __builtin_amdgcn_wave_barrier();
        ne = 0;
    };
    for (int64_t i0 = start; i0 < hi; i0 += step * kUnroll) {   // i0 is wave-uniform
        bool pass[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const int64_t i = i0 + u * step + lane;
            pass[u] = i < hi;
        }
        if (want_type >= 0) {
            int32_t ty[kUnroll];
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) ty[u] = pass[u] ? inc_type[i0 + u * step + lane] : want_type;
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) pass[u] = pass[u] && ty[u] == want_type;
        }
        if constexpr (MODE != kSym) {
            uint8_t f[kUnroll];
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) f[u] = pass[u] ? yf[i0 + u * step + lane] : (uint8_t)0;
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) pass[u] = pass[u] && ((f[u] >> MODE) & 1u);
        }
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const int64_t i = i0 + u * step + lane;
            n_scan += i < hi;
            const u64 m = __ballot(pass[u]);
            if (m == 0ull) continue;   // wave-uniform
            if (ne + 64 > kEBuf) drain();
            if (pass[u]) sh.ent[ne + __popcll(m & lt)] = (int32_t)(i - start);
            ne += __popcll(m);
            __builtin_amdgcn_wave_barrier();
        }
    }
    if (ne) drain();
}

// The nonzero words of a row (lane w holds word w, already loaded) into the wave's LDS table; returns
// their count (wave-uniform).
__device__ __forceinline__ int row_words_of(u64 x, OPushLds& sh) {
    const int lane = threadIdx.x & 63;
    const u64 nz = __ballot(x != 0ull);
    if (x != 0ull) {
        const int r = __popcll(nz & ((1ull << lane) - 1ull));
        sh.widx[r] = lane;
        sh.wval[r] = x;
    }
    __builtin_amdgcn_wave_barrier();
    return __popcll(nz);
}

// The nonzero words of v's row into the wave's LDS table; returns their count (wave-uniform).
template <int W>
__device__ __forceinline__ int row_words(const u64* __restrict__ lvl, int64_t v, OPushLds& sh) {
    const int lane = threadIdx.x & 63;
    const u64 x = lane < W ? lvl[v * W + lane] : 0ull;
    const u64 nz = __ballot(x != 0ull);
    if (x != 0ull) {
        const int r = __popcll(nz & ((1ull << lane) - 1ull));
        sh.widx[r] = lane;
        sh.wval[r] = x;
    }
    __builtin_amdgcn_wave_barrier();
    return __popcll(nz);
}

// Light frontier atoms (0 < deg <= kHeavyDegree) appended to a list (order-free), so the push
// kernels give one wave per atom whatever the bitmap's sparsity.  A thread owns one frontier word;
// a block counts its words' atoms, claims its list range with one atomic, then writes them (a
// per-wave atomic on the list counter serialised: 76 us per level on config 5's sparse frontiers).
__global__ void __launch_bounds__(256) hgx_frontier_list(int64_t A, const u64* __restrict__ fa,
                                                         const int64_t* __restrict__ inc_off,
                                                         int32_t* __restrict__ list, u64* __restrict__ n_list,
                                                         int64_t light_max) {
    __shared__ int wsum[4];
    __shared__ u64 sbase;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t nw = (A + 63) / 64;
    // the light atoms of word w
    auto keep_of = [&](int64_t w) -> u64 {
        if (w >= nw) return 0ull;
        u64 x = fa[w], keep = 0ull;
        for (u64 y = x; y; y &= y - 1ull) {
            const int b = __ffsll((long long)y) - 1;
            const int64_t v = w * 64 + b;
            const int64_t d = inc_off[v + 1] - inc_off[v];
            if (d > 0 && d <= light_max) keep |= 1ull << b;
        }
        return keep;
    };
    auto block_scan = [&](int c, int& before, int& total) {
        int incl = c;
        for (int off = 1; off < 64; off <<= 1) {
            const int y = __shfl_up(incl, off);
            if (lane >= off) incl += y;
        }
        if (lane == 63) wsum[wv] = incl;
        __syncthreads();
        before = 0;
        total = 0;
        for (int k = 0; k < 4; ++k) {
            before += k < wv ? wsum[k] : 0;
            total += wsum[k];
        }
        __syncthreads();
        before += incl - c;
    };
    // pass 1: the block's total over all its chunks -> one atomic
    int mine = 0;
    for (int64_t w0 = (int64_t)blockIdx.x * 256; w0 < nw; w0 += (int64_t)gridDim.x * 256)
        mine += __popcll(keep_of(w0 + threadIdx.x));
    int before, total;
    block_scan(mine, before, total);
    if (threadIdx.x == 0) sbase = total ? atomicAdd(n_list, (u64)total) : 0ull;
    __syncthreads();
    if (total == 0) return;   // block-uniform
    // pass 2: positions in chunk order
    u64 run = sbase;
    for (int64_t w0 = (int64_t)blockIdx.x * 256; w0 < nw; w0 += (int64_t)gridDim.x * 256) {   // block-uniform
        const int64_t w = w0 + threadIdx.x;
        u64 keep = keep_of(w);
        int b4, t4;
        block_scan(__popcll(keep), b4, t4);
        u64 pos = run + (u64)b4;
        while (keep) {
            const int b = __ffsll((long long)keep) - 1;
            list[pos++] = (int32_t)(w * 64 + b);
            keep &= keep - 1ull;
        }
        run += (u64)t4;
    }
}

template <int W, int MODE>
__global__ void __launch_bounds__(256) hgx_opush(const int32_t* __restrict__ list, const u64* __restrict__ n_list,
                                                 const int64_t* __restrict__ inc_off,
                                                 const int32_t* __restrict__ inc_row,
                                                 const int32_t* __restrict__ inc_type, int32_t want_type,
                                                 const uint8_t* __restrict__ yf,
                                                 const int64_t* __restrict__ tgt_off,
                                                 const int32_t* __restrict__ tgt_idx, const u64* __restrict__ lvl,
                                                 const u64* __restrict__ full, u64* __restrict__ cand,
                                                 int32_t* __restrict__ clist, u64* __restrict__ n_clist,
                                                 u64* __restrict__ acc, u64* __restrict__ ctr,
                                                 u64* __restrict__ fa_next, int64_t n_words,
                                                 const HeavyChunk* __restrict__ chunks, int64_t n_chunks,
                                                 const u64* __restrict__ fa) {
    __shared__ OPushLds lds[4];
    OPushLds& sh = lds[threadIdx.x >> 6];
    const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    const int64_t nwave = ((int64_t)gridDim.x * blockDim.x) >> 6;
    // the next frontier bitmap (set by the finalise) is cleared here instead of by a memset
    for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < n_words; w += (int64_t)gridDim.x * blockDim.x)
        fa_next[w] = 0ull;
    u64 n_links = 0, n_pins = 0, n_pairs = 0, n_scan = 0;
    int cc = 0;   // staged candidates (wave-uniform)
    // hub chunks first (the hgx_opush_heavy launch folded in: one launch less per level): a block per
    // kPushChunk-entry chunk of a frontier hub, its four waves striding over the chunk
    for (int64_t ch = blockIdx.x; ch < n_chunks; ch += gridDim.x) {   // block-uniform
        const HeavyChunk c = chunks[ch];
        if (!bit(fa, c.atom)) continue;
        const int nnz = row_words<W>(lvl, c.atom, sh);
        if (nnz == 0) continue;
        opush_links<W, MODE>(c.atom, c.beg + (threadIdx.x >> 6) * 64, c.end, 256, inc_row, inc_type, want_type, yf,
                             tgt_off, tgt_idx, nnz, sh, full, cand, clist, n_clist, acc, n_links, n_pins, n_pairs,
                             n_scan, cc);
    }
    const int64_t n = (int64_t)*n_list;
    // A wave pushes the atoms k, k + nwave, ... of the list one after the other; the list entry, the
    // incidence range and the row of the NEXT atom (three dependent round trips of every atom) are
    // loaded while this one is pushed.  A list entry < 0: a candidate list reused as the frontier list
    // (not new / not light).
    const int lane = threadIdx.x & 63;
    auto list_at = [&](int64_t k) -> int32_t { return k < n ? list[k] : -1; };
    int64_t k = wave;
    int32_t v = list_at(k), vn = list_at(k + nwave);
    int64_t beg = 0, end = 0;
    u64 x = 0ull;
    if (v >= 0) {
        beg = inc_off[v];
        end = inc_off[v + 1];
        x = lane < W ? lvl[(int64_t)v * W + lane] : 0ull;
    }
    for (; k < n; k += nwave) {   // wave-uniform
        const int32_t vnn = list_at(k + 2 * nwave);
        int64_t nbeg = 0, nend = 0;
        u64 nx = 0ull;
        if (vn >= 0) {
            nbeg = inc_off[vn];
            nend = inc_off[vn + 1];
            nx = lane < W ? lvl[(int64_t)vn * W + lane] : 0ull;
        }
        if (v >= 0) {
            const int nnz = row_words_of(x, sh);
            if (nnz)
                opush_links<W, MODE>(v, beg, end, 64, inc_row, inc_type, want_type, yf, tgt_off, tgt_idx, nnz, sh,
                                     full, cand, clist, n_clist, acc, n_links, n_pins, n_pairs, n_scan, cc);
        }
        v = vn;
        vn = vnn;
        beg = nbeg;
        end = nend;
        x = nx;
    }
    cand_flush(sh, cc, clist, n_clist);
    wave_add_sh(ctr + cActiveLinks, n_links);
    wave_add_sh(ctr + cActivePins, n_pins);
    wave_add_sh(ctr + cIncLight, n_pairs);
    wave_add_sh(ctr + cScanned, n_scan);
}

// (The flattened push of round 2, HGX_OPT_PUSH_BATCH K > 0 -- K frontier atoms a wave, their entries in
// one stream -- was slower on the sum of config 5's directions at every K and was removed in round 5.)

template <int W, int MODE>
__global__ void __launch_bounds__(256) hgx_opush_heavy(const HeavyChunk* __restrict__ chunks,
                                                       const u64* __restrict__ fa,
                                                       const int32_t* __restrict__ inc_row,
                                                       const int32_t* __restrict__ inc_type, int32_t want_type,
                                                       const uint8_t* __restrict__ yf,
                                                       const int64_t* __restrict__ tgt_off,
                                                       const int32_t* __restrict__ tgt_idx,
                                                       const u64* __restrict__ lvl, const u64* __restrict__ full,
                                                       u64* __restrict__ cand, int32_t* __restrict__ clist,
                                                       u64* __restrict__ n_clist, u64* __restrict__ acc,
                                                       u64* __restrict__ ctr) {
    __shared__ OPushLds lds[4];
    const HeavyChunk c = chunks[blockIdx.x];
    if (!bit(fa, c.atom)) return;   // block-uniform
    const int wib = threadIdx.x >> 6;
    OPushLds& sh = lds[wib];
    const int nnz = row_words<W>(lvl, c.atom, sh);
    if (nnz == 0) return;   // the same row for every wave of the block
    u64 n_links = 0, n_pins = 0, n_pairs = 0, n_scan = 0;
    int cc = 0;
    opush_links<W, MODE>(c.atom, c.beg + wib * 64, c.end, 256, inc_row, inc_type, want_type, yf, tgt_off, tgt_idx,
                         nnz, sh, full, cand, clist, n_clist, acc, n_links, n_pins, n_pairs, n_scan, cc);
    cand_flush(sh, cc, clist, n_clist);
    wave_add_sh(ctr + cActiveLinks, n_links);
    wave_add_sh(ctr + cActivePins, n_pins);
    wave_add_sh(ctr + cIncLight, n_pairs);
    wave_add_sh(ctr + cScanned, n_scan);
}

// The level's counters straight to host memory (no copy in the stream between two levels): the last
// block to finish sums the shards (device-scope atomic reads), stores the totals into the mapped
// host slot, then the sequence number the host spins on.  Every thread of every block calls it.
__device__ __forceinline__ void level_counters_out(u64* __restrict__ ctr, u64* __restrict__ ticket,
                                                   u64* __restrict__ hout, u64 seq, unsigned nblocks) {
    __shared__ bool last;
    __syncthreads();   // the block's counter atomics are issued
    if (threadIdx.x == 0) {
        __threadfence();
        last = atomicAdd(ticket, 1ull) == (u64)nblocks - 1ull;
    }
    __syncthreads();
    if (!last) return;   // block-uniform
    __threadfence();
    if (threadIdx.x < cNum) {
        u64 v = 0;
        for (int k = 0; k < kCtrShards; ++k) v += atomicAdd(ctr + k * kCtrStride + threadIdx.x, 0ull);
        __hip_atomic_store(hout + threadIdx.x, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) {
        *ticket = 0ull;
        __threadfence_system();
        __hip_atomic_store(hout + cNum, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// Finalise the candidates of a push level: new = acc & ~vis, the accumulator row is re-zeroed.
// One G-lane group per candidate; fa_next (cleared beforehand) / ever / full bits by atomics.
template <int W>
__global__ void __launch_bounds__(256) hgx_push_finalize_list(int32_t* __restrict__ clist,
                                                              const u64* __restrict__ n_clist,
                                                              const int64_t* __restrict__ inc_off,
                                                              u64* __restrict__ acc, u64* __restrict__ cand,
                                                              u64* __restrict__ vis,
                                                              u64* __restrict__ ever, u64* __restrict__ full,
                                                              u64* __restrict__ lvl_next, u64* __restrict__ fa_next,
                                                              u64* __restrict__ ctr, FullMask fm, int relist,
                                                              u64* __restrict__ n_spent, u64* __restrict__ ticket,
                                                              u64* __restrict__ hout, u64 seq,
                                                              u64* __restrict__ lcount) {
    constexpr int WPL = Lay<W>::WPL, G = Lay<W>::G;
    typedef Vec<WPL> V;
    const int64_t n = (int64_t)*n_clist;
    // Blocks past the list leave at once and take no ticket: the grid is sized for the largest lists
    // (512 blocks), a config-5 level lists a few thousand candidates (32 a block per pass at W = 16),
    // and 512 same-address ticket atomics serialise for several microseconds a level.
    const unsigned nactive =
        (unsigned)max((int64_t)1, min((int64_t)gridDim.x, (n + (int64_t)(blockDim.x / G) - 1) / (int64_t)(blockDim.x / G)));
    if (blockIdx.x >= nactive) return;   // block-uniform
    // lcount: the next level's per-source counts, accumulated here (a push level's new rows are sparse:
    // one LDS add per set bit, one global add per nonzero source per block) instead of a readout pass
    __shared__ uint32_t lc[W * 64];
    if (lcount) {
        for (int j = threadIdx.x; j < W * 64; j += blockDim.x) lc[j] = 0u;
        __syncthreads();
    }
    const int sub = threadIdx.x & (G - 1);
    const int64_t grp = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / G;
    const int64_t ngrp = ((int64_t)gridDim.x * blockDim.x) / G;
    const typename V::T FULL = full_part<W>(fm, sub);
    // the consumed frontier list's counter: zero for the next level's candidates (chained levels)
    if (n_spent && blockIdx.x == 0 && threadIdx.x == 0) *n_spent = 0ull;
    u64 n_cand = 0, n_vis = 0, n_new = 0, n_newdeg = 0, n_newdeg_nf = 0, n_full = 0;
    for (int64_t k0 = grp - (grp % (64 / G)); k0 < n; k0 += ngrp) {   // wave-uniform trip count
        const int64_t k = k0 + (grp % (64 / G));
        const bool valid = k < n;
        const int64_t t = valid ? clist[k] : 0;
        typename V::T a = valid ? V::ld(acc + t * W + sub * WPL) : V::zero();
        if (valid) V::st(acc + t * W + sub * WPL, V::zero());
        if (valid && sub == 0) cand[t >> 6] = 0ull;   // every candidate of the word is in the list
        const bool ev = valid && bit(ever, t);
        const typename V::T old = ev ? V::ld(vis + t * W + sub * WPL) : V::zero();
        const typename V::T nw = a & ~old;
        const bool isnew = group_any<G>(V::nz(nw));
        const bool becomes_full = group_all<G>(V::eq(old | nw, FULL));
        int64_t dg = 0;
        if (valid && isnew) {
            V::st(lvl_next + t * W + sub * WPL, nw);
            V::st(vis + t * W + sub * WPL, old | nw);
            if (lcount) {
                if constexpr (WPL == 1) {
                    for (u64 m = nw; m; m &= m - 1ull) atomicAdd(&lc[sub * 64 + __ffsll((long long)m) - 1], 1u);
                } else {
                    for (u64 m = nw.x; m; m &= m - 1ull) atomicAdd(&lc[sub * 128 + __ffsll((long long)m) - 1], 1u);
                    for (u64 m = nw.y; m; m &= m - 1ull) atomicAdd(&lc[sub * 128 + 64 + __ffsll((long long)m) - 1], 1u);
                }
            }
            if (sub == 0) {
                set_bit(fa_next, t);
                if (!ev) set_bit(ever, t);
                if (becomes_full) set_bit(full, t);
                ++n_new;
                n_full += becomes_full;
                dg = inc_off[t + 1] - inc_off[t];
                n_newdeg += (u64)dg;
                if (!becomes_full) n_newdeg_nf += (u64)dg;
            }
        }
        // the next push level's frontier list in place: the new light atoms, -1 elsewhere
        if (relist && valid && sub == 0) clist[k] = (dg > 0 && dg <= kPushLight) ? (int32_t)t : -1;
        if (valid && sub == 0) {
            ++n_cand;
            n_vis += ev;
        }
    }
    wave_add_sh(ctr + cCand, n_cand);
    wave_add_sh(ctr + cNewFull, n_full);
    wave_add_sh(ctr + cVisLight, n_vis);
    wave_add_sh(ctr + cNewLight, n_new);
    wave_add_sh(ctr + cNewAtoms, n_new);
    wave_add_sh(ctr + cNewDeg, n_newdeg);
    wave_add_sh(ctr + cNewDegNF, n_newdeg_nf);
    if (lcount && __syncthreads_or(n_new != 0)) {   // blocks that found no new atom skip the flush
        for (int j = threadIdx.x; j < W * 64; j += blockDim.x)
            if (lc[j]) atomicAdd(lcount + j, (u64)lc[j]);
    }
    if (hout) level_counters_out(ctr, ticket, hout, seq, nactive);
}

// ---------------------------------------------------------------------------------------------
// Late dense levels (symmetric mode): once most atoms are visited by every traversal ("full"),
// the few that are not pull straight from the frontier rows of their neighbours -- no link gather,
// no lf rows.  Atom t's next row = OR over links L in inc(t) (type-filtered) of OR over targets u
// of L in the frontier of lvl[u] (t's own row is a subset of vis[t] and masks out), minus vis[t].
// ---------------------------------------------------------------------------------------------
// bit v of hasinc <=> inc(v) is non-empty (computed once per snapshot, for the non-full list)
__global__ void __launch_bounds__(256) hgx_hasinc(int64_t A, const int64_t* __restrict__ inc_off,
                                                  u64* __restrict__ hasinc) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    const int64_t nwave = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t w = wave; w * 64 < A; w += nwave) {
        const int64_t v = w * 64 + lane;
        const u64 m = __ballot(v < A && inc_off[v + 1] > inc_off[v]);
        if (lane == 0) hasinc[w] = m;
    }
}

// Atoms with incidence not yet visited by every traversal, appended to a list (order-free).  A
// thread owns one bitmap word; a block scans its 256 words' counts and claims its list range with
// one atomic (a same-address atomic per wave would serialise on the counter).
__global__ void __launch_bounds__(256) hgx_nonfull_list(int64_t A, const u64* __restrict__ full,
                                                        const u64* __restrict__ hasinc, int32_t* __restrict__ list,
                                                        u64* __restrict__ n_list) {
    __shared__ int wsum[4];
    __shared__ u64 sbase;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t nw = (A + 63) / 64;
    for (int64_t w0 = (int64_t)blockIdx.x * 256; w0 < nw; w0 += (int64_t)gridDim.x * 256) {   // block-uniform
        const int64_t w = w0 + threadIdx.x;
        u64 x = w < nw ? (hasinc[w] & ~full[w]) : 0ull;   // hasinc is zero beyond A
        const int c = __popcll(x);
        int incl = c;
        for (int off = 1; off < 64; off <<= 1) {
            const int y = __shfl_up(incl, off);
            if (lane >= off) incl += y;
        }
        if (lane == 63) wsum[wv] = incl;
        __syncthreads();
        int before = 0, total = 0;
        for (int k = 0; k < 4; ++k) {
            before += k < wv ? wsum[k] : 0;
            total += wsum[k];
        }
        if (threadIdx.x == 0) sbase = total ? atomicAdd(n_list, (u64)total) : 0ull;
        __syncthreads();
        u64 pos = sbase + (u64)(before + incl - c);
        while (x) {
            const int b = __ffsll((long long)x) - 1;
            list[pos++] = (int32_t)(w * 64 + b);
            x &= x - 1ull;
        }
        __syncthreads();   // wsum / sbase are rewritten by the next chunk
    }
}

template <int W>
__global__ void __launch_bounds__(256) hgx_nf_pull(const int32_t* __restrict__ list, const u64* __restrict__ n_list,
                                                   const int64_t* __restrict__ inc_off,
                                                   const int32_t* __restrict__ inc_row,
                                                   const int32_t* __restrict__ inc_type, int32_t want_type,
                                                   const int64_t* __restrict__ tgt_off,
                                                   const int32_t* __restrict__ tgt_idx, const u64* __restrict__ fa,
                                                   const u64* __restrict__ lvl, u64* __restrict__ vis,
                                                   u64* __restrict__ ever, u64* __restrict__ full,
                                                   u64* __restrict__ lvl_next, u64* __restrict__ fa_next,
                                                   u64* __restrict__ ctr, FullMask fm, int flags) {
    constexpr int WPL = Lay<W>::WPL, G = Lay<W>::G;
    static_assert(G >= 4, "nf pull needs G >= 4");
    typedef Vec<WPL> V;
    const bool early = flags & 2;
    const int lane = threadIdx.x & 63, sub = lane & (G - 1), base = lane & ~(G - 1);
    const u64 gmask = (1ull << G) - 1ull;
    const int64_t grp = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / G;
    const int64_t ngrp = ((int64_t)gridDim.x * blockDim.x) / G;
    const typename V::T FULL = full_part<W>(fm, sub);
    const int64_t n = (int64_t)*n_list;
    u64 n_cand = 0, n_ent = 0, n_pins = 0, n_rows = 0, n_vis = 0, n_new = 0, n_newdeg = 0, n_newdeg_nf = 0,
        n_full = 0;
    for (int64_t k0 = grp - (grp % (64 / G)); k0 < n; k0 += ngrp) {   // wave-uniform trip count
        const int64_t k = k0 + (grp % (64 / G));
        if (k >= n) continue;   // group-uniform; no cross-group shuffles below
        const int64_t t = list[k];
        const int64_t b = inc_off[t], e = inc_off[t + 1];
        const bool ev = bit(ever, t);
        const typename V::T old = ev ? V::ld(vis + t * W + sub * WPL) : V::zero();
        typename V::T acc = V::zero();
        for (int64_t i0 = b; i0 < e; i0 += G) {   // group-uniform
            const int64_t q = i0 + sub;
            int32_t myL = q < e ? inc_row[q] : -1;
            if (myL >= 0 && want_type >= 0 && inc_type[q] != want_type) myL = -1;
            int64_t bme = 0;
            int nme = 0;
            if (myL >= 0) {
                bme = tgt_off[myL];
                nme = (int)(tgt_off[myL + 1] - bme);
                ++n_ent;
                n_pins += (u64)nme;
            }
            int32_t v[G];
            int nn[G];
            int64_t bb[G];
#pragma unroll
            for (int j = 0; j < G; ++j) {
                bb[j] = __shfl(bme, base + j);
                nn[j] = __shfl(nme, base + j);
                v[j] = sub < nn[j] ? tgt_idx[bb[j] + sub] : -1;
            }
            unsigned pa = 0;
#pragma unroll
            for (int j = 0; j < G; ++j)
                if (v[j] >= 0 && bit(fa, v[j])) pa |= 1u << j;
#pragma unroll
            for (int j = 0; j < G; ++j) {
                const unsigned ga = (unsigned)((__ballot((pa >> j) & 1u) >> base) & gmask);
                if (ga) {   // group-uniform
                    typename V::T r[G];
#pragma unroll
                    for (int kk = 0; kk < G; ++kk) {
                        const int32_t vk = __shfl(v[j], base + kk);
                        r[kk] = ((ga >> kk) & 1u) ? V::ld(lvl + (int64_t)vk * W + sub * WPL) : V::zero();
                    }
#pragma unroll
                    for (int kk = 0; kk < G; ++kk) acc |= r[kk];
                    n_rows += __popc(ga);
                }
                if (nn[j] > G) {   // a link longer than G (rare): the rest of its targets
                    for (int64_t p = bb[j] + G; p < bb[j] + nn[j]; p += G) {
                        const int64_t qq = p + sub;
                        const int32_t myv = qq < bb[j] + nn[j] ? tgt_idx[qq] : -1;
                        const unsigned g2 = (unsigned)((__ballot(myv >= 0 && bit(fa, myv)) >> base) & gmask);
                        typename V::T r[G];
#pragma unroll
                        for (int kk = 0; kk < G; ++kk) {
                            const int32_t vk = __shfl(myv, base + kk);
                            r[kk] = ((g2 >> kk) & 1u) ? V::ld(lvl + (int64_t)vk * W + sub * WPL) : V::zero();
                        }
#pragma unroll
                        for (int kk = 0; kk < G; ++kk) acc |= r[kk];
                        n_rows += __popc(g2);
                    }
                }
            }
            if (early && i0 + G < e && group_all<G>(V::eq(acc | old, FULL))) break;
        }
        const typename V::T nw = acc & ~old;
        if (group_any<G>(V::nz(nw))) {
            V::st(lvl_next + t * W + sub * WPL, nw);
            V::st(vis + t * W + sub * WPL, old | nw);
            const bool becomes_full = group_all<G>(V::eq(old | nw, FULL));
            if (sub == 0) {
                set_bit(fa_next, t);
                if (!ev) set_bit(ever, t);
                if (becomes_full) set_bit(full, t);
                ++n_new;
                n_full += becomes_full;
                const u64 dg = (u64)(e - b);
                n_newdeg += dg;
                if (!becomes_full) n_newdeg_nf += dg;
            }
        }
        if (sub == 0) {
            ++n_cand;
            n_vis += ev;
        }
    }
    if (sub != 0) n_rows = 0;   // n_ent / n_pins: each lane counted its own entry
    wave_add_sh(ctr + cActiveLinks, n_ent);
    wave_add_sh(ctr + cActivePins, n_pins);
    wave_add_sh(ctr + cIncLight, n_ent);
    wave_add_sh(ctr + cCand, n_cand);
    wave_add_sh(ctr + cNewFull, n_full);
    wave_add_sh(ctr + cVisLight, n_vis);
    wave_add_sh(ctr + cNewLight, n_new);
    wave_add_sh(ctr + cNewAtoms, n_new);
    wave_add_sh(ctr + cNewDeg, n_newdeg);
    wave_add_sh(ctr + cNewDegNF, n_newdeg_nf);
    wave_add_sh(ctr + cNfRows, n_rows);
}

// ---------------------------------------------------------------------------------------------
// Frontier-code pull (round 6; symmetric-mode dense levels over a SMALL frontier, HGX_OPT_BFS_FLAGS
// bit 17).  Config 2's level 1 expands 235K frontier atoms whose incidence covers nearly every link:
// the gather wrote a 128-byte lf row for each of the 40M links and the pull read one such row at
// random per incidence entry (200M x 128 B from a 5 GB table: 33 GB of the level's traffic).  Here
// the pull reads, per incidence entry (t, L) in entry order, a 32-byte record of L's targets
// (hgx_fc_rec, built once per snapshot), probes their frontier bits and ORs the frontier rows of
// the targets into t's accumulator:
//   next(t) = OR_{L in inc(t)} OR_{u in L, u in F_d} lvl_d[u]  minus vis[t]
// (t's own row is a subset of vis[t]).  Most frontier rows are sparse (~1.2 source bits), so each
// becomes a 64-bit CODE of up to kFcIds 10-bit source ids (hgx_fc_codes) in a compact array indexed
// through a per-word prefix of the frontier bitmap; codes and prefixes stay in L2, the records stream.
// The few rows with more bits (config 2 level 1: 912 atoms, but half of the (entry, frontier target)
// pairs -- they are the hubs) get a DENSE SLOT: an entry sets the slot's bit in its atom's dense mask
// (one LDS atomic, as a source id), and the atom ORs the dense rows of its mask once, at the end.  Past
// kFcDenseCap dense rows a code names its atom and the pair ORs the whole row (slow, exact).
// ---------------------------------------------------------------------------------------------
constexpr int kFc = 1 << 17;            // HGX_OPT_BFS_FLAGS bit 17: frontier-code pull levels
constexpr int kFcIds = 6;               // source ids per code (6 x 10 bits + a 3-bit count)
constexpr u64 kFcDense = 1ull << 63;    // code flag: more than kFcIds bits; low bits = dense slot
constexpr u64 kFcRow = 1ull << 62;      //   with kFcDense: no slot left; low 32 bits = the atom (row in lvl_d)
constexpr int kFcDenseCap = 1024;       // dense slots per level
constexpr int kFcDW = kFcDenseCap / 64; // dense-mask words per atom
constexpr int kFcTile = 128;            // atoms per workgroup tile of hgx_fc_pull (256 threads)
constexpr int kFcHubs = 2048;           // hub slots: the snapshot's highest-degree atoms, looked up in LDS

// Entry i = (t, L) of the incidence: the targets of link inc_row[i] other than t (t's own row is a subset
// of vis[t]), -1 padded; a target that is one of the snapshot's kFcHubs hubs (hubs[], ascending) is
// stored as -2 - its hub slot, so the pull finds its frontier code in LDS (a hub is a target of a large
// share of the links: config 2's top 2048 atoms hold ~30% of the pins and most frontier hits).  A thread
// per entry (its atom by binary search over inc_off: built once per snapshot).  A link of arity > 8 sets
// *over (the snapshot then has no records and the level keeps gather + pull).
__global__ void __launch_bounds__(256) hgx_fc_rec(int64_t A, int64_t I, const int64_t* __restrict__ inc_off,
                                                  const int32_t* __restrict__ inc_row,
                                                  const int64_t* __restrict__ tgt_off,
                                                  const int32_t* __restrict__ tgt_idx, const int32_t* __restrict__ hubs,
                                                  int32_t n_hubs, int4* __restrict__ rec, unsigned int* __restrict__ over) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < I; i += (int64_t)gridDim.x * blockDim.x) {
        int64_t lo = 0, hi = A;   // inc_off[lo] <= i < inc_off[hi]
        while (hi - lo > 1) {
            const int64_t mid = (lo + hi) >> 1;
            if (inc_off[mid] <= i) lo = mid;
            else hi = mid;
        }
        const int32_t self = (int32_t)lo;
        const int32_t L = inc_row[i];
        const int64_t b = tgt_off[L];
        const int64_t n = tgt_off[L + 1] - b;
        if (n > 8) atomicOr(over, 1u);
        int32_t t[8];
        int m = 0;
        for (int q = 0; q < 8 && q < n; ++q) {
            const int32_t u = tgt_idx[b + q];
            if (u == self) continue;
            int a = 0, z = n_hubs;   // hubs[a] <= u < hubs[z]
            while (z - a > 1) {
                const int mid = (a + z) >> 1;
                if (hubs[mid] <= u) a = mid;
                else z = mid;
            }
            t[m++] = (n_hubs > 0 && hubs[a] == u) ? -2 - a : u;
        }
        for (; m < 8; ++m) t[m] = -1;
        rec[2 * i] = make_int4(t[0], t[1], t[2], t[3]);
        rec[2 * i + 1] = make_int4(t[4], t[5], t[6], t[7]);
    }
}

// The frontier code of every hub slot this level (0: the hub is not on the frontier).
__global__ void __launch_bounds__(256) hgx_fc_hubs(int32_t n_hubs, const int32_t* __restrict__ hubs,
                                                   const u64x2* __restrict__ fw, const u64* __restrict__ fcode,
                                                   u64* __restrict__ hubtab) {
    for (int h = blockIdx.x * blockDim.x + threadIdx.x; h < n_hubs; h += gridDim.x * blockDim.x) {
        const int32_t u = hubs[h];
        const u64x2 f = fw[u >> 6];
        const bool on = (f.x >> (u & 63)) & 1ull;
        hubtab[h] = on ? fcode[f.y + __popcll(f.x & ((1ull << (u & 63)) - 1ull))] : 0ull;
    }
}

// degrees of n atoms (the hub choice)
__global__ void __launch_bounds__(256) hgx_fc_deg(int64_t n, const int32_t* __restrict__ atoms,
                                                  const int64_t* __restrict__ inc_off, int64_t* __restrict__ deg) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x)
        deg[k] = inc_off[atoms[k] + 1] - inc_off[atoms[k]];
}

// fw[w] = (fa[w], code slot of the first frontier atom of word w): one 16-byte load answers both "is
// v on the frontier" and "where is its code" (slot = fw[w].y + popcount(fa[w] below bit v & 63)).  Slots
// are dense, assigned a block of 256 words at a time with one atomic (not in atom order).
__global__ void __launch_bounds__(256) hgx_fc_slots(int64_t nwords, const u64* __restrict__ fa,
                                                    u64x2* __restrict__ fw, u64* __restrict__ n_slots) {
    __shared__ int wsum[4];
    __shared__ u64 sbase;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int64_t w0 = (int64_t)blockIdx.x * 256; w0 < nwords; w0 += (int64_t)gridDim.x * 256) {   // block-uniform
        const int64_t w = w0 + threadIdx.x;
        const u64 x = w < nwords ? fa[w] : 0ull;
        const int c = __popcll(x);
        int incl = c;
        for (int off = 1; off < 64; off <<= 1) {
            const int y = __shfl_up(incl, off);
            if (lane >= off) incl += y;
        }
        if (lane == 63) wsum[wv] = incl;
        __syncthreads();
        int before = 0, total = 0;
        for (int k = 0; k < 4; ++k) {
            before += k < wv ? wsum[k] : 0;
            total += wsum[k];
        }
        if (threadIdx.x == 0) sbase = total ? atomicAdd(n_slots, (u64)total) : 0ull;
        __syncthreads();
        if (w < nwords) fw[w] = u64x2{x, sbase + (u64)(before + incl - c)};
        __syncthreads();   // wsum / sbase are rewritten by the next chunk
    }
}

// The code of every frontier atom (a thread per atom; only frontier atoms load their row).  Dense rows
// are copied to drow[slot] (slots from one counter; kFcDenseCap of them).
template <int W>
__global__ void __launch_bounds__(256) hgx_fc_codes(int64_t A, const u64x2* __restrict__ fw,
                                                    const u64* __restrict__ lvl, u64* __restrict__ fcode, int64_t cap,
                                                    u64* __restrict__ drow, unsigned int* __restrict__ n_dense,
                                                    u64* __restrict__ ctr) {
    u64 n_dn = 0;
    for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < A; v += (int64_t)gridDim.x * blockDim.x) {
        const u64x2 f = fw[v >> 6];
        const int b = (int)(v & 63);
        if (!((f.x >> b) & 1ull)) continue;
        const int64_t slot = (int64_t)f.y + __popcll(f.x & ((1ull << b) - 1ull));
        if (slot >= cap) continue;   // never (cap = the frontier size); guards the store
        u64 r[W];
#pragma unroll
        for (int k = 0; k < W; ++k) r[k] = lvl[v * W + k];
        int cnt = 0;
#pragma unroll
        for (int k = 0; k < W; ++k) cnt += __popcll(r[k]);
        u64 code;
        if (cnt > kFcIds) {
            const unsigned ds = atomicAdd(n_dense, 1u);
            if (ds < (unsigned)kFcDenseCap) {
                code = kFcDense | (u64)ds;
#pragma unroll
                for (int k = 0; k < W; ++k) drow[(int64_t)ds * W + k] = r[k];
            } else {
                code = kFcDense | kFcRow | (u64)v;
            }
            ++n_dn;
        } else {
            code = (u64)cnt << 60;
            int m = 0;
#pragma unroll
            for (int k = 0; k < W; ++k) {
                u64 x = r[k];
                while (x) {
                    code |= (u64)(k * 64 + __ffsll((long long)x) - 1) << (10 * m);
                    ++m;
                    x &= x - 1ull;
                }
            }
        }
        fcode[slot] = code;
    }
    wave_add_sh(ctr + cCand, n_dn);   // (the push levels' counter slot: frontier rows coded dense)
}

// The frontier contribution of one incidence entry's record: src(word, bits) for every source id of
// every sparse frontier target, dense(slot) for every dense one, row(atom) past the dense slots.
// Returns the frontier targets seen (a dependent chain of three loads: record, fw words, codes).
template <class FS, class FD, class FR>
__device__ __forceinline__ int fc_entry(const int4* __restrict__ rec, int64_t i, const u64x2* __restrict__ fw,
                                        const u64* __restrict__ fcode, const u64* hubtab, FS src, FD dense, FR row) {
    const int4 r0 = rec[2 * i], r1 = rec[2 * i + 1];
    const int32_t t[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
    u64x2 f[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) f[q] = t[q] >= 0 ? fw[t[q] >> 6] : u64x2{0ull, 0ull};
    u64 code[8];
    unsigned hit = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        code[q] = t[q] <= -2 ? hubtab[-2 - t[q]] : 0ull;   // hub slot: its code from LDS (0 = not on the frontier)
        if (t[q] >= 0 && ((f[q].x >> (t[q] & 63)) & 1ull)) hit |= 1u << q;
    }
    unsigned hhit = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q)
        if (t[q] <= -2 && code[q] != 0ull) hhit |= 1u << q;
    if (!(hit | hhit)) return 0;
#pragma unroll
    for (int q = 0; q < 8; ++q)
        if ((hit >> q) & 1u) code[q] = fcode[f[q].y + __popcll(f[q].x & ((1ull << (t[q] & 63)) - 1ull))];
    hit |= hhit;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        if (!((hit >> q) & 1u)) continue;
        const u64 c = code[q];
        if (c & kFcDense) {
            if (c & kFcRow) row((int64_t)(c & 0xffffffffull));
            else dense((int)(c & 0xffffull));
        } else {
            const int n = (int)((c >> 60) & 7ull);
            for (int m = 0; m < n; ++m) {
                const int s = (int)((c >> (10 * m)) & 1023ull);
                src(s >> 6, 1ull << (s & 63));
            }
        }
    }
    return __popc(hit);
}

// OR of the dense rows named by a dense mask into a G-lane group's share of a row (lane sub holds words
// sub*WPL ..): dm = the kFcDW mask words (LDS, read by every lane of the group).
template <int W>
__device__ __forceinline__ typename Vec<Lay<W>::WPL>::T fc_dense_or(const u64* dm, const u64* __restrict__ drow, int sub,
                                                                     typename Vec<Lay<W>::WPL>::T a) {
    constexpr int WPL = Lay<W>::WPL;
    typedef Vec<WPL> V;
    for (int w = 0; w < kFcDW; ++w) {
        u64 x = dm[w];
        while (x) {
            const int ds = w * 64 + __ffsll((long long)x) - 1;
            x &= x - 1ull;
            a |= V::ld(drow + (int64_t)ds * W + sub * WPL);
        }
    }
    return a;
}

// Light atoms (degree <= kHeavyDegree, not yet visited by every traversal): a workgroup takes a tile
// of kFcTile consecutive atoms, spreads the tile's incidence entries flat over its 256 threads (an
// entry's atom by binary search over the tile's degree prefix) and ORs the source bits into the
// atoms' LDS rows (dense frontier targets: a bit of the atom's LDS dense mask); then a G-lane group per
// atom adds the dense rows and applies new = acc & ~vis[t] as hgx_atom_pull2 does.  The tile's
// fa_next / ever / full words belong to the workgroup (plain stores; the hub finalise that follows sets
// heavy atoms' bits with atomics).
template <int W>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8))) hgx_fc_pull(int64_t A, const int64_t* __restrict__ inc_off,
                                                   const int4* __restrict__ rec, const int32_t* __restrict__ inc_type,
                                                   int32_t want_type, const u64x2* __restrict__ fw,
                                                   const u64* __restrict__ fcode, const u64* __restrict__ drow,
                                                   const u64* __restrict__ hubtab_g, int32_t n_hubs,
                                                   const u64* __restrict__ lvl, u64* __restrict__ vis,
                                                   u64* __restrict__ ever, u64* __restrict__ full,
                                                   u64* __restrict__ lvl_next, u64* __restrict__ fa_next,
                                                   u64* __restrict__ ctr, FullMask fm, int flags) {
    constexpr int WPL = Lay<W>::WPL, G = Lay<W>::G, T = kFcTile, NW = T / 64;
    static_assert(G >= 4, "fc pull needs G >= 4");
    static_assert(T <= 256 && T % 64 == 0, "tile");
    typedef Vec<WPL> V;
    __shared__ u64 acc[T * W];
    __shared__ u64 dmask[T * kFcDW];
    __shared__ u64 hubtab[kFcHubs];
    __shared__ int64_t sbeg[T];
    __shared__ int32_t spre[T + 1];
    __shared__ int32_t wsum[4];
    __shared__ u64 snew[NW], sfull[NW];
    const bool skip_full = flags & 4;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int sub = tid & (G - 1), gi = tid / G;
    const typename V::T FULL = full_part<W>(fm, sub);
    for (int h = tid; h < n_hubs; h += 256) hubtab[h] = hubtab_g[h];   // (the tile loop's barriers order it)
    u64 n_ent = 0, n_front = 0, n_rows = 0, n_vis = 0, n_newdeg = 0, n_newdeg_nf = 0, n_new = 0, n_full = 0;
    for (int64_t tile = blockIdx.x; tile * T < A; tile += gridDim.x) {   // block-uniform
        const int64_t v = tile * T + tid;
        int64_t b = 0;
        int d = 0;
        if (tid < T && v < A && !(skip_full && bit(full, v))) {
            b = inc_off[v];
            const int64_t dd = inc_off[v + 1] - b;
            d = (dd > 0 && dd <= kHeavyDegree) ? (int)dd : 0;
        }
        int incl = d;
        for (int off = 1; off < 64; off <<= 1) {
            const int y = __shfl_up(incl, off);
            if (lane >= off) incl += y;
        }
        if (lane == 63) wsum[wv] = incl;
        __syncthreads();
        int before = 0, total = 0;
        for (int k = 0; k < 4; ++k) {
            before += k < wv ? wsum[k] : 0;
            total += wsum[k];
        }
        if (total == 0) {   // block-uniform: no light entries in the tile (e.g. link atoms without incidence)
            if (tid < NW && (tile * NW + tid) * 64 < A) fa_next[tile * NW + tid] = 0ull;
            __syncthreads();   // wsum is rewritten by the next tile
            continue;
        }
        for (int k = tid; k < T * W; k += 256) acc[k] = 0ull;
        for (int k = tid; k < T * kFcDW; k += 256) dmask[k] = 0ull;
        if (tid < NW) {
            snew[tid] = 0ull;
            sfull[tid] = 0ull;
        }
        if (tid < T) {
            sbeg[tid] = b;
            spre[tid] = before + incl - d;
            if (tid == T - 1) spre[T] = before + incl;
        }
        __syncthreads();
        for (int j = tid; j < total; j += 256) {
            int lo = 0, hi = T;   // spre[lo] <= j < spre[hi]: the entry's atom is lo (its degree is > 0)
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if (spre[mid] <= j) lo = mid;
                else hi = mid;
            }
            const int64_t i = sbeg[lo] + (j - spre[lo]);
            if (want_type >= 0 && inc_type[i] != want_type) continue;
            ++n_ent;
            u64* arow = acc + lo * W;
            u64* drm = dmask + lo * kFcDW;
            n_front += (u64)fc_entry(
                rec, i, fw, fcode, hubtab, [&](int k, u64 x) { atomicOr(arow + k, x); },
                [&](int ds) { atomicOr(drm + (ds >> 6), 1ull << (ds & 63)); },
                [&](int64_t u) {
                    ++n_rows;
#pragma unroll 1
                    for (int k = 0; k < W; ++k) {
                        const u64 x = lvl[u * W + k];
                        if (x) atomicOr(arow + k, x);
                    }
                });
        }
        __syncthreads();
        for (int a0 = 0; a0 < T; a0 += 256 / G) {   // block-uniform; a G-lane group per atom
            const int k = a0 + gi;
            const int64_t t = tile * T + k;
            const int dk = k < T ? spre[k + 1] - spre[k] : 0;
            bool isnew = false, becomes_full = false;
            if (dk > 0) {   // group-uniform
                const typename V::T a = fc_dense_or<W>(dmask + k * kFcDW, drow, sub, V::ld(acc + k * W + sub * WPL));
                if (group_any<G>(V::nz(a))) {
                    const bool ev = bit(ever, t);
                    const typename V::T old = ev ? V::ld(vis + t * W + sub * WPL) : V::zero();
                    const typename V::T nw = a & ~old;
                    if (sub == 0 && ev) ++n_vis;
                    if (group_any<G>(V::nz(nw))) {
                        V::st(lvl_next + t * W + sub * WPL, nw);
                        V::st(vis + t * W + sub * WPL, old | nw);
                        isnew = true;
                        becomes_full = group_all<G>(V::eq(old | nw, FULL));
                    }
                }
            }
            if (sub == 0 && isnew) {
                atomicOr(&snew[k >> 6], 1ull << (k & 63));
                if (becomes_full) atomicOr(&sfull[k >> 6], 1ull << (k & 63));
                n_newdeg += (u64)dk;
                if (!becomes_full) n_newdeg_nf += (u64)dk;
            }
        }
        __syncthreads();
        if (tid < NW) {
            const int64_t w = tile * NW + tid;
            if (w * 64 < A) {
                const u64 nw = snew[tid], fw_ = sfull[tid];
                fa_next[w] = nw;
                if (nw) ever[w] |= nw;
                if (fw_) full[w] |= fw_;
                n_new += (u64)__popcll(nw);
                n_full += (u64)__popcll(fw_);
            }
        }
        __syncthreads();   // the LDS rows and prefixes are rewritten by the next tile
    }
    wave_add_sh(ctr + cIncLight, n_ent);
    wave_add_sh(ctr + cActivePins, n_front);
    wave_add_sh(ctr + cNfRows, n_rows);
    wave_add_sh(ctr + cVisLight, n_vis);
    wave_add_sh(ctr + cNewLight, n_new);
    wave_add_sh(ctr + cNewAtoms, n_new);
    wave_add_sh(ctr + cNewFull, n_full);
    wave_add_sh(ctr + cNewDeg, n_newdeg);
    wave_add_sh(ctr + cNewDegNF, n_newdeg_nf);
}

// Heavy atoms: a workgroup per kChunkEntries-entry chunk of a hub; source bits and dense-slot bits go to
// the workgroup's LDS row and mask (every entry belongs to the same hub), which are reduced once per
// chunk into hubacc (then hgx_hub_finalize as in the dense levels).  (Per-lane register rows with
// select chains instead of the LDS atomics measured 10.9 against 3.2 ms on config 2's level 1.)  A chunk
// whose hub is already covered -- by the accumulator the hub's earlier chunks filled this level,
// together with vis -- exits before streaming its entries.
template <int W>
__global__ void __launch_bounds__(256) hgx_fc_pull_heavy(const HeavyChunk* __restrict__ chunks,
                                                         const int4* __restrict__ rec,
                                                         const int32_t* __restrict__ inc_type, int32_t want_type,
                                                         const u64x2* __restrict__ fw, const u64* __restrict__ fcode,
                                                         const u64* __restrict__ drow, const u64* __restrict__ hubtab_g,
                                                         int32_t n_hubs, const u64* __restrict__ lvl,
                                                         const u64* __restrict__ vis, const u64* __restrict__ ever,
                                                         const u64* __restrict__ full, u64* __restrict__ hubacc,
                                                         u64* __restrict__ ctr, FullMask fm, int flags) {
    __shared__ u64 acc[W];
    __shared__ u64 dmask[kFcDW];
    __shared__ u64 hubtab[kFcHubs];
    __shared__ int covered;
    const HeavyChunk c = chunks[blockIdx.x];
    if ((flags & 4) && bit(full, c.atom)) return;   // block-uniform
    const int tid = threadIdx.x;
    if (tid < W) acc[tid] = 0ull;
    if (tid < kFcDW) dmask[tid] = 0ull;
    if (tid == 0) covered = 1;
    for (int h = tid; h < n_hubs; h += 256) hubtab[h] = hubtab_g[h];
    __syncthreads();
    if (tid < W) {   // word tid of the hub's row: covered by this level's accumulator + vis?
        const bool ev = bit(ever, c.atom);
        const u64 h = __hip_atomic_load(hubacc + (int64_t)c.slot * W + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const u64 o = ev ? vis[(int64_t)c.atom * W + tid] : 0ull;
        if (((h | o) & fm.w[tid]) != fm.w[tid]) covered = 0;
    }
    __syncthreads();
    if (covered) return;   // block-uniform
    u64 n_ent = 0, n_front = 0, n_rows = 0;
    for (int64_t i = c.beg + tid; i < c.end; i += 256) {
        if (want_type >= 0 && inc_type[i] != want_type) continue;
        ++n_ent;
        n_front += (u64)fc_entry(
            rec, i, fw, fcode, hubtab, [&](int k, u64 x) { atomicOr(acc + k, x); },
            [&](int ds) { atomicOr(dmask + (ds >> 6), 1ull << (ds & 63)); },
            [&](int64_t u) {
                ++n_rows;
#pragma unroll 1
                for (int k = 0; k < W; ++k) {
                    const u64 x = lvl[u * W + k];
                    if (x) atomicOr(acc + k, x);
                }
            });
    }
    __syncthreads();
    // the chunk's row: its source bits + the dense rows of its mask, word k by thread k
    if (tid < W) {
        u64 x = acc[tid];
        for (int w = 0; w < kFcDW; ++w) {
            u64 m = dmask[w];
            while (m) {
                const int ds = w * 64 + __ffsll((long long)m) - 1;
                m &= m - 1ull;
                x |= drow[(int64_t)ds * W + tid];
            }
        }
        if (x) atomicOr(hubacc + (int64_t)c.slot * W + tid, x);
    }
    wave_add_sh(ctr + cIncHeavy, n_ent);
    wave_add_sh(ctr + cActivePins, n_front);
    wave_add_sh(ctr + cNfRows, n_rows);
}

// The seeds' incidence volume (the level-0 direction choice) straight into mapped host memory: one
// block sums the degrees, stores the total, then the sequence number the host spins on (a
// device-to-host copy and a stream synchronisation cost ~40 us before the first level).
__global__ void __launch_bounds__(256) hgx_seed_degree_host(int32_t n, const int32_t* __restrict__ atoms,
                                                            const int64_t* __restrict__ inc_off,
                                                            u64* __restrict__ hout, u64 seq) {
    __shared__ u64 part[4];
    u64 d = 0;
    for (int k = threadIdx.x; k < n; k += 256) d += (u64)(inc_off[atoms[k] + 1] - inc_off[atoms[k]]);
    for (int off = 32; off > 0; off >>= 1) d += __shfl_xor(d, off);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = d;
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_store(hout, part[0] + part[1] + part[2] + part[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __threadfence_system();
        __hip_atomic_store(hout + 1, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// Level 0: seed rows.  rows[i*W ..] is the mask row of unique seed atom atoms[i].
template <int W>
__global__ void hgx_seed(int32_t n, const int32_t* __restrict__ atoms, const u64* __restrict__ rows,
                         u64* __restrict__ lvl0, u64* __restrict__ vis, u64* __restrict__ fa0,
                         u64* __restrict__ ever, u64* __restrict__ full, FullMask fm) {
    int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    int64_t a = atoms[k];
    bool is_full = true;
    for (int w = 0; w < W; ++w) {
        u64 r = rows[(int64_t)k * W + w];
        lvl0[a * W + w] = r;
        vis[a * W + w] = r;
        is_full &= (r == fm.w[w]);
    }
    set_bit(fa0, a);
    set_bit(ever, a);
    if (is_full) set_bit(full, a);
}

// ---------------------------------------------------------------------------------------------
// Result extraction / accounting (not on the timed path)
// ---------------------------------------------------------------------------------------------

// Bit-sliced per-source counts of one level: counts[w*64 + b] += |{v : bit b of lvl[v][w]}|.
// Also traversed += sum_v popcount(lvl[v]) * deg(v) (the hyperedge TEPS numerator).
template <int W>
__global__ void __launch_bounds__(256) hgx_level_count(int64_t A, const u64* __restrict__ fa,
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

// Position of the n-th set bit (n < popcount(x)) of x: binary search over popcounts (6 steps).

// Per-source counts of one level (the result readout of a batch): the count of source w*64 + b =
// |{v : fa(v), bit b of lvl[v][w]}|, reading only the rows of the level's atoms.  A wave takes 64
// bitmap words at a time and visits the nonzero ones; the set bits of a word are spread over the
// lanes W at a time (lane l always holds word l % W of its rows), U = 8 rows per lane in flight at
// once.  A lane adds its 8 words with a carry-save (Harley-Seal) tree -- ones, twos, fours, and the
// eights carried into K vertical planes, stopping once no lane carries -- about 12 VALU ops a word
// instead of a 3K-op ripple per word (the ripple made the kernel ALU-bound at 1.8 TB/s).  The
// planes are folded once per lane; each block stores its 1024 partial counts (no global atomics:
// thousands of blocks adding to the same 1024 words serialised), hgx_count_reduce sums them.  With
// `own` only the atoms of that bitmap count (a partition part's owned atoms).
__device__ __forceinline__ void csa(u64& h, u64& l, u64 a, u64 b, u64 c) {
    const u64 u = a ^ b;
    h = (a & b) | (u & c);
    l = u ^ c;
}

constexpr int kCountBlocks = 2048;

template <int W>
__device__ __forceinline__ void count_rows_body(int64_t A, const u64* __restrict__ fa, const u64* __restrict__ own,
                                                const u64* __restrict__ lvl, uint32_t* __restrict__ partial);

template <int W>
__global__ void __launch_bounds__(256) hgx_count_rows(int64_t A, const u64* __restrict__ fa, const u64* __restrict__ own,
                                                      const u64* __restrict__ lvl, uint32_t* __restrict__ partial) {
    count_rows_body<W>(A, fa, own, lvl, partial);
}

// Every level of one batch in one launch (blockIdx.y = level slot): a traversal of tens of short
// levels (config 5) paid one launch per level for its readout.
template <int W>
__global__ void __launch_bounds__(256) hgx_count_rows_multi(int64_t A, const u64* const* __restrict__ fa_p,
                                                            const u64* __restrict__ own,
                                                            const u64* const* __restrict__ lvl_p,
                                                            const int64_t* __restrict__ poff, int slot0,
                                                            uint32_t* __restrict__ partial) {
    const int sl = slot0 + (int)blockIdx.y;
    if (!fa_p[sl]) return;   // counted by its push finalise
    count_rows_body<W>(A, fa_p[sl], own, lvl_p[sl], partial + poff[sl]);
}

template <int W>
__device__ __forceinline__ void count_rows_body(int64_t A, const u64* __restrict__ fa, const u64* __restrict__ own,
                                                const u64* __restrict__ lvl, uint32_t* __restrict__ partial) {
    // planes of the eights: K = 8 holds < 2^11 rows per lane, flushed into the block's LDS counts before
    // they can overflow (22 planes kept 44 VGPRs live for the whole kernel: 120 VGPRs, 4 waves/SIMD)
    constexpr int K = 8;
    constexpr int R = 64 / W, U = 8;
    __shared__ unsigned int lc[W * 64];
    for (int j = threadIdx.x; j < W * 64; j += 256) lc[j] = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, k = lane / W, wd = lane % W;
    const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    const int64_t nwave = ((int64_t)gridDim.x * blockDim.x) >> 6;
    const int64_t nwords = (A + 63) / 64;
    u64 ones = 0, twos = 0, fours = 0;
    u64 c[K];
#pragma unroll
    for (int q = 0; q < K; ++q) c[q] = 0;
    int since = 0;   // rows per lane added since the last flush (wave-uniform)
    auto flush = [&]() {
        for (int b = 0; b < 64; ++b) {
            unsigned int n = (unsigned int)((ones >> b) & 1ull) | ((unsigned int)((twos >> b) & 1ull) << 1) |
                             ((unsigned int)((fours >> b) & 1ull) << 2);
#pragma unroll
            for (int q = 0; q < K; ++q) n += (unsigned int)((c[q] >> b) & 1ull) << (q + 3);
            if (n) atomicAdd(&lc[wd * 64 + b], n);
        }
        ones = twos = fours = 0;
#pragma unroll
        for (int q = 0; q < K; ++q) c[q] = 0;
        since = 0;
    };
    for (int64_t base = wave * 64; base < nwords; base += nwave * 64) {
        const int64_t wi = base + lane;
        const u64 x = wi < nwords ? (fa[wi] & (own ? own[wi] : ~0ull)) : 0ull;
        u64 m = __ballot(x != 0ull);
        auto add8 = [&](const u64 (&v)[U]) {   // 8 row words into the carry-save planes
            u64 t2a, t2b, t4a, t4b, t8;
            csa(t2a, ones, ones, v[0], v[1]);
            csa(t2b, ones, ones, v[2], v[3]);
            csa(t4a, twos, twos, t2a, t2b);
            csa(t2a, ones, ones, v[4], v[5]);
            csa(t2b, ones, ones, v[6], v[7]);
            csa(t4b, twos, twos, t2a, t2b);
            csa(t8, fours, fours, t4a, t4b);
            u64 carry = t8;
#pragma unroll
            for (int q = 0; q < K; ++q) {
                if (__ballot(carry != 0ull) == 0ull) break;   // wave-uniform
                const u64 tq = c[q] & carry;
                c[q] ^= carry;
                carry = tq;
            }
        };
        while (m) {   // two nonzero words at a time: their row loads in flight together
            const int kw1 = __ffsll((long long)m) - 1;
            m &= m - 1ull;
            const int kw2 = m ? __ffsll((long long)m) - 1 : -1;
            if (m) m &= m - 1ull;
            const u64 xw1 = (u64)__shfl(x, kw1);
            const u64 s2 = (u64)__shfl(x, kw2 < 0 ? 0 : kw2);
            const u64 xw2 = kw2 < 0 ? 0ull : s2;
            const int64_t t1 = (base + kw1) * 64, t2 = (base + (kw2 < 0 ? 0 : kw2)) * 64;
            const int n1 = __popcll(xw1), n2 = __popcll(xw2), nm = n1 > n2 ? n1 : n2;
            for (int r0 = 0; r0 < nm; r0 += R * U) {   // wave-uniform
                u64 v1[U], v2[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int j = r0 + u * R + k;
                    v1[u] = j < n1 ? lvl[(t1 + nth_set_bit(xw1, j)) * W + wd] : 0ull;
                    v2[u] = j < n2 ? lvl[(t2 + nth_set_bit(xw2, j)) * W + wd] : 0ull;
                }
                add8(v1);
                add8(v2);
                since += 2 * U;
                if (since > (8 << K) - 4 * U) flush();   // wave-uniform
            }
        }
    }
    flush();
    __syncthreads();
    for (int j = threadIdx.x; j < W * 64; j += 256) partial[(int64_t)blockIdx.x * (W * 64) + j] = lc[j];
}

// counts[l][j] += the partial counts of level slot l over one range of kReduceSpan blocks (one launch
// for every level of the readout; counts zeroed first): a thread per (slot, source, block range), the
// partials read 8 loads in flight.  One thread per (slot, source) walking all 2048 blocks took ~0.18 ms.
constexpr int kReduceSpan = 128;
__global__ void __launch_bounds__(256) hgx_count_reduce(int nslot, const int32_t* __restrict__ nblk,
                                                        const int32_t* __restrict__ width,
                                                        const uint32_t* const* __restrict__ pp,
                                                        const u64* const* __restrict__ direct,
                                                        u64* __restrict__ counts) {
    constexpr int NR = kCountBlocks / kReduceSpan;
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= (int64_t)nslot * 1024 * NR) return;
    const int r = (int)(i % NR);
    const int64_t sj = i / NR;
    const int sl = (int)(sj / 1024), j = (int)(sj % 1024);
    const int wj = width[sl];
    if (j >= wj) return;
    const uint32_t* p = pp[sl] + j;
    const int b0 = r * kReduceSpan, b1 = min(nblk[sl], b0 + kReduceSpan);
    u64 sum = (r == 0 && direct[sl]) ? direct[sl][j] : 0ull;   // a push level's counts from its finalise
    for (int b = b0; b < b1; b += 8) {
        uint32_t v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = b + u < b1 ? p[(int64_t)(b + u) * wj] : 0u;
#pragma unroll
        for (int u = 0; u < 8; ++u) sum += v[u];
    }
    if (sum) atomicAdd(&counts[(int64_t)sl * 1024 + j], sum);
}

// Compaction of {v : fa(v) && bit s of lvl[v]} in ascending order.  Pass 1 (write = false)
// counts per block; pass 2 writes at the block's exclusive offset.  Each block owns the
// contiguous atom range [blk*span, (blk+1)*span).
__global__ void __launch_bounds__(256) hgx_extract(int64_t A, int64_t span, int W, int s,
                                                   const u64* __restrict__ fa, const u64* __restrict__ own,
                                                   const u64* __restrict__ lvl,
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
        bool hit = v < hi && bit(fa, v) && (!own || bit(own, v)) && ((lvl[v * W + (s >> 6)] >> (s & 63)) & 1ull);
        u64 m = __ballot(hit);
        int before = __popcll(m & ((1ull << lane) - 1ull));
        if (lane == 0) wave_tot[wid] = __popcll(m);
        __syncthreads();
        int64_t wbase = run;
        for (int k = 0; k < wid; ++k) wbase += wave_tot[k];
        if (write && hit) {
            int64_t pos = wbase + before;   // (blk_off may start below 0: a range read from a later position)
            if (pos >= 0 && pos < cap) out[pos] = (int32_t)v;
        }
        __syncthreads();
        if (threadIdx.x == 0) run += wave_tot[0] + wave_tot[1] + wave_tot[2] + wave_tot[3];
        __syncthreads();
    }
    if (!write && threadIdx.x == 0) blk_cnt[blockIdx.x] = run;
}

// SURVEY.md 8(d) push-model quantities of one level, link-parallel:
//   out[0] = |U_d|, out[1] = sum_{v in U_d} deg(v) = sum_L |distinct targets of L in U_d|,
//   out[2] = P_d = sum_{v in U_d} sum_{L in inc v} arity(L) = sum_L arity(L) * |distinct U_d targets|
__global__ void __launch_bounds__(256) hgx_level_survey(int64_t A, int64_t M, const u64* __restrict__ fa,
                                                        const int64_t* __restrict__ tgt_off,
                                                        const int32_t* __restrict__ tgt_idx, u64* __restrict__ out) {
    u64 nu = 0, sd = 0, pd = 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w * 64 < A; w += stride) nu += __popcll(fa[w]);
    for (int64_t L = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; L < M; L += stride) {
        const int64_t b = tgt_off[L], e = tgt_off[L + 1];
        u64 k = 0;
        for (int64_t p = b; p < e; ++p) {
            const int32_t v = tgt_idx[p];
            if (!bit(fa, v)) continue;
            bool dup = false;
            for (int64_t q = b; q < p; ++q) dup |= tgt_idx[q] == v;
            k += !dup;
        }
        sd += k;
        pd += k * (u64)(e - b);
    }
    wave_add(out + 0, nu);
    wave_add(out + 1, sd);
    wave_add(out + 2, pd);
}

__global__ void hgx_depth_probe(int32_t nlev, const u64* const* __restrict__ fa, const u64* const* __restrict__ lvl,
                                int W, int s, int64_t atom, int32_t* __restrict__ out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    int32_t d = -1;
    for (int k = 0; k < nlev && d < 0; ++k)
        if (bit(fa[k], atom) && ((lvl[k][atom * W + (s >> 6)] >> (s & 63)) & 1ull)) d = k;
    *out = d;
}

// ---------------------------------------------------------------------------------------------
// Partitioned BFS (vertex cut): per-level exchange of S-bit rows.
// After the local expansion a part holds, for every local atom with a frontier bit, the news its
// own links produced (lvl_next; vis already ORed).  For a ghost that is a PARTIAL row:
//   reduce    hgx_xr_pack ships ghost rows to their owners; hgx_x_apply<REDUCE> (one launch per
//             source part, an atom appears at most once per source) ORs them in: new = row & ~vis;
//   broadcast hgx_xb_pack ships every owned atom's final row to its other holders; hgx_x_apply
//             overwrites the holder's row (final is a superset of the partial) and ORs vis.
// Records are compressed to the row's nonzero 64-bit words (about half of them at config 4): a
// 16-byte header {local id on the receiver, word mask, payload offset} in the header stream and
// the nonzero words, in word order, at the payload offset of the payload stream.  Both streams are
// segmented by destination part and shipped by one all-to-all each.
// ---------------------------------------------------------------------------------------------

// Slots are reserved per BLOCK: a block walks a contiguous range of tiles twice -- pass 1 loads the
// rows and counts its records and payload words per destination in LDS, one global atomic per
// destination and stream claims the block's ranges (cursors kCurStride words apart, each pair on a
// line of its own), pass 2 loads the rows again and writes the records at LDS-counted offsets.  One
// atomic per wave per destination (7 cursors on one line) serialised to ~25 ms a level at config-4
// scale.
constexpr int kCurStride = 32;   // cursor q: [q * kCurStride] records, [q * kCurStride + 16] words (own lines)
constexpr int kMaxParts = 64;

struct PackLds {
    unsigned int rec[kMaxParts];
    unsigned int wrd[kMaxParts];
    unsigned long long base_r[kMaxParts];
    unsigned long long base_w[kMaxParts];
    unsigned long long slot[kMaxParts];   // pass 2: records | words << 32 handed out so far
};

// Word-nonzero mask of the row of this lane's G-lane group (bit w = row word w != 0).  Wave-uniform.
template <int W>
__device__ __forceinline__ uint32_t group_mask(typename Vec<Lay<W>::WPL>::T row) {
    constexpr int WPL = Lay<W>::WPL, G = Lay<W>::G;
    const int gbase = (threadIdx.x & 63) & ~(G - 1);
    if constexpr (WPL == 1) {
        return (uint32_t)((__ballot(row != 0ull) >> gbase) & ((1ull << G) - 1ull));
    } else {
        const uint32_t m0 = (uint32_t)((__ballot(row.x != 0ull) >> gbase) & ((1ull << G) - 1ull));
        const uint32_t m1 = (uint32_t)((__ballot(row.y != 0ull) >> gbase) & ((1ull << G) - 1ull));
        uint32_t m = 0;
#pragma unroll
        for (int k = 0; k < G; ++k) m |= (((m0 >> k) & 1u) << (2 * k)) | (((m1 >> k) & 1u) << (2 * k + 1));
        return m;
    }
}

// Write one record: the group's leader the header, every lane its words (dense: all W words, mask
// all ones -- a block whose rows are mostly nonzero skips the counting pass's row loads).
template <int W>
__device__ __forceinline__ void put_record(u64* __restrict__ hdr, u64* __restrict__ pay, int64_t slot, int64_t woff,
                                           int32_t lid, uint32_t mask, typename Vec<Lay<W>::WPL>::T row, bool dense) {
    constexpr int WPL = Lay<W>::WPL, G = Lay<W>::G;
    typedef Vec<WPL> V;
    const int sub = (threadIdx.x & 63) & (G - 1);
    if (sub == 0)
        *reinterpret_cast<u64x2*>(hdr + 2 * slot) = u64x2{(u64)(uint32_t)lid | ((u64)mask << 32), (u64)woff};
    if (dense) {
        V::st(pay + woff + sub * WPL, row);
    } else if constexpr (WPL == 1) {
        if (row != 0ull) pay[woff + __popc(mask & ((1u << sub) - 1u))] = row;
    } else {
        const int w0 = sub * 2;
        const int64_t p0 = woff + __popc(mask & ((1u << w0) - 1u));
        if (row.x != 0ull) pay[p0] = row.x;
        if (row.y != 0ull) pay[p0 + (row.x != 0ull)] = row.y;
    }
}

constexpr uint32_t full_word_mask(int W) { return W >= 32 ? 0xffffffffu : ((1u << W) - 1u); }

// A block packs dense (all W words per record, no row loads while counting) when the rows of its
// sample -- the first tile of each of its waves -- have more than 70% nonzero words.  Wave-uniform.
__device__ __forceinline__ void sample_add(unsigned int* samp, bool leader, uint32_t mask) {
    if (leader) {
        atomicAdd(&samp[0], (unsigned int)__popc(mask));
        atomicAdd(&samp[1], 1u);
    }
}
__device__ __forceinline__ bool sample_dense(const unsigned int* samp, int W) {
    return samp[1] > 0 && (u64)samp[0] * 10ull > (u64)samp[1] * (u64)W * 7ull;
}

// The tiles of block b: [b * per, min((b + 1) * per, ntiles)).
__device__ __forceinline__ void block_tiles(int64_t ntiles, int64_t& lo, int64_t& hi) {
    const int64_t per = (ntiles + gridDim.x - 1) / gridDim.x;
    lo = (int64_t)blockIdx.x * per;
    hi = lo + per < ntiles ? lo + per : ntiles;
}

__device__ __forceinline__ void pack_reserve(PackLds& sh, u64* __restrict__ cursor, int NP) {
    for (int d = threadIdx.x; d < NP; d += 256) {
        const unsigned int r = sh.rec[d], w = sh.wrd[d];
        sh.base_r[d] = r ? atomicAdd(&cursor[d * kCurStride], (u64)r) : 0ull;
        sh.base_w[d] = w ? atomicAdd(&cursor[d * kCurStride + 16], (u64)w) : 0ull;
        sh.slot[d] = 0ull;
    }
}

// The tiles of this wave in its block's range (lo + wv, lo + wv + 4, ...) whose word of fa & own
// (OWNED) or fa & ~own is nonzero: 64 tile words per coalesced load, body(tile, word) runs
// wave-uniformly on the nonzero ones.  first_only stops after the first (the density sample).
template <bool OWNED, class F>
__device__ __forceinline__ void for_wave_tiles(int64_t lo, int64_t hi, const u64* __restrict__ fa,
                                               const u64* __restrict__ own, bool first_only, F body) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int64_t b = lo + wv; b < hi; b += 4 * 64) {
        const int64_t tile = b + 4 * (int64_t)lane;
        u64 x = 0;
        if (tile < hi) {
            const u64 f = fa[tile], o = own[tile];
            x = OWNED ? (f & o) : (f & ~o);
        }
        u64 m = __ballot(x != 0ull);
        while (m) {
            const int k = __ffsll((long long)m) - 1;
            m &= m - 1ull;
            body(b + 4 * (int64_t)k, (u64)__shfl(x, k));
            if (first_only) return;
        }
    }
}

// Reduce pack: one record per ghost with news, to its owner.  seg_h / seg_p: the destination
// segments' starts in the header (records) and payload (words) streams.  A wave loads U rows per
// group at once (the row loads are the latency chain of the kernel).
template <int W>
__global__ void __launch_bounds__(256) hgx_xr_pack(int64_t A, const u64* __restrict__ fa_next,
                                                   const u64* __restrict__ own_bm, const int32_t* __restrict__ xo_part,
                                                   const int32_t* __restrict__ xo_lid, const u64* __restrict__ lvl_next,
                                                   u64* __restrict__ cursor, const int64_t* __restrict__ seg_h,
                                                   const int64_t* __restrict__ seg_p, u64* __restrict__ hdr,
                                                   u64* __restrict__ pay, u64* __restrict__ nzw, int NP) {
    constexpr int WPL = Lay<W>::WPL, G = Lay<W>::G, PER = 64 / G, U = 4;
    constexpr uint32_t FULLM = full_word_mask(W);
    typedef Vec<WPL> V;
    __shared__ PackLds sh;
    __shared__ unsigned int samp[2];
    const int lane = threadIdx.x & 63, g = lane / G, sub = lane & (G - 1), gbase = lane & ~(G - 1);
    int64_t lo, hi;
    block_tiles((A + 63) / 64, lo, hi);
    for (int d = threadIdx.x; d < NP; d += 256) sh.rec[d] = sh.wrd[d] = 0;
    if (threadIdx.x < 2) samp[threadIdx.x] = 0;
    __syncthreads();
    for (int pass = -1; pass < 2; ++pass) {   // density sample, counts, records
        const bool dense = pass >= 0 && sample_dense(samp, W);
        const bool load = !(pass == 0 && dense);
        u64 nz = 0;
        for_wave_tiles<false>(lo, hi, fa_next, own_bm, pass < 0, [&](int64_t tile, u64 gh) {
            const int n = __popcll(gh);
            for (int r0 = 0; r0 < n; r0 += PER * U) {   // wave-uniform
                typename V::T row[U];
                int64_t t[U];
                int q[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int j = r0 + u * PER + g;
                    t[u] = tile * 64 + (j < n ? nth_set_bit(gh, j) : 0);
                    row[u] = (load && j < n) ? V::ld(lvl_next + t[u] * W + sub * WPL) : V::zero();
                    q[u] = (pass >= 0 && j < n) ? xo_part[t[u]] : 0;
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    if (r0 + u * PER < n) {   // wave-uniform
                        const bool ok = r0 + u * PER + g < n;
                        const uint32_t nzm = group_mask<W>(row[u]);
                        const uint32_t mask = dense ? FULLM : nzm;
                        if (pass < 0) {
                            sample_add(samp, ok && sub == 0, nzm);
                        } else if (pass == 0) {
                            if (ok && sub == 0) {
                                atomicAdd(&sh.rec[q[u]], 1u);
                                atomicAdd(&sh.wrd[q[u]], (unsigned int)__popc(mask));
                            }
                        } else {
                            u64 pk = 0;
                            if (ok && sub == 0) pk = atomicAdd(&sh.slot[q[u]], 1ull | ((u64)__popc(mask) << 32));
                            pk = __shfl(pk, gbase);   // wave-uniform point
                            if (ok) {
                                const int64_t slot = seg_h[q[u]] + (int64_t)sh.base_r[q[u]] + (int64_t)(pk & 0xffffffffull);
                                const int64_t woff = (int64_t)sh.base_w[q[u]] + (int64_t)(pk >> 32);
                                put_record<W>(hdr, pay + seg_p[q[u]], slot, woff, xo_lid[t[u]], mask, row[u], dense);
                                if (sub == 0) nz += (u64)__popc(nzm);
                            }
                        }
                    }
                }
            }
        });
        __syncthreads();
        if (pass == 0) {
            pack_reserve(sh, cursor, NP);
            __syncthreads();
        } else if (pass == 1) {
            block_add_sh(nzw, 2, nz);
        }
    }
}

// Broadcast pack: one record per (owned atom with news, other holder).
template <int W>
__global__ void __launch_bounds__(256) hgx_xb_pack(int64_t A, const u64* __restrict__ fa_next,
                                                   const u64* __restrict__ own_bm, const int64_t* __restrict__ bc_off,
                                                   const int32_t* __restrict__ bc_part, const int32_t* __restrict__ bc_lid,
                                                   const u64* __restrict__ lvl_next, u64* __restrict__ cursor,
                                                   const int64_t* __restrict__ seg_h, const int64_t* __restrict__ seg_p,
                                                   u64* __restrict__ hdr, u64* __restrict__ pay, u64* __restrict__ nzw,
                                                   int NP) {
    constexpr int WPL = Lay<W>::WPL, G = Lay<W>::G, PER = 64 / G, U = 2;
    constexpr uint32_t FULLM = full_word_mask(W);
    typedef Vec<WPL> V;
    __shared__ PackLds sh;
    __shared__ unsigned int samp[2];
    const int lane = threadIdx.x & 63, g = lane / G, sub = lane & (G - 1), gbase = lane & ~(G - 1);
    int64_t lo, hi;
    block_tiles((A + 63) / 64, lo, hi);
    for (int d = threadIdx.x; d < NP; d += 256) sh.rec[d] = sh.wrd[d] = 0;
    if (threadIdx.x < 2) samp[threadIdx.x] = 0;
    __syncthreads();
    for (int pass = -1; pass < 2; ++pass) {   // density sample, counts, records
        const bool dense = pass >= 0 && sample_dense(samp, W);
        const bool load = !(pass == 0 && dense);
        u64 nz = 0;
        bool sampled = false;
        for_wave_tiles<true>(lo, hi, fa_next, own_bm, false, [&](int64_t tile, u64 ow) {
            if (pass < 0 && sampled) return;
            const int64_t t = tile * 64 + lane;
            int64_t b = 0;
            int n = 0;
            if ((ow >> lane) & 1ull) {
                b = bc_off[t];
                n = (int)(bc_off[t + 1] - b);
            }
            const u64 hits = __ballot(n > 0);   // owned atoms with news that other parts hold
            const int nh = __popcll(hits);
            if (nh == 0) return;   // wave-uniform
            sampled = true;
            for (int r0 = 0; r0 < nh; r0 += PER * U) {   // wave-uniform
                typename V::T row[U];
                int64_t sb[U];
                int sn[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int j = r0 + u * PER + g;
                    const int bsel = j < nh ? nth_set_bit(hits, j) : 0;
                    // shuffles at wave-uniform points only: a source lane that is inactive during a
                    // ds_bpermute yields garbage, and lane bsel's own group may be past nh
                    sb[u] = __shfl(b, bsel);
                    const int sn_src = __shfl(n, bsel);
                    sn[u] = j < nh ? sn_src : 0;
                    row[u] = (load && sn[u] > 0) ? V::ld(lvl_next + (tile * 64 + bsel) * W + sub * WPL) : V::zero();
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    if (r0 + u * PER < nh) {   // wave-uniform
                        const uint32_t nzm = group_mask<W>(row[u]);
                        const uint32_t mask = dense ? FULLM : nzm;
                        const unsigned int nnz = (unsigned int)__popc(mask);
                        if (pass < 0) {
                            sample_add(samp, sn[u] > 0 && sub == 0, nzm);
                            continue;
                        }
                        if (pass == 1 && sn[u] > 0 && sub == 0) nz += (u64)__popc(nzm);
                        int emax = sn[u];
                        for (int off = 32; off > 0; off >>= 1) emax = max(emax, __shfl_xor(emax, off));
                        // the atom's other holders, G at a time: lane sub of the group loads entry e0 + sub
                        // (independent loads instead of one dependent load per holder)
                        for (int e0 = 0; e0 < emax; e0 += G) {   // wave-uniform
                            const bool mine = e0 + sub < sn[u];
                            const int hq = mine ? bc_part[sb[u] + e0 + sub] : 0;
                            const int32_t hl = mine ? bc_lid[sb[u] + e0 + sub] : 0;
                            if (pass == 0) {
                                if (mine) {
                                    atomicAdd(&sh.rec[hq], 1u);
                                    atomicAdd(&sh.wrd[hq], nnz);
                                }
                                continue;
                            }
                            const int kmax = min(G, emax - e0);
                            for (int k = 0; k < kmax; ++k) {   // wave-uniform: holder e0 + k of each group's atom
                                const int q = __shfl(hq, gbase + k);
                                const int32_t lid = __shfl(hl, gbase + k);
                                const bool has = e0 + k < sn[u];
                                u64 pk = 0;
                                if (has && sub == 0) pk = atomicAdd(&sh.slot[q], 1ull | ((u64)nnz << 32));
                                pk = __shfl(pk, gbase);
                                if (has) {
                                    const int64_t slot = seg_h[q] + (int64_t)sh.base_r[q] + (int64_t)(pk & 0xffffffffull);
                                    const int64_t woff = (int64_t)sh.base_w[q] + (int64_t)(pk >> 32);
                                    put_record<W>(hdr, pay + seg_p[q], slot, woff, lid, mask, row[u], dense);
                                }
                            }
                        }
                    }
                }
            }
        });
        __syncthreads();
        if (pass == 0) {
            pack_reserve(sh, cursor, NP);
            __syncthreads();
        } else if (pass == 1) {
            block_add_sh(nzw, 2, nz);
        }
    }
}

// Broadcast pack of a dense level over the broadcast entries (bc_atom / bc_part / bc_lid, grouped by
// owned atom): one dense record per (owned atom with news, other holder), 64 entries per wave step.
// Slots are ranked inside the wave by ballots -- one LDS atomic per wave and destination, none per
// record -- so a wave's records are contiguous in each destination segment, and every lane group
// writes a record (hgx_xb_pack walks atoms and idles the groups whose atom has fewer holders than
// the wave's most-held atom).  Two passes: counts, records.
template <int W>
__global__ void __launch_bounds__(256) hgx_xb_pack_flat(int64_t E, const int32_t* __restrict__ bc_atom,
                                                        const int32_t* __restrict__ bc_part,
                                                        const int32_t* __restrict__ bc_lid, const u64* __restrict__ fa_next,
                                                        const u64* __restrict__ lvl_next, u64* __restrict__ cursor,
                                                        const int64_t* __restrict__ seg_h, const int64_t* __restrict__ seg_p,
                                                        u64* __restrict__ hdr, u64* __restrict__ pay, u64* __restrict__ nzw,
                                                        int NP) {
    constexpr int WPL = Lay<W>::WPL, G = Lay<W>::G, PER = 64 / G, U = 2;
    constexpr uint32_t FULLM = full_word_mask(W);
    typedef Vec<WPL> V;
    __shared__ PackLds sh;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, g = lane / G, sub = lane & (G - 1);
    const u64 lt = (1ull << lane) - 1ull;
    int64_t lo, hi;
    block_tiles((E + 63) / 64, lo, hi);
    for (int d = threadIdx.x; d < NP; d += 256) sh.rec[d] = sh.slot[d] = 0;
    __syncthreads();
    for (int pass = 0; pass < 2; ++pass) {
        u64 nz = 0;
        for (int64_t c = lo + wv; c < hi; c += 4) {   // wave-uniform
            const int64_t e = c * 64 + lane;
            int32_t t = 0, q = -1, lid = 0;
            if (e < E) {
                t = bc_atom[e];
                if (bit(fa_next, t)) {
                    q = bc_part[e];
                    lid = bc_lid[e];
                }
            }
            const u64 news = __ballot(q >= 0);
            if (!news) continue;   // wave-uniform
            int64_t local = 0;     // this lane's record: its rank among the block's records to q
            for (int d = 0; d < NP; ++d) {   // wave-uniform
                const u64 m = __ballot(q == d);
                if (!m) continue;
                unsigned long long b = 0;
                if (lane == 0) {
                    if (pass == 0) atomicAdd(&sh.rec[d], (unsigned int)__popcll(m));
                    else b = atomicAdd(&sh.slot[d], (unsigned long long)__popcll(m));
                }
                b = __shfl(b, 0);
                if (q == d) local = (int64_t)b + __popcll(m & lt);
            }
            if (pass == 0) continue;
            const int n = __popcll(news);
            for (int r0 = 0; r0 < n; r0 += PER * U) {   // wave-uniform
                typename V::T row[U];
                int64_t lc[U];
                int qq[U];
                int32_t ll[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int j = r0 + u * PER + g;
                    const int src = j < n ? nth_set_bit(news, j) : 0;
                    const int32_t ts = __shfl(t, src);
                    qq[u] = __shfl(q, src);
                    ll[u] = __shfl(lid, src);
                    lc[u] = (int64_t)__shfl((long long)local, src);
                    row[u] = j < n ? V::ld(lvl_next + (int64_t)ts * W + sub * WPL) : V::zero();
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    if (r0 + u * PER < n) {   // wave-uniform
                        const uint32_t nzm = group_mask<W>(row[u]);
                        if (r0 + u * PER + g < n) {
                            const int d = qq[u];
                            put_record<W>(hdr, pay + seg_p[d], seg_h[d] + (int64_t)sh.base_r[d] + lc[u],
                                          (int64_t)sh.base_w[d] + lc[u] * W, ll[u], FULLM, row[u], true);
                            if (sub == 0) nz += (u64)__popc(nzm);
                        }
                    }
                }
            }
        }
        __syncthreads();
        if (pass == 0) {
            for (int d = threadIdx.x; d < NP; d += 256) sh.wrd[d] = sh.rec[d] * (unsigned int)W;
            __syncthreads();
            pack_reserve(sh, cursor, NP);
            __syncthreads();
        } else {
            block_add_sh(nzw, 2, nz);
        }
    }
}

// Broadcast of a level on which (nearly) every ghost of the group has news: every broadcast entry
// writes a dense record at its static slot (bc_slot: the holder's ghosts of this owner in ascending
// order, so the holder knows every segment's size) -- mask all ones with news, 0 without (the holder
// skips it).  One pass, no counting, no LDS atomics; the phase needs no count read-back and no count
// all-gather.  U entries per lane group in flight.
template <int W>
__global__ void __launch_bounds__(256) hgx_xb_pack_static(int64_t E, int NP, const int32_t* __restrict__ bc_atom,
                                                          const int32_t* __restrict__ bc_part,
                                                          const int32_t* __restrict__ bc_lid,
                                                          const int32_t* __restrict__ bc_slot,
                                                          const u64* __restrict__ fa_next, const u64* __restrict__ lvl_next,
                                                          const int64_t* __restrict__ seg_h,
                                                          const int64_t* __restrict__ seg_p, u64* __restrict__ hdr,
                                                          u64* __restrict__ pay, u64* __restrict__ nzw) {
    constexpr int WPL = Lay<W>::WPL, G = Lay<W>::G, PER = 64 / G, U = 4;
    constexpr uint32_t FULLM = full_word_mask(W);
    typedef Vec<WPL> V;
    __shared__ int64_t sh_h[kMaxParts], sh_p[kMaxParts];
    for (int q = threadIdx.x; q < NP; q += blockDim.x) {
        sh_h[q] = seg_h[q];
        sh_p[q] = seg_p[q];
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, g = lane / G, sub = lane & (G - 1);
    const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    const int64_t nwave = ((int64_t)gridDim.x * blockDim.x) >> 6;
    u64 nz = 0;
    for (int64_t base = wave * PER * U; base < E; base += nwave * PER * U) {   // wave-uniform
        typename V::T row[U];
        int32_t q[U], lid[U], slot[U];
        bool ok[U], news[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t e = base + u * PER + g;
            ok[u] = e < E;
            const int32_t t = ok[u] ? bc_atom[e] : 0;
            q[u] = ok[u] ? bc_part[e] : 0;
            lid[u] = ok[u] ? bc_lid[e] : 0;
            slot[u] = ok[u] ? bc_slot[e] : 0;
            news[u] = ok[u] && bit(fa_next, t);
            row[u] = news[u] ? V::ld(lvl_next + (int64_t)t * W + sub * WPL) : V::zero();
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t nzm = group_mask<W>(row[u]);
            if (ok[u]) {
                put_record<W>(hdr, pay + sh_p[q[u]], sh_h[q[u]] + slot[u], (int64_t)slot[u] * W, lid[u],
                              news[u] ? FULLM : 0u, row[u], true);
                if (sub == 0) nz += (u64)__popc(nzm);
            }
        }
    }
    block_add_sh(nzw, 2, nz);
}

// Apply n received records (headers hdr, payload pay of one source), one G-lane group each.
// REDUCE: OR a partial row into an owned atom (new = row & ~vis; a source sends an atom at most
// once, so one launch per source segment); BROADCAST: a ghost's final row replaces the partial one
// (each ghost gets exactly one record).
template <int W, bool REDUCE>
__global__ void __launch_bounds__(256) hgx_x_apply(int64_t n, const u64* __restrict__ hdr, const u64* __restrict__ pay,
                                                   u64* __restrict__ lvl_next, u64* __restrict__ fa_next,
                                                   u64* __restrict__ vis, u64* __restrict__ ever, u64* __restrict__ full,
                                                   FullMask fm) {
    constexpr int WPL = Lay<W>::WPL, G = Lay<W>::G, PER = 64 / G;
    typedef Vec<WPL> V;
    const int lane = threadIdx.x & 63, g = lane / G, sub = lane & (G - 1);
    const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    const int64_t nwave = ((int64_t)gridDim.x * blockDim.x) >> 6;
    const typename V::T FULL = full_part<W>(fm, sub);
    for (int64_t base = wave * PER; base < n; base += nwave * PER) {   // wave-uniform
        const int64_t i = base + g;
        const bool valid = i < n;
        const u64x2 h = valid ? *reinterpret_cast<const u64x2*>(hdr + 2 * i) : u64x2{0ull, 0ull};
        const int64_t t = (int64_t)(uint32_t)h.x;
        const uint32_t mask = (uint32_t)(h.x >> 32);
        typename V::T row = V::zero();
        if (valid) {
            if constexpr (WPL == 1) {
                if ((mask >> sub) & 1u) row = pay[h.y + __popc(mask & ((1u << sub) - 1u))];
            } else {
                const int w0 = sub * 2;
                const int64_t p0 = (int64_t)h.y + __popc(mask & ((1u << w0) - 1u));
                const bool b0 = (mask >> w0) & 1u, b1 = (mask >> (w0 + 1)) & 1u;
                row.x = b0 ? pay[p0] : 0ull;
                row.y = b1 ? pay[p0 + b0] : 0ull;
            }
        }
        // the bitmap words and both rows are loaded at once (the rows of an atom not yet reached
        // or without news this level are read and discarded: one round trip instead of two)
        const bool ev = valid && bit(ever, t);
        const bool was = valid && bit(fa_next, t);
        const typename V::T vis0 = valid ? V::ld(vis + t * W + sub * WPL) : V::zero();
        const typename V::T lv0 = (REDUCE && valid) ? V::ld(lvl_next + t * W + sub * WPL) : V::zero();
        const typename V::T old = ev ? vis0 : V::zero();
        const typename V::T nw = REDUCE ? (row & ~old) : row;
        const bool any = group_any<G>(V::nz(nw));
        const bool isfull = group_all<G>(V::eq(old | nw, FULL));
        if (valid && (REDUCE ? any : mask != 0u)) {   // a static broadcast record without news has mask 0
            typename V::T lv = nw;
            if (REDUCE && was) lv = lv0 | nw;
            V::st(lvl_next + t * W + sub * WPL, lv);
            V::st(vis + t * W + sub * WPL, old | nw);
            if (sub == 0) {
                if (!was) set_bit(fa_next, t);
                if (!ev) set_bit(ever, t);
                if (isfull) set_bit(full, t);
            }
        }
    }
}

// (The static-slot exchange of round 2, HGX_OPT_PART_EXCHANGE 2 -- every ghost's whole row to a fixed slot
// of its owner, three launches a level -- measured 42.8 against 34.0 ms a part a step and was removed in
// round 5)

// out[0] += |frontier & own| (the part's share of the group's new atoms), out[1] += sum of |inc(v)|
// over the whole local frontier (the next level's local push volume).  A thread per bitmap word; the
// degrees of a run of consecutive frontier atoms are one difference of incidence offsets, so a
// dense word costs two loads (a wave walking its nonzero words one after the other took ~50 us of
// dependent loads even on a near-empty level).
__global__ void __launch_bounds__(256) hgx_frontier_stats(int64_t A, const u64* __restrict__ fa,
                                                          const u64* __restrict__ own,
                                                          const int64_t* __restrict__ inc_off, u64* __restrict__ out) {
    const int64_t nwords = (A + 63) / 64;
    u64 n = 0, deg = 0;
    for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < nwords; w += (int64_t)gridDim.x * blockDim.x) {
        u64 x = fa[w];
        if (!x) continue;
        n += __popcll(x & own[w]);
        const int64_t base = w * 64;
        while (x) {
            const int a0 = __ffsll((long long)x) - 1;
            const u64 rest = ~(x >> a0);
            const int r = rest ? __ffsll((long long)rest) - 1 : 64 - a0;   // run length
            deg += (u64)(inc_off[base + a0 + r] - inc_off[base + a0]);
            x &= (r + a0 >= 64) ? 0ull : (~0ull << (a0 + r));
        }
    }
    block_add_sh(out, 0, n);
    block_add_sh(out, 1, deg);
}

}  // namespace hgx

using namespace hgx;

// ---------------------------------------------------------------------------------------------
// Host orchestration
// ---------------------------------------------------------------------------------------------

// blocks of a counting pass (a wave per 64 bitmap words at least, kCountBlocks at most)
inline int count_grid(int64_t A) {
    const int64_t nwords = ceil_div(std::max<int64_t>(A, 1), 64);
    return (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(nwords, 64 * 4), kCountBlocks));
}

constexpr int kDirectLevels = 256;   // levels whose push-level counts the finalise accumulates
constexpr int kZeroLevels = 64;      // level counter blocks / count rows cleared per launch

// Up to kZeroParts device ranges cleared by one launch (a traversal's prologue cleared six buffers
// with six fill launches, each a few microseconds of device time and a gap).
constexpr int kZeroParts = 8;
struct ZeroSpans {
    u64* p[kZeroParts];
    int64_t n[kZeroParts];   // words
    int k;
};
__global__ void __launch_bounds__(256) hgx_zero_multi(ZeroSpans z) {
    const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x, nt = (int64_t)gridDim.x * blockDim.x;
    for (int j = 0; j < z.k; ++j) {
        u64x2* p = reinterpret_cast<u64x2*>(z.p[j]);
        const int64_t n2 = z.n[j] >> 1;
        for (int64_t i = t; i < n2; i += nt) p[i] = u64x2{0ull, 0ull};
        if ((z.n[j] & 1) && t == 0) z.p[j][z.n[j] - 1] = 0ull;
    }
}
struct ZeroList {
    ZeroSpans z{};
    int64_t most = 0;
    void add(void* p, size_t bytes) {
        if (z.k == kZeroParts) fail(HGX_E_DEVICE, "ZeroList: too many spans");
        z.p[z.k] = (u64*)p;
        z.n[z.k] = (int64_t)(bytes / sizeof(u64));
        most = std::max(most, z.n[z.k]);
        ++z.k;
    }
    void launch(hipStream_t s) {
        if (z.k == 0) return;
        hgx_zero_multi<<<grid_for(std::max<int64_t>(most / 2, 1), 256, 2048), 256, 0, s>>>(z);
        HGX_CHECK_LAUNCH();
    }
};

struct BfsBatch {
    int32_t seed0 = 0, S = 0, W = 0;
    int32_t n_expanded = 0;       // levels whose frontier was expanded (advance() iterated)
    std::vector<u64*> lvl;        // per level, A*W words (rows valid where fa bit set)
    std::vector<u64*> fa;         // per level, A bits
    u64* pcnt = nullptr;          // [kDirectLevels][1024] per-source counts of push levels (whole graph)
    std::vector<char> direct;     // direct[d]: level d's counts are in pcnt (no counting pass)
    // counting launched on g->stream2 as soon as a level is final, next to the following levels
    // (cpart[d]: its block partials, cgrid blocks of W*64 words; null = counted at readout)
    std::vector<uint32_t*> cpart;
    int cgrid = 0;
    size_t cpart_bytes = 0;
};

struct hgx_bfs_result {
    hgx_graph* g = nullptr;
    int32_t n_seeds = 0, n_levels = 0;
    std::vector<BfsBatch> batches;
    hgx_bfs_stats stats{};
    bool counts_ready = false, accounting_ready = false;
    bool typed = false;
    std::map<int32_t, int32_t> isolated;   // shards: seed index -> owned seed atom without incidence
    std::vector<int64_t> counts;   // [n_seeds * n_levels]
    // Seeds finished by the workgroup engine (HGX_OPT_BFS_BLOCK); the batches then hold only the
    // others, compacted: orig[k] = seed index of batch seed k, compact[i] = k (-1: a workgroup seed).
    std::unique_ptr<hgx::BlockSet> blk;
    std::vector<int32_t> orig, compact;
    int32_t orig_of(int32_t k) const { return orig.empty() ? k : orig[k]; }
    size_t row_bytes(const BfsBatch& b) const { return sizeof(u64) * (size_t)g->A * b.W; }
    size_t bm_bytes() const { return sizeof(u64) * (size_t)(g->A / 64 + 2); }
};

namespace {

struct Events {
    hipEvent_t a = nullptr, b = nullptr;
};

// Brackets kernels with events when timing is on; kind = HGX_K_*, level = BFS level.
struct Timer {
    hgx_graph* g;
    struct Rec {
        int kind, level;
        Events e;
        bool own_a;   // false: e.a is the previous record's e.b (chained levels, one event per boundary)
    };
    std::vector<Rec> rec;
    Events all{};
    bool on;
    hipEvent_t chain = nullptr;   // the last stop event when nothing was enqueued after it
    explicit Timer(hgx_graph* gg) : g(gg), on(gg->timing) {
        if (on) {
            all.a = take();
            all.b = take();
        }
    }
    ~Timer() {   // events go back to the graph's pool (the caller holds g->mu)
        for (auto& r : rec) {
            if (r.own_a) g->ev_pool.push_back(r.e.a);
            g->ev_pool.push_back(r.e.b);
        }
        if (all.a) g->ev_pool.push_back(all.a);
        if (all.b) g->ev_pool.push_back(all.b);
    }
    hipEvent_t take() {
        if (!g->ev_pool.empty()) {
            hipEvent_t e = g->ev_pool.back();
            g->ev_pool.pop_back();
            return e;
        }
        hipEvent_t e;
        HGX_HIP(hipEventCreate(&e));
        return e;
    }
    Events start(int kind, int level) {
        Events e{};
        chain = nullptr;
        if (!on) return e;
        e.a = take();
        e.b = take();
        HGX_HIP(hipEventRecord(e.a, g->stream));
        rec.push_back({kind, level, e, true});
        return e;
    }
    void stop(const Events& e) {
        if (on) HGX_HIP(hipEventRecord(e.b, g->stream));
    }
    // Consecutive push levels: a level starts at the previous level's stop event when nothing was
    // enqueued in between (an event record between two kernels costs several microseconds of idle
    // queue on a level of a few tens of microseconds).
    Events start_chained(int kind, int level) {
        if (!on || !chain) return start(kind, level);
        Events e{chain, take()};
        rec.push_back({kind, level, e, false});
        chain = nullptr;
        return e;
    }
    void stop_chained(const Events& e) {
        if (!on) return;
        HGX_HIP(hipEventRecord(e.b, g->stream));
        chain = e.b;
    }
    void break_chain() { chain = nullptr; }
    void collect(hgx_bfs_stats& st) {
        for (auto& r : rec) {
            float ms = 0;
            HGX_HIP(hipEventElapsedTime(&ms, r.e.a, r.e.b));
            if (r.kind == HGX_K_COUNT) {   // the partitioned exchange (pack / apply kernels)
                st.ms_exchange += ms;
                if (r.level < 64) {
                    st.level_ms[r.level] += ms;
                    st.level_xms[r.level] += ms;
                }
                continue;
            }
            st.ms_kernel[r.kind] += ms;
            if (r.level < 64) st.level_ms[r.level] += ms;
        }
    }
};

enum { kKindGather = HGX_K_LINK_GATHER, kKindPull = HGX_K_ATOM_PULL, kKindHeavy = HGX_K_PULL_HEAVY,
       kKindHub = HGX_K_HUB_FINALIZE, kKindPush = HGX_K_FRONTIER_PUSH, kKindNf = HGX_K_NF_PULL,
       kKindFc = HGX_K_FC_PULL, kKindFcHeavy = HGX_K_FC_HEAVY, kKindExchange = HGX_K_COUNT };

// Frontier-code pull: a level qualifies when its frontier rows (frontier atoms x S/8 bytes) fit well
// inside the 256 MiB Infinity Cache -- the codes then sit in L2 and the rare dense rows are cache hits.
constexpr double kFcFrontBytes = 64.0 * (1 << 20);
// The records cost 32 bytes per incidence entry for the snapshot's lifetime (config 2: 6.4 GB); larger
// snapshots (config 4: 32 GB) keep gather + pull rather than hold that much next to the level rows.
constexpr size_t kFcRecBudget = (size_t)16 << 30;

// The snapshot's per-entry target records (hgx_fc_rec), built on first use on the root snapshot and
// shared by its contexts; nullptr when over budget, when a quarter of the free device memory cannot
// hold them, or when some link has more than 8 targets.  Caller holds g->mu.
const int4* fc_records(hgx_graph* g, hipStream_t s) {
    hgx_graph* root = g->base ? g->base : g;
    std::lock_guard<std::mutex> lk(root->ylist_mu);
    if (root->fc_rec_state == 0) {
        root->fc_rec_state = -1;
        const size_t bytes = (size_t)32 * (size_t)root->I;
        size_t fr = 0, tot = 0;
        int4* rec = nullptr;
        if (root->I > 0 && bytes <= kFcRecBudget && hipMemGetInfo(&fr, &tot) == hipSuccess && bytes <= fr / 4 &&
            hipMalloc(&rec, bytes) == hipSuccess) {
            // the hubs: the kFcHubs heavy atoms of highest degree (ascending ids, for the records' binary search)
            std::vector<int32_t> hubs;
            if (root->n_heavy > 0) {
                const int64_t nh = root->n_heavy;
                std::vector<int32_t> ha((size_t)nh);
                std::vector<int64_t> hd((size_t)nh);
                int64_t* dd = (int64_t*)g->alloc(sizeof(int64_t) * (size_t)nh);
                hgx_fc_deg<<<grid_for(nh, 256, 4096), 256, 0, s>>>(nh, root->heavy_atom, root->inc_off, dd);
                HGX_CHECK_LAUNCH();
                HGX_HIP(hipMemcpyAsync(ha.data(), root->heavy_atom, sizeof(int32_t) * (size_t)nh, hipMemcpyDeviceToHost, s));
                HGX_HIP(hipMemcpyAsync(hd.data(), dd, sizeof(int64_t) * (size_t)nh, hipMemcpyDeviceToHost, s));
                HGX_HIP(hipStreamSynchronize(s));
                g->release(dd, sizeof(int64_t) * (size_t)nh);
                std::vector<int64_t> ord((size_t)nh);
                for (int64_t k = 0; k < nh; ++k) ord[(size_t)k] = k;
                const size_t keep = std::min<size_t>((size_t)nh, (size_t)kFcHubs);
                std::partial_sort(ord.begin(), ord.begin() + (int64_t)keep, ord.end(),
                                  [&](int64_t a, int64_t b) { return hd[(size_t)a] != hd[(size_t)b] ? hd[(size_t)a] > hd[(size_t)b] : a < b; });
                for (size_t k = 0; k < keep; ++k) hubs.push_back(ha[(size_t)ord[k]]);
                std::sort(hubs.begin(), hubs.end());
            }
            int32_t* dh = nullptr;
            if (!hubs.empty()) {
                HGX_HIP(hipMalloc(&dh, sizeof(int32_t) * hubs.size()));
                HGX_HIP(hipMemcpyAsync(dh, hubs.data(), sizeof(int32_t) * hubs.size(), hipMemcpyHostToDevice, s));
            }
            unsigned int* dov = (unsigned int*)g->alloc(16);
            HGX_HIP(hipMemsetAsync(dov, 0, sizeof(unsigned int), s));
            hgx_fc_rec<<<grid_for(root->I, 256, 16384), 256, 0, s>>>(root->A, root->I, root->inc_off, root->inc_row,
                                                                      root->tgt_off, root->tgt_idx, dh,
                                                                      (int32_t)hubs.size(), rec, dov);
            HGX_CHECK_LAUNCH();
            unsigned int over = 1;
            HGX_HIP(hipMemcpyAsync(&over, dov, sizeof(unsigned int), hipMemcpyDeviceToHost, s));
            HGX_HIP(hipStreamSynchronize(s));
            g->release(dov, 16);
            if (over) {
                (void)hipFree(rec);
                if (dh) (void)hipFree(dh);
            } else {
                root->fc_rec = rec;
                root->fc_hubs = dh;
                root->fc_nhubs = (int32_t)hubs.size();
                root->fc_rec_state = 1;
            }
        } else {
            (void)hipGetLastError();   // a failed hipMalloc: the levels keep gather + pull
        }
    }
    return root->fc_rec_state == 1 ? root->fc_rec : nullptr;
}

// Atoms with more than thr incidences and their ranges (order-free compaction).
__global__ void __launch_bounds__(256) hgx_push_heavy_find(int64_t A, const int64_t* __restrict__ inc_off,
                                                           int64_t thr, int64_t* __restrict__ out,
                                                           unsigned int* __restrict__ n) {
    for (int64_t a = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; a < A; a += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = inc_off[a], e = inc_off[a + 1];
        if (e - b > thr) {
            const unsigned k = atomicAdd(n, 1u);
            out[3 * (int64_t)k] = a;
            out[3 * (int64_t)k + 1] = b;
            out[3 * (int64_t)k + 2] = e;
        }
    }
}

// The frontier push's chunk table (once per snapshot): kPushChunk-entry chunks of every atom with
// more than kPushLight incidences, in atom order.
void build_push_chunks(hgx_graph* g) {
    hipStream_t s = g->stream;
    const int64_t A = g->A;
    // at most I / (kPushLight + 1) atoms have more than kPushLight incidences
    const int64_t nmax = std::min<int64_t>(g->I / (kPushLight + 1) + 1, std::max<int64_t>(A, 1));
    int64_t* dout = (int64_t*)g->alloc(sizeof(int64_t) * 3 * (size_t)nmax);
    unsigned int* dn = (unsigned int*)g->alloc(16);
    HGX_HIP(hipMemsetAsync(dn, 0, 4, s));
    hgx_push_heavy_find<<<grid_for(A, 256, 4096), 256, 0, s>>>(A, g->inc_off, kPushLight, dout, dn);
    HGX_CHECK_LAUNCH();
    unsigned int nh = 0;
    HGX_HIP(hipMemcpyAsync(&nh, dn, 4, hipMemcpyDeviceToHost, s));
    HGX_HIP(hipStreamSynchronize(s));
    std::vector<int64_t> h(3 * (size_t)nh);
    if (nh) HGX_HIP(hipMemcpyAsync(h.data(), dout, sizeof(int64_t) * 3 * nh, hipMemcpyDeviceToHost, s));
    HGX_HIP(hipStreamSynchronize(s));
    g->release(dout, sizeof(int64_t) * 3 * (size_t)nmax);
    g->release(dn, 16);
    std::vector<size_t> ord(nh);
    for (size_t i = 0; i < nh; ++i) ord[i] = i;
    std::sort(ord.begin(), ord.end(), [&](size_t x, size_t y) { return h[3 * x] < h[3 * y]; });
    std::vector<HeavyChunk> ch;
    for (size_t i : ord)
        for (int64_t b = h[3 * i + 1]; b < h[3 * i + 2]; b += kPushChunk)
            ch.push_back({b, std::min(h[3 * i + 2], b + kPushChunk), (int32_t)h[3 * i], -1});
    if (g->pchunks) HGX_HIP(hipFree(g->pchunks));
    g->pchunks = nullptr;
    HGX_HIP(hipMalloc(&g->pchunks, sizeof(HeavyChunk) * std::max<size_t>(ch.size(), 1)));
    if (!ch.empty())
        HGX_HIP(hipMemcpyAsync(g->pchunks, ch.data(), sizeof(HeavyChunk) * ch.size(), hipMemcpyHostToDevice, s));
    HGX_HIP(hipStreamSynchronize(s));
    g->n_pchunks = (int64_t)ch.size();
}

FullMask full_mask(int S, int W) {
    FullMask fm;
    for (int w = 0; w < 16; ++w) {
        int n = S - w * 64;
        fm.w[w] = (w >= W || n <= 0) ? 0ull : (n >= 64 ? ~0ull : ((1ull << n) - 1ull));
    }
    return fm;
}

// The exchange's count vectors, gathered on the device (Transport::allgather_dev: RCCL all-gathers
// them without a host copy in between).  Reduce / broadcast phase: [records to q (NP), words to q (NP),
// my ghosts, nonzero words shipped]; end of level: [owned new atoms, push volume, nonzero words].
__global__ void k_x_counts(int NP, const u64* __restrict__ dctr, int64_t ghosts, int64_t* __restrict__ out) {
    const int t = threadIdx.x;
    if (t < NP) {
        out[t] = (int64_t)dctr[(size_t)t * kCurStride];
        out[NP + t] = (int64_t)dctr[(size_t)t * kCurStride + 16];
    }
    if (t == 0) {
        const u64* xs = dctr + (size_t)NP * kCurStride;
        u64 z = 0;
        for (int k = 0; k < kStatShards; ++k) z += xs[k * kStatStride + 2];
        out[2 * NP] = ghosts;
        out[2 * NP + 1] = (int64_t)z;
    }
}
__global__ void k_x_finish(const u64* __restrict__ xs, int64_t* __restrict__ out) {
    const int t = threadIdx.x;
    if (t < 3) {
        u64 v = 0;
        for (int k = 0; k < kStatShards; ++k) v += xs[k * kStatStride + t];
        out[t] = (int64_t)v;
    }
}

// Per-batch buffers of the partitioned exchange (vertex cut).  Segment
// capacities are static: part q receives from me at most my ghosts owned by q (reduce) and my
// owned atoms held by q (broadcast); symmetrically for what I receive.  A segment of cap records
// has cap 16-byte headers and at most cap * W payload words.
struct Exchange {
    hgx_graph* g;
    Transport* tr;
    int W;
    int64_t cap_recs = 0;               // send / receive area capacity (records)
    u64* send_h = nullptr;              // header streams (2 words per record)
    u64* recv_h = nullptr;
    u64* send_p = nullptr;              // payload streams (W words per record at most)
    u64* recv_p = nullptr;
    u64* dctr = nullptr;                // [NP * kCurStride] cursors, then kStatShards x kStatStride stats:
                                        // [0] owned new atoms, [1] push volume, [2] nonzero words
    int64_t* seg = nullptr;             // [4 * NP] device: reduce h / p, broadcast h / p segment starts
    std::vector<int64_t> rseg, bseg;    // host copies (reduce, broadcast; records), NP + 1 entries
    double bytes_sent = 0, nz_words = 0, words = 0;
    u64* hpin = nullptr;                // pinned landing area of the cursor / stats read-backs
    int64_t* dvec = nullptr;            // [2 * NP + 2] device count vector of the next all-gather
    int64_t* gpin = nullptr;            // [(2 * NP + 2) * NP] pinned landing area of the gathered vectors
    Exchange(hgx_graph* gg, Transport* t, int w) : g(gg), tr(t), W(w) {
        ShardInfo& sh = *g->shard;
        const int NP = sh.n_parts;
        HGX_HIP(hipHostMalloc(&hpin, sizeof(u64) * (NP * kCurStride + kStatShards * kStatStride), hipHostMallocDefault));
        HGX_HIP(hipHostMalloc(&gpin, sizeof(int64_t) * (2 * NP + 2) * NP, hipHostMallocDefault));
        rseg.assign(NP + 1, 0);
        bseg.assign(NP + 1, 0);
        for (int q = 0; q < NP; ++q) {
            rseg[q + 1] = rseg[q] + sh.ghost_count[q];
            bseg[q + 1] = bseg[q] + sh.bc_count[q];
        }
        cap_recs = std::max<int64_t>(std::max(rseg[NP], bseg[NP]), 1);
        if (cap_recs >= ((int64_t)1 << 32)) fail(HGX_E_INVALID, "partitioned BFS: exchange segment above 2^32 records");
        send_h = (u64*)g->alloc(sizeof(u64) * 2 * (size_t)cap_recs);
        recv_h = (u64*)g->alloc(sizeof(u64) * 2 * (size_t)cap_recs);
        send_p = (u64*)g->alloc(sizeof(u64) * W * (size_t)cap_recs);
        recv_p = (u64*)g->alloc(sizeof(u64) * W * (size_t)cap_recs);
        dctr = (u64*)g->alloc(sizeof(u64) * (NP * kCurStride + kStatShards * kStatStride));
        dvec = (int64_t*)g->alloc(sizeof(int64_t) * (2 * NP + 2));
        seg = (int64_t*)g->alloc(sizeof(int64_t) * 4 * NP);
        std::vector<int64_t> hs(4 * (size_t)NP);
        for (int q = 0; q < NP; ++q) {
            hs[q] = rseg[q];
            hs[NP + q] = rseg[q] * W;
            hs[2 * NP + q] = bseg[q];
            hs[3 * NP + q] = bseg[q] * W;
        }
        HGX_HIP(hipMemcpyAsync(seg, hs.data(), sizeof(int64_t) * 4 * NP, hipMemcpyHostToDevice, g->stream));
        HGX_HIP(hipStreamSynchronize(g->stream));   // hs is a local
    }
    // cursor / stats words back to the host (pinned copy, polled: no staging, no sleeping wait)
    int trips = 0;                      // host round trips of the current level (read-backs, count all-gathers)
    void read_back(std::vector<u64>& hc, size_t cbytes) {
        ++trips;
        HGX_HIP(hipMemcpyAsync(hpin, dctr, cbytes, hipMemcpyDeviceToHost, g->stream));
        spin_sync(g->stream);
        std::memcpy(hc.data(), hpin, cbytes);
    }
    ~Exchange() {
        if (hpin) (void)hipHostFree(hpin);
        if (gpin) (void)hipHostFree(gpin);
        const int NP = g->shard->n_parts;
        g->release(dvec, sizeof(int64_t) * (2 * NP + 2));
        g->release(send_h, sizeof(u64) * 2 * (size_t)cap_recs);
        g->release(recv_h, sizeof(u64) * 2 * (size_t)cap_recs);
        g->release(send_p, sizeof(u64) * W * (size_t)cap_recs);
        g->release(recv_p, sizeof(u64) * W * (size_t)cap_recs);
        g->release(dctr, sizeof(u64) * (NP * kCurStride + kStatShards * kStatStride));
        g->release(seg, sizeof(int64_t) * 4 * NP);
    }
    // collective step: the part's device work is bracketed by compute_begin / compute_end
    template <class F>
    void coll(F f) {
        tr->compute_end(g->stream);
        f();
        tr->compute_begin(g->stream);
    }
    // One exchange phase: counts -> all-to-all of the header and payload segments.  sbase / rbase:
    // segment starts (records) of what I send / receive; rbase[q+1] - rbase[q] bounds what q sends
    // me.  Returns the per-source record counts; source q's records land at recv_h + 2 * rbase[q],
    // its payload at recv_p + W * rbase[q].  *pair_max: the largest bytes I send one peer.
    // *group (optional): the group's records, words and ghosts (every part gets the same numbers).
    // The count vectors of a record phase (k_x_counts after the phase's pack), gathered from every
    // part: all[p * K ..] is part p's (K = 2 NP + 2); my records / words per destination go to cnt /
    // wcnt.  RCCL gathers them on the device: one host round trip instead of a read-back plus a
    // host all-gather.
    void gather_counts(std::vector<int64_t>& all, std::vector<u64>& cnt, std::vector<u64>& wcnt) {
        ShardInfo& sh = *g->shard;
        const int NP = sh.n_parts, me = sh.part;
        const int K = 2 * NP + 2;
        all.assign((size_t)NP * K, 0);
        k_x_counts<<<1, 64, 0, g->stream>>>(NP, dctr, rseg[NP], dvec);
        HGX_CHECK_LAUNCH();
        coll([&] { trips += tr->allgather_dev(dvec, K, all.data(), g->stream, gpin); });
        for (int q = 0; q < NP; ++q) {
            cnt[q] = (u64)all[(size_t)me * K + q];
            wcnt[q] = (u64)all[(size_t)me * K + NP + q];
            words += (double)cnt[q] * W;
        }
        nz_words += (double)all[(size_t)me * K + 2 * NP + 1];
    }
    void ship(const std::vector<int64_t>& sbase, const std::vector<int64_t>& rbase, const std::vector<int64_t>& all,
              std::vector<int64_t>& rcnt, double* pair_max, double* group = nullptr) {
        ShardInfo& sh = *g->shard;
        const int NP = sh.n_parts, me = sh.part;
        const int K = 2 * NP + 2;   // records and words to every part, my ghost count, nonzero words
        const int64_t* mine = all.data() + (size_t)me * K;
        if (group) {
            group[0] = group[1] = group[2] = 0;
            for (int p = 0; p < NP; ++p) {
                for (int q = 0; q < NP; ++q) {
                    group[0] += (double)all[(size_t)p * K + q];
                    group[1] += (double)all[(size_t)p * K + NP + q];
                }
                group[2] += (double)all[(size_t)p * K + 2 * NP];
            }
        }
        std::vector<int64_t> soff(NP), sbytes(NP), roff(NP), rbytes(NP), psoff(NP), psbytes(NP), proff(NP),
            prbytes(NP);
        rcnt.assign(NP, 0);
        *pair_max = 0;
        for (int q = 0; q < NP; ++q) {
            const int64_t rr = all[(size_t)q * K + me], rw = all[(size_t)q * K + NP + me];
            if (rr > rbase[q + 1] - rbase[q] || rw > rr * W) fail(HGX_E_DEVICE, "partitioned BFS: receive overflow");
            rcnt[q] = rr;
            soff[q] = sbase[q] * 16;
            sbytes[q] = mine[q] * 16;
            roff[q] = rbase[q] * 16;
            rbytes[q] = rr * 16;
            psoff[q] = sbase[q] * W * 8;
            psbytes[q] = mine[NP + q] * 8;
            proff[q] = rbase[q] * W * 8;
            prbytes[q] = rw * 8;
            bytes_sent += (double)(sbytes[q] + psbytes[q]);
            *pair_max = std::max(*pair_max, (double)(sbytes[q] + psbytes[q]));
        }
        coll([&] {
            tr->alltoallv(send_h, soff.data(), sbytes.data(), recv_h, roff.data(), rbytes.data(), g->stream);
            tr->alltoallv(send_p, psoff.data(), psbytes.data(), recv_p, proff.data(), prbytes.data(), g->stream);
        });
    }
    // Reduce + broadcast of one level.  Returns the group-wide number of new atoms; *push_volume =
    // sum of |inc| over my (local) new frontier; *level_bytes: bytes I sent; *pair_max: the sum over
    // the level's two phases of the largest bytes I send one peer (the phases run one after the other).
    template <int Wt>
    // last: the traversal's final level (depth limit reached): the owners still need their ghosts'
    // news (the result counts and lists are the owners'), but no later level reads a ghost's row, so
    // the broadcast phase (pack, transfer, apply) is skipped.
    u64 level(u64* lvl_next, u64* fa_next, u64* vis, u64* ever, u64* full, const FullMask& fm, u64* push_volume,
              double* level_bytes, double* pair_max, Timer& tm, int d, bool last) {
        ShardInfo& sh = *g->shard;
        const int NP = sh.n_parts, me = sh.part;
        hipStream_t s = g->stream;
        const int64_t A = g->A;
        const int pgrid = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(A, 64) / 4 + 1, 2048));
        const double before = bytes_sent;
        trips = 0;
        const size_t cbytes = sizeof(u64) * (NP * kCurStride + kStatShards * kStatStride);
        u64* xs = dctr + NP * kCurStride;   // sharded stats (see dctr)
        std::vector<u64> hc(NP * kCurStride + kStatShards * kStatStride), cnt(NP), wcnt(NP);
        std::vector<int64_t> rcnt;
        auto apply = [&](bool reduce, const std::vector<int64_t>& rbase) {
            for (int q = 0; q < NP; ++q) {
                if (q == me || rcnt[q] == 0) continue;
                const int grid = grid_for(ceil_div(rcnt[q], 64 / Lay<Wt>::G) * 64, 256, 8192);
                const u64* h = recv_h + 2 * rbase[q];
                const u64* p = recv_p + (size_t)Wt * rbase[q];
                if (reduce)
                    hgx_x_apply<Wt, true><<<grid, 256, 0, s>>>(rcnt[q], h, p, lvl_next, fa_next, vis, ever, full, fm);
                else
                    hgx_x_apply<Wt, false><<<grid, 256, 0, s>>>(rcnt[q], h, p, lvl_next, fa_next, vis, ever, full, fm);
                HGX_CHECK_LAUNCH();
            }
        };
        double pm_r = 0, pm_b = 0;
        // reduce: partial rows of my ghosts -> their owners
        Events e0 = tm.start(kKindExchange, d);
        HGX_HIP(hipMemsetAsync(dctr, 0, cbytes, s));
        hgx_xr_pack<Wt><<<pgrid, 256, 0, s>>>(A, fa_next, (const u64*)sh.own_bm, sh.xo_part, sh.xo_lid, lvl_next, dctr,
                                              seg, seg + NP, send_h, send_p, xs, NP);
        HGX_CHECK_LAUNCH();
        tm.stop(e0);
        std::vector<int64_t> all;
        gather_counts(all, cnt, wcnt);
        // a dense level (at least half of my ghosts with news, rows > 70% nonzero words) packs its
        // broadcast over the entries (hgx_xb_pack_flat); HGX_OPT_XB_FLAT 0 keeps the atom walk on every
        // level, 2 takes the entries on every level (A/B and tests)
        u64 sent_r = 0, sent_w = 0;
        for (int q = 0; q < NP; ++q) {
            sent_r += cnt[q];
            sent_w += wcnt[q];
        }
        const int flat_opt = g->xb_flat >= 0 ? g->xb_flat : 1;
        const bool flat = bseg[NP] > 0 && (flat_opt == 2 || (flat_opt == 1 && sent_r * 2 >= (u64)rseg[NP] &&
                                                             sent_w * 10 > sent_r * (u64)Wt * 7));
        double grp[3];
        ship(rseg, bseg, all, rcnt, &pm_r, grp);
        // static broadcast (group-wide choice from the all-gathered reduce counts, so every part
        // agrees): at least 85% of the group's ghosts had news and their rows were > 70% nonzero
        // words -- shipping a record for every entry then costs < 18% more bytes than the news alone
        // and saves the counting pass and the phase's count round trips.  HGX_OPT_XB_STATIC 0 never,
        // 2 on every level (A/B and tests; every part of a group must use the same value).
        const int static_opt = g->xb_static >= 0 ? g->xb_static : 1;
        const bool bstatic = static_opt == 2 || (static_opt == 1 && grp[2] > 0 && grp[0] >= 0.85 * grp[2] &&
                                                 grp[1] * 10.0 > grp[0] * Wt * 7.0);
        Events e1 = tm.start(kKindExchange, d);
        apply(true, bseg);
        if (last) {   // no broadcast after the final level
            HGX_HIP(hipMemsetAsync(dctr, 0, cbytes, s));
            hgx_frontier_stats<<<grid_for(ceil_div(A, 64), 256, 2048), 256, 0, s>>>(
                A, fa_next, (const u64*)sh.own_bm, g->inc_off, xs);
            HGX_CHECK_LAUNCH();
            tm.stop(e1);
            return finish_level(push_volume, level_bytes, pair_max, before, pm_r);
        }
        // broadcast: final rows of my owned atoms -> their other holders
        HGX_HIP(hipMemsetAsync(dctr, 0, cbytes, s));
        if (bstatic) {
            const int64_t E = bseg[NP];
            if (E > 0) {
                const int sgrid = grid_for(ceil_div(E, 4) * Lay<Wt>::G, 256, 4096);
                hgx_xb_pack_static<Wt><<<sgrid, 256, 0, s>>>(E, NP, sh.bc_atom, sh.bc_part, sh.bc_lid, sh.bc_slot,
                                                             fa_next, lvl_next, seg + 2 * NP, seg + 3 * NP, send_h,
                                                             send_p, xs);
                HGX_CHECK_LAUNCH();
            }
            tm.stop(e1);
            ship_known(bseg, sh.bc_count, rseg, sh.ghost_count, &pm_b);
            rcnt.assign(sh.ghost_count.begin(), sh.ghost_count.end());
            Events e2 = tm.start(kKindExchange, d);
            apply(false, rseg);
            hgx_frontier_stats<<<grid_for(ceil_div(A, 64), 256, 2048), 256, 0, s>>>(
                A, fa_next, (const u64*)sh.own_bm, g->inc_off, xs);
            HGX_CHECK_LAUNCH();
            tm.stop(e2);
            return finish_level(push_volume, level_bytes, pair_max, before, pm_r + pm_b, true);
        }
        if (flat) {
            const int64_t E = bseg[NP];
            const int fgrid = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(E, 64) / 4 + 1, 2048));
            hgx_xb_pack_flat<Wt><<<fgrid, 256, 0, s>>>(E, sh.bc_atom, sh.bc_part, sh.bc_lid, fa_next, lvl_next, dctr,
                                                       seg + 2 * NP, seg + 3 * NP, send_h, send_p, xs, NP);
        } else {
            hgx_xb_pack<Wt><<<pgrid, 256, 0, s>>>(A, fa_next, (const u64*)sh.own_bm, sh.bc_off, sh.bc_part, sh.bc_lid,
                                                  lvl_next, dctr, seg + 2 * NP, seg + 3 * NP, send_h, send_p, xs, NP);
        }
        HGX_CHECK_LAUNCH();
        tm.stop(e1);
        gather_counts(all, cnt, wcnt);
        ship(bseg, rseg, all, rcnt, &pm_b);
        Events e2 = tm.start(kKindExchange, d);
        apply(false, rseg);
        hgx_frontier_stats<<<grid_for(ceil_div(A, 64), 256, 2048), 256, 0, s>>>(
            A, fa_next, (const u64*)sh.own_bm, g->inc_off, xs);
        HGX_CHECK_LAUNCH();
        tm.stop(e2);
        return finish_level(push_volume, level_bytes, pair_max, before, pm_r + pm_b);
    }
    // the level's statistics back to the host, the group's new-atom total
    // (gathered on the device like the record counts; add_nz: count the nonzero words the level's
    // static broadcast shipped)
    u64 finish_level(u64* push_volume, double* level_bytes, double* pair_max, double before, double pm,
                     bool add_nz = false) {
        const int NP = g->shard->n_parts, me = g->shard->part;
        hipStream_t s = g->stream;
        k_x_finish<<<1, 64, 0, s>>>(dctr + (size_t)NP * kCurStride, dvec);
        HGX_CHECK_LAUNCH();
        std::vector<int64_t> all(3 * (size_t)NP);
        coll([&] { trips += tr->allgather_dev(dvec, 3, all.data(), s, gpin); });
        *push_volume = (u64)all[(size_t)me * 3 + 1];
        if (add_nz) nz_words += (double)all[(size_t)me * 3 + 2];
        *level_bytes = bytes_sent - before;
        *pair_max = pm;
        u64 tot = 0;
        for (int q = 0; q < NP; ++q) tot += (u64)all[(size_t)q * 3];
        return tot;
    }
    // A record phase whose sizes both sides know (static broadcast): scnt[q] records (headers and W
    // words each) from my segments sbase[q] to q, rcnt[q] from q into rbase[q].  No count exchange.
    void ship_known(const std::vector<int64_t>& sbase, const std::vector<int64_t>& scnt,
                    const std::vector<int64_t>& rbase, const std::vector<int64_t>& rcnt, double* pair_max) {
        const int NP = g->shard->n_parts;
        std::vector<int64_t> soff(NP), sbytes(NP), roff(NP), rbytes(NP), psoff(NP), psbytes(NP), proff(NP),
            prbytes(NP);
        *pair_max = 0;
        for (int q = 0; q < NP; ++q) {
            soff[q] = sbase[q] * 16;
            sbytes[q] = scnt[q] * 16;
            roff[q] = rbase[q] * 16;
            rbytes[q] = rcnt[q] * 16;
            psoff[q] = sbase[q] * W * 8;
            psbytes[q] = scnt[q] * W * 8;
            proff[q] = rbase[q] * W * 8;
            prbytes[q] = rcnt[q] * W * 8;
            bytes_sent += (double)(sbytes[q] + psbytes[q]);
            words += (double)scnt[q] * W;
            *pair_max = std::max(*pair_max, (double)(sbytes[q] + psbytes[q]));
        }
        coll([&] {
            tr->alltoallv(send_h, soff.data(), sbytes.data(), recv_h, roff.data(), rbytes.data(), g->stream);
            tr->alltoallv(send_p, psoff.data(), psbytes.data(), recv_p, proff.data(), prbytes.data(), g->stream);
        });
    }
};

template <int W, int MODE>
void run_levels(hgx_graph* g, hgx_bfs_result* res, BfsBatch& bt, int32_t max_depth, int32_t want_type,
                const std::vector<int32_t>& seed_atoms, const std::vector<u64>& seed_rows, Timer& tm,
                std::vector<std::vector<u64>>& level_ctr, Transport* tr) {
    hipStream_t s = g->stream;
    const int64_t A = g->A, M = g->M;
    const size_t row_bytes = sizeof(u64) * (size_t)A * W;
    const size_t bm_bytes = res->bm_bytes();
    const size_t la_bytes = sizeof(u64) * (size_t)(M / 64 + 2);
    const FullMask fm = full_mask(bt.S, W);
    const u64* own_bm = g->shard ? (const u64*)g->shard->own_bm : nullptr;   // partition part: owned atoms
    // a partition part's device work runs between compute_begin / compute_end (the exchange releases
    // it around each collective); the guard releases it on an error path too
    struct Gate {
        Transport* tr;
        hipStream_t s;
        explicit Gate(Transport* t, hipStream_t st) : tr(t), s(st) {
            if (tr) tr->compute_begin(s);
        }
        ~Gate() {
            if (tr) tr->compute_release(s);
        }
    } gate(tr, s);

    u64* vis = (u64*)g->alloc(row_bytes);
    u64* lf = (MODE == kSym) ? (u64*)g->alloc(sizeof(u64) * (size_t)std::max<int64_t>(M, 1) * W) : nullptr;
    u64* hubacc = (u64*)g->alloc(sizeof(u64) * (size_t)std::max<int64_t>(g->n_heavy, 1) * W);
    u64* ever = (u64*)g->alloc(bm_bytes);
    u64* full = (u64*)g->alloc(bm_bytes);
    u64* la = (u64*)g->alloc(la_bytes);
    const int max_levels_cap = 4096;
    u64* ctr = (u64*)g->alloc(sizeof(u64) * kCtrBlock * max_levels_cap);
    int32_t* d_atoms = (int32_t*)g->alloc(sizeof(int32_t) * seed_atoms.size());
    u64* d_rows = (u64*)g->alloc(sizeof(u64) * seed_rows.size());
    // one pinned region: two levels' counters in flight, then the seed atoms and rows going up (a copy
    // from pageable memory is staged by the runtime and holds the host)
    const size_t o_atoms = sizeof(u64) * kCtrBlock * 2;
    const size_t o_rows = (o_atoms + sizeof(int32_t) * seed_atoms.size() + 15) & ~(size_t)15;
    char* hp = (char*)g->pinned_buf(o_rows + sizeof(u64) * seed_rows.size());
    u64* h_sh = (u64*)hp;
    u64 h_new[cNum];
    std::memcpy(hp + o_atoms, seed_atoms.data(), sizeof(int32_t) * seed_atoms.size());
    std::memcpy(hp + o_rows, seed_rows.data(), sizeof(u64) * seed_rows.size());

    // the prologue's buffers cleared by one launch; level counter blocks (and push-level count rows)
    // are cleared kZeroLevels at a time as the traversal reaches them
    bt.lvl.push_back((u64*)g->alloc(row_bytes));
    bt.fa.push_back((u64*)g->alloc(bm_bytes));
    const bool sparse_ok = (g->bfs_flags & 8) != 0;
    u64* lcand = sparse_ok ? (u64*)g->alloc(la_bytes) : nullptr;
    u64* cand = sparse_ok ? (u64*)g->alloc(bm_bytes) : nullptr;
    const size_t flist_bytes = sizeof(int32_t) * (size_t)std::max<int64_t>(A, 1);
    int32_t* flist = sparse_ok ? (int32_t*)g->alloc(flist_bytes) : nullptr;   // frontier list (push levels)
    int32_t* clist = sparse_ok ? (int32_t*)g->alloc(flist_bytes) : nullptr;   // push candidates
    ZeroList z{};
    if (cand) z.add(cand, bm_bytes);   // the first push level's candidate words (no memset of their own)
    z.add(ever, bm_bytes);
    z.add(full, bm_bytes);
    z.add(bt.fa[0], bm_bytes);
    z.add(hubacc, sizeof(u64) * (size_t)std::max<int64_t>(g->n_heavy, 1) * W);
    z.add(ctr, sizeof(u64) * kCtrBlock * kZeroLevels);
    z.add(ctr + (size_t)(max_levels_cap - 1) * kCtrBlock, sizeof(u64) * kCtrBlock);   // scratch slots
    if (!tr) {   // per-source counts of push levels, accumulated by their finalise (readout without a pass)
        bt.pcnt = (u64*)g->alloc(sizeof(u64) * 1024 * kDirectLevels);
        z.add(bt.pcnt, sizeof(u64) * 1024 * kZeroLevels);
        bt.direct.assign(kDirectLevels, 0);
    }
    z.launch(s);
    HGX_HIP(hipMemcpyAsync(d_atoms, hp + o_atoms, sizeof(int32_t) * seed_atoms.size(), hipMemcpyHostToDevice, s));
    HGX_HIP(hipMemcpyAsync(d_rows, hp + o_rows, sizeof(u64) * seed_rows.size(), hipMemcpyHostToDevice, s));
    {
        int n = (int)seed_atoms.size();
        hgx_seed<W><<<grid_for(n, 256, 1 << 20), 256, 0, s>>>(n, d_atoms, d_rows, bt.lvl[0], vis, bt.fa[0], ever,
                                                              full, fm);
        HGX_CHECK_LAUNCH();
    }
    // Readout counting next to the traversal (A/B, HGX_COUNT_EAGER=1): a level's rows are final once
    // it is produced, so its counting pass can run on a second stream while the following levels run.
    // Measured slower on config 2 (19.36 against 18.66 ms for traversal + readout,
    // profiles/r02zj_readout_*.log): the passes share HBM and CUs with the dense levels and delay
    // them by more than they save.  Default: counted at readout time.  Push levels count their news
    // in their finalise and need no pass either way.
    const char* ce = ab_env("HGX_COUNT_EAGER");
    const bool eager = !tr && !g->shard && ce && ce[0] == '1';
    if (eager && !g->stream2) {
        HGX_HIP(hipStreamCreateWithFlags(&g->stream2, hipStreamNonBlocking));
        HGX_HIP(hipEventCreateWithFlags(&g->ev_count, hipEventDisableTiming));
    }
    auto count_now = [&](size_t lev, hipEvent_t after) {   // level lev of bt: its counting pass on stream2
        if (!eager) return;
        if (lev < bt.direct.size() && bt.direct[lev]) return;
        if (bt.cpart.size() <= lev) bt.cpart.resize(lev + 1, nullptr);
        bt.cgrid = count_grid(A);
        bt.cpart_bytes = sizeof(uint32_t) * (size_t)bt.cgrid * W * 64;
        bt.cpart[lev] = (uint32_t*)g->alloc(bt.cpart_bytes);
        HGX_HIP(hipStreamWaitEvent(g->stream2, after, 0));
        hgx_count_rows<W><<<bt.cgrid, 256, 0, g->stream2>>>(A, bt.fa[lev], nullptr, bt.lvl[lev], bt.cpart[lev]);
        HGX_CHECK_LAUNCH();
    };
    if (eager) {
        HGX_HIP(hipEventRecord(g->ev_count, s));
        count_now(0, g->ev_count);
    }

    const int block = 256;
    const int gather_grid = grid_for(ceil_div(M, 64) * 64, block, 256 * 16);
    const int pull_grid = grid_for(ceil_div(A, 64) * 64, block, 256 * 16);
    const int hub_grid = grid_for(std::max<int64_t>(g->n_heavy, 1) * Lay<W>::G, block, 256 * 16);
    const int32_t maxd = max_depth < 0 ? INT32_MAX : max_depth;

    // Direction choice per level (Beamer-style): when the frontier's incidence volume
    // sum_{v in F} |inc(v)| is small, the level runs sparse -- candidate links are pushed from the
    // frontier atoms and only candidate tiles are gathered / pulled.  Otherwise every tile is scanned.
    std::unique_ptr<Exchange> ex;   // one part: no ghosts, nothing to exchange
    if (tr && tr->world > 1) ex.reset(new Exchange(g, tr, W));
    // push levels: fl = this level's frontier list, cl = its candidates; the finalise turns cl into the
    // next level's frontier list (chained), so consecutive push levels swap the two
    int32_t *fl = flist, *cl = clist;
    u64* n_fl = ctr + (size_t)(max_levels_cap - 1) * kCtrBlock + 10;   // scratch slots
    u64* n_cl = n_fl + 1;
    u64* ticket = n_fl + 2;   // the finalise's last-block ticket (re-zeroed by that block)
    if (!g->ctr_host) {       // two level slots + the seed-volume slot of mapped, coherent host memory
        void* hp = nullptr;  // (once per graph)
        HGX_HIP(hipHostMalloc(&hp, sizeof(u64) * 3 * kHostSlot, hipHostMallocMapped | hipHostMallocCoherent));
        std::memset(hp, 0, sizeof(u64) * 3 * kHostSlot);
        g->ctr_host = (u64*)hp;
    }
    if (!g->pend_ev[0])   // the two in-flight levels' events (once per graph)
        for (int k = 0; k < 2; ++k) HGX_HIP(hipEventCreateWithFlags(&g->pend_ev[k], hipEventDisableTiming));
    // cand was cleared by the prologue launch, and so were the scratch slots n_fl / n_cl (until a level
    // uses them): the first push level issues no memset (each costs a host API call, ~20 us between
    // the prologue's device operations on config 5)
    bool chained = false, cand_clean = cand != nullptr, scratch_clean = true;
    const bool trace = trace_env("HGX_BFS_TRACE");   // per-level counters to stderr
    const int64_t I_total = g->I;
    int64_t full_deg_total = 0;   // sum of |inc(v)| over the atoms visited by every traversal
    u64 push_volume = 0, push_volume_nf = 0;   // frontier incidence volume (all / not yet full atoms)
    u64 front_atoms = seed_atoms.size();       // atoms of the current level's frontier
    if (sparse_ok) {
        u64* slot = g->ctr_host + 2 * kHostSlot;
        const u64 seq = ++g->ctr_seq;
        __atomic_store_n(slot + 1, (u64)0, __ATOMIC_RELEASE);
        hgx_seed_degree_host<<<1, 256, 0, s>>>((int32_t)seed_atoms.size(), d_atoms, g->inc_off, slot, seq);
        HGX_CHECK_LAUNCH();
        for (unsigned spin = 0; __atomic_load_n(slot + 1, __ATOMIC_ACQUIRE) != seq; ++spin) {
            if ((spin & 1023u) != 1023u) continue;   // the stream is asked every 1024 polls
            const hipError_t e = hipStreamQuery(s);
            if (e == hipErrorNotReady) continue;
            if (e != hipSuccess) HGX_HIP(e);
            if (__atomic_load_n(slot + 1, __ATOMIC_ACQUIRE) != seq) fail(HGX_E_DEVICE, "batched BFS: seed volume never arrived");
        }
        push_volume = __atomic_load_n(slot, __ATOMIC_RELAXED);
        push_volume_nf = push_volume;
    }
    // HGX_SPARSE_SCALE (A/B builds): multiplies the push / dense threshold (M / 16 incidence entries)
    static const double kSparseScale = [] {
        const char* e = ab_env("HGX_SPARSE_SCALE");
        const double v = e ? std::atof(e) : 1.0;
        return v > 0 ? v : 1.0;
    }();
    const u64 sparse_limit = (u64)std::max<int64_t>((int64_t)((double)(M / 16) * kSparseScale), 1024);
    // Full-visited skipping costs two bitmap probes per pin; it pays once a sizeable share of the
    // atoms is visited by every traversal (seeds that are full count from the start).
    u64 full_total = 0;

    struct Pend {
        int32_t d = 0;
        u64* lvl_next = nullptr;
        u64* fa_next = nullptr;
        int kind = 0, allrows = 0;
        u64 new_global = 0, part_push = 0;
        u64* h = nullptr;
        hipEvent_t ev = nullptr;
        bool flag = false;    // counters in slot[0..cNum) once slot[cNum] == seq (mapped host memory)
        u64 seq = 0;
        u64* slot = nullptr;
    } pend[2];
    for (int k = 0; k < 2; ++k) {
        pend[k].h = h_sh + (size_t)k * kCtrBlock;
        pend[k].ev = g->pend_ev[k];
    }
    int npend = 0;
    bool stop = false;
    u64* cur_lvl = bt.lvl[0];
    u64* cur_fa = bt.fa[0];
    const bool pipe_ok = sparse_ok && !ex && MODE != kSym && (g->bfs_flags & 512);
    // End-of-level wait: a host spin (the blocking wait adds tens of microseconds per level, and
    // unbounded traversals run tens of short levels).
    auto wait_event = [](hipEvent_t ev) {
        hipError_t e;
        while ((e = hipEventQuery(ev)) == hipErrorNotReady) {
        }
        HGX_HIP(e);
    };
    // One level's counters -> host state; false once the level found no new atom (its rows released).
    auto read_level = [&](Pend& p) -> bool {
        if (p.flag) {   // spin on the sequence word; a stream that finished or failed without it is an error
            for (unsigned spin = 0; __atomic_load_n(p.slot + cNum, __ATOMIC_ACQUIRE) != p.seq; ++spin) {
                if ((spin & 1023u) != 1023u) continue;   // the stream is asked every 1024 polls
                const hipError_t e = hipStreamQuery(s);
                if (e == hipErrorNotReady) continue;
                if (e != hipSuccess) HGX_HIP(e);
                if (__atomic_load_n(p.slot + cNum, __ATOMIC_ACQUIRE) != p.seq)
                    fail(HGX_E_DEVICE, "batched BFS: level counters never arrived");
            }
            for (int k = 0; k < cNum; ++k) h_new[k] = __atomic_load_n(p.slot + k, __ATOMIC_RELAXED);
        } else {
            wait_event(p.ev);
            for (int k = 0; k < cNum; ++k) {
                h_new[k] = 0;
                for (int sh = 0; sh < kCtrShards; ++sh) h_new[k] += p.h[sh * kCtrStride + k];
            }
        }
        if (ex) {   // the group decides termination; the next level's push volume is my frontier's
            h_new[cNewAtoms] = p.new_global;
            h_new[cNewDeg] = p.part_push;
        }
        level_ctr.push_back(std::vector<u64>(h_new, h_new + cNum));
        level_ctr.back()[cDirRows] = (u64)p.kind;   // (host-side) kind of this level
        if (!ex) full_deg_total += (int64_t)(h_new[cNewDeg] - h_new[cNewDegNF]);   // incidence of atoms now full
        if (trace)
            std::fprintf(stderr, "[hgx bfs] level %d kind %d allrows %d active_links %llu new %llu push %llu push_nf %llu "
                         "new_full %llu\n", p.d, p.kind, p.allrows,
                         (unsigned long long)h_new[cActiveLinks], (unsigned long long)h_new[cNewAtoms],
                         (unsigned long long)h_new[cNewDeg], (unsigned long long)h_new[cNewDegNF],
                         (unsigned long long)h_new[cNewFull]);
        push_volume = h_new[cNewDeg];
        push_volume_nf = ex ? push_volume : h_new[cNewDegNF];
        front_atoms = h_new[cNewAtoms];
        full_total += h_new[cNewFull];
        if (h_new[cNewAtoms] == 0) {
            g->release(p.lvl_next, row_bytes);
            g->release(p.fa_next, bm_bytes);
            return false;
        }
        bt.lvl.push_back(p.lvl_next);
        bt.fa.push_back(p.fa_next);
        if (!p.flag) count_now(bt.lvl.size() - 1, p.ev);   // p.ev follows the level's kernels
        return true;
    };

    for (int32_t d = 0; d < maxd && d < max_levels_cap - 1 && !stop; ++d) {
        if ((d + 1) % kZeroLevels == 0) {   // the next kZeroLevels counter blocks / count rows
            ZeroList zl{};
            const int64_t b0 = d + 1, b1 = std::min<int64_t>(b0 + kZeroLevels, max_levels_cap - 1);
            zl.add(ctr + (size_t)b0 * kCtrBlock, sizeof(u64) * kCtrBlock * (size_t)(b1 - b0));
            if (bt.pcnt && b0 < kDirectLevels)
                zl.add(bt.pcnt + (size_t)b0 * 1024, sizeof(u64) * 1024 * (size_t)(std::min<int64_t>(b1, kDirectLevels) - b0));
            zl.launch(s);
        }
        u64* lvl = cur_lvl;
        u64* fa = cur_fa;
        const bool scratch_zero = scratch_clean;   // first level: n_fl / n_cl still zero from the prologue
        scratch_clean = false;
        bool flag_level = false;   // counters written by the finalise into mapped host memory
        u64 flag_seq = 0;
        u64* flag_slot = nullptr;
        const bool spec = npend > 0;   // issued before the previous level's counters were read
        u64* lvl_next = (u64*)g->alloc(row_bytes);
        u64* fa_next = (u64*)g->alloc(bm_bytes);   // every word written by hgx_atom_pull
        u64* c = ctr + (size_t)d * kCtrBlock;
        const bool sparse = spec || (sparse_ok && push_volume < sparse_limit);
        int lflags = g->bfs_flags;
        if ((lflags & 16) && (int64_t)full_total * 16 < A) lflags &= ~4;   // adaptive full skip
        const bool opush = sparse && (MODE != kSym || (lflags & 32));
        // late dense level with few atoms left unfull: those pull from the frontier directly
        const bool nfp = !sparse && sparse_ok && MODE == kSym && Lay<W>::G >= 4 && !ex && (lflags & 256) &&
                         (lflags & 4) && 4 * (int64_t)(I_total - full_deg_total) < I_total;
        // dense level over a frontier whose rows fit the Infinity Cache: the frontier-code pull (bit 17)
        const int4* fcrec = nullptr;
        if (!nfp && !sparse && MODE == kSym && Lay<W>::G >= 4 && !ex && (lflags & kFc) &&
            (double)front_atoms * W * 8.0 <= kFcFrontBytes)
            fcrec = fc_records(g, s);
        const bool fcp = fcrec != nullptr;
        if (!opush) {   // the lists are reused as scratch; the sparse gather leaves candidate bits set
            chained = false;
            if (sparse) cand_clean = false;
        }
        if (fcp) {
            if constexpr (Lay<W>::G >= 4 && MODE == kSym) {
                const int64_t nwords = ceil_div(A, 64);
                const int64_t cap = std::max<int64_t>((int64_t)front_atoms, 1);
                const size_t fw_bytes = sizeof(u64x2) * (size_t)std::max<int64_t>(nwords, 1);
                const size_t drow_bytes = sizeof(u64) * (size_t)kFcDenseCap * W;
                u64x2* fwd = (u64x2*)g->alloc(fw_bytes);
                u64* fcode = (u64*)g->alloc(sizeof(u64) * (size_t)cap);
                u64* drow = (u64*)g->alloc(drow_bytes);
                const hgx_graph* root = g->base ? g->base : g;
                const int32_t n_hubs = root->fc_nhubs;
                u64* hubtab = (u64*)g->alloc(sizeof(u64) * (size_t)std::max<int32_t>(n_hubs, 1));
                u64* n_slots = ctr + (size_t)(max_levels_cap - 1) * kCtrBlock + 8;   // scratch slots
                unsigned int* n_dense = (unsigned int*)(n_slots + 1);
                Events e1 = tm.start(kKindFc, d);
                HGX_HIP(hipMemsetAsync(n_slots, 0, 2 * sizeof(u64), s));
                hgx_fc_slots<<<grid_for(nwords, 256, 2048), 256, 0, s>>>(nwords, fa, fwd, n_slots);
                HGX_CHECK_LAUNCH();
                hgx_fc_codes<W><<<grid_for(A, 256, 8192), 256, 0, s>>>(A, fwd, lvl, fcode, cap, drow, n_dense, c);
                HGX_CHECK_LAUNCH();
                if (n_hubs > 0) {
                    hgx_fc_hubs<<<grid_for(n_hubs, 256, 64), 256, 0, s>>>(n_hubs, root->fc_hubs, fwd, fcode, hubtab);
                    HGX_CHECK_LAUNCH();
                }
                hgx_fc_pull<W><<<grid_for(ceil_div(A, kFcTile) * 256, 256, 4096), 256, 0, s>>>(
                    A, g->inc_off, fcrec, g->inc_type, want_type, fwd, fcode, drow, hubtab, n_hubs, lvl, vis, ever,
                    full, lvl_next, fa_next, c, fm, lflags);
                HGX_CHECK_LAUNCH();
                tm.stop(e1);
                if (g->n_chunks > 0) {
                    Events e3 = tm.start(kKindFcHeavy, d);
                    hgx_fc_pull_heavy<W><<<(unsigned)g->n_chunks, 256, 0, s>>>(g->chunks, fcrec, g->inc_type, want_type,
                                                                             fwd, fcode, drow, hubtab, n_hubs, lvl,
                                                                             vis, ever, full, hubacc, c, fm, lflags);
                    HGX_CHECK_LAUNCH();
                    tm.stop(e3);
                    Events e4 = tm.start(kKindHub, d);
                    hgx_hub_finalize<W><<<hub_grid, block, 0, s>>>(g->n_heavy, g->heavy_atom, g->inc_off, hubacc, vis,
                                                                   ever, full, lvl_next, fa_next, c, fm);
                    HGX_CHECK_LAUNCH();
                    tm.stop(e4);
                }
                g->release(fwd, fw_bytes);   // stream-ordered reuse
                g->release(fcode, sizeof(u64) * (size_t)cap);
                g->release(drow, drow_bytes);
                g->release(hubtab, sizeof(u64) * (size_t)std::max<int32_t>(n_hubs, 1));
            }
        } else if (nfp) {
            if constexpr (Lay<W>::G >= 4 && MODE == kSym) {
                Events e2 = tm.start(kKindNf, d);
                HGX_HIP(hipMemsetAsync(fa_next, 0, bm_bytes, s));
                u64* n_list = ctr + (size_t)(max_levels_cap - 1) * kCtrBlock + 8;   // scratch slot
                HGX_HIP(hipMemsetAsync(n_list, 0, sizeof(u64), s));
                if (!g->hasinc) {   // once per snapshot
                    HGX_HIP(hipMalloc(&g->hasinc, sizeof(u64) * (size_t)(ceil_div(A, 64) + 1)));
                    hgx_hasinc<<<grid_for(ceil_div(A, 64) * 64, 256, 4096), 256, 0, s>>>(A, g->inc_off, (u64*)g->hasinc);
                    HGX_CHECK_LAUNCH();
                }
                const u64* hasinc = (const u64*)g->hasinc;
                hgx_nonfull_list<<<grid_for(ceil_div(A, 64), 256, 2048), 256, 0, s>>>(A, full, hasinc, clist, n_list);
                HGX_CHECK_LAUNCH();
                hgx_nf_pull<W><<<4096, 256, 0, s>>>(clist, n_list, g->inc_off, g->inc_row, g->inc_type, want_type,
                                                    g->tgt_off, g->tgt_idx, fa, lvl, vis, ever, full, lvl_next, fa_next,
                                                    c, fm, lflags);
                HGX_CHECK_LAUNCH();
                tm.stop(e2);
            }
        } else if (opush) {
            // frontier-driven push (mark candidates, zero their rows, OR rows, finalise): the ordered
            // modes always, the symmetric mode with HGX_OPT_BFS_FLAGS bit 5
            const bool pre_work = !g->zacc_clean || g->zacc_bytes < row_bytes || (MODE != kSym && !g->inc_yf) ||
                                  g->n_pchunks < 0 || !cand_clean || !chained;
            if (pre_work) tm.break_chain();
            if (!g->zacc_clean || g->zacc_bytes < row_bytes) {   // (re)establish the all-zero accumulator
                if (g->zacc_bytes < row_bytes) {
                    if (g->zacc) HGX_HIP(hipFree(g->zacc));
                    g->zacc = nullptr;
                    g->zacc_bytes = 0;
                    HGX_HIP(hipMalloc(&g->zacc, row_bytes));
                    g->zacc_bytes = row_bytes;
                }
                HGX_HIP(hipMemsetAsync(g->zacc, 0, g->zacc_bytes, s));
            }
            g->zacc_clean = false;   // until this level's finalise has run
            u64* acc = (u64*)g->zacc;
            if (MODE != kSym && !g->inc_yf) {   // once per snapshot
                HGX_HIP(hipMalloc(&g->inc_yf, (size_t)g->I + 64));
                hgx_inc_yield<<<grid_for(A * 64, 256, 8192), 256, 0, s>>>(A, g->inc_off, g->inc_row, g->tgt_off,
                                                                       g->tgt_idx, g->inc_yf);
                HGX_CHECK_LAUNCH();
            }
            const uint8_t* yf = g->inc_yf;
            if (g->n_pchunks < 0) build_push_chunks(g);
            // chained levels need no memset: the candidate words are zero-invariant, fa_next is cleared by
            // hgx_opush and n_cl by the previous finalise
            if (!cand_clean) HGX_HIP(hipMemsetAsync(cand, 0, bm_bytes, s));
            if (!chained) {   // the frontier list from the bitmap (else the last finalise left it in fl)
                if (!scratch_zero) {
                    HGX_HIP(hipMemsetAsync(n_cl, 0, sizeof(u64), s));
                    HGX_HIP(hipMemsetAsync(n_fl, 0, sizeof(u64), s));
                }
                const int fgrid = grid_for(ceil_div(A, 64), 256, 256);   // <= 256 list atomics per level
                hgx_frontier_list<<<fgrid, 256, 0, s>>>(A, fa, g->inc_off, fl, n_fl, kPushLight);
                HGX_CHECK_LAUNCH();
            }
            // 2048 waves grid-striding over the frontier list: config 5 levels of 20 to 35K atoms measured
            // 19-113 us against 30-142 us with 8192 waves (the launch of mostly idle workgroups and
            // the candidate-append contention) and 20-171 us with 1024 waves
            static const int kPushGrid = [] {   // HGX_PUSH_GRID (A/B builds): override of the push grid (blocks)
                const char* e = ab_env("HGX_PUSH_GRID");
                const int v = e ? std::atoi(e) : 0;
                return v >= 64 && v <= 8192 ? v : 512;
            }();
            const int lgrid = kPushGrid;
            Events e2 = tm.start_chained(kKindPush, d);
            // hub chunks inside hgx_opush while there are few of them (config 5: ~350 chunks, one launch
            // less per level); a block per chunk in hgx_opush_heavy when there are many (config 2:
            // ~380K chunks of 26K hubs: folded into 512 blocks the seed level took 0.58 ms against 0.41)
            const bool fold = g->n_pchunks <= 8 * lgrid;
            // hub chunks in the same launch when folded
            hgx_opush<W, MODE><<<lgrid, 256, 0, s>>>(fl, n_fl, g->inc_off, g->inc_row, g->inc_type, want_type, yf,
                                                         g->tgt_off, g->tgt_idx, lvl, full, cand, cl, n_cl, acc, c,
                                                         fa_next, (int64_t)(bm_bytes / sizeof(u64)), g->pchunks,
                                                         fold ? g->n_pchunks : 0, fa);
            HGX_CHECK_LAUNCH();
            if (!fold && g->n_pchunks > 0) {
                hgx_opush_heavy<W, MODE><<<(unsigned)g->n_pchunks, 256, 0, s>>>(
                    g->pchunks, fa, g->inc_row, g->inc_type, want_type, yf, g->tgt_off, g->tgt_idx, lvl, full, cand,
                    cl, n_cl, acc, c);
                HGX_CHECK_LAUNCH();
            }
            // finalise; re-zeroes the accumulator rows and candidate words it consumed and, without a
            // ghost exchange, rewrites the candidate list into the next level's frontier list
            // without an exchange the level's counters go straight to mapped host memory (no copy in the
            // stream between this level and the next)
            if (!ex) {
                flag_level = true;
                flag_seq = ++g->ctr_seq;
                flag_slot = g->ctr_host + (size_t)(d & 1) * kHostSlot;
                __atomic_store_n(flag_slot + cNum, (u64)0, __ATOMIC_RELEASE);
            }
            u64* lcount = nullptr;   // the new level's counts accumulated by the finalise (no exchange)
            if (!ex && bt.pcnt && d + 1 < kDirectLevels) {
                lcount = bt.pcnt + (size_t)(d + 1) * 1024;
                bt.direct[d + 1] = 1;
            }
            hgx_push_finalize_list<W><<<512, 256, 0, s>>>(cl, n_cl, g->inc_off, acc, cand, vis, ever, full,
                                                           lvl_next, fa_next, c, fm, ex ? 0 : 1, ex ? nullptr : n_fl,
                                                           ticket, flag_level ? flag_slot : nullptr, flag_seq, lcount);
            HGX_CHECK_LAUNCH();
            g->zacc_clean = true;   // every accumulated row is in the candidate list and re-zeroed
            cand_clean = true;
            chained = !ex;
            std::swap(fl, cl);
            std::swap(n_fl, n_cl);
            tm.stop_chained(e2);
        } else {
        if (sparse) {
            Events e0 = tm.start(kKindGather, d);
            HGX_HIP(hipMemsetAsync(lcand, 0, la_bytes, s));
            HGX_HIP(hipMemsetAsync(cand, 0, bm_bytes, s));
            hgx_frontier_links<<<grid_for(ceil_div(A, 64) * 64, 256, 4096), 256, 0, s>>>(
                A, fa, g->inc_off, g->inc_row, g->link_type, want_type, lcand);
            HGX_CHECK_LAUNCH();
            if (g->n_chunks > 0) {
                hgx_frontier_links_heavy<<<(unsigned)g->n_chunks, 256, 0, s>>>(g->chunks, fa, g->inc_row,
                                                                             g->link_type, want_type, lcand);
                HGX_CHECK_LAUNCH();
            }
            tm.stop(e0);
        }
        u64* lc = sparse ? lcand : nullptr;
        u64* cd = sparse ? cand : nullptr;

        const bool v2 = Lay<W>::G >= 4 && !sparse && !(lflags & 64);   // MLP-restructured dense kernels
        // A frontier whose incidence volume covers the links twice leaves few links inactive: the
        // gather then writes a (zero) row for every link and the pull reads rows without probing la
        // -- one dependent load fewer per incidence chunk (HGX_OPT_BFS_FLAGS bit 7).
        if (v2 && (lflags & 128) && MODE == kSym && push_volume_nf >= 2 * (u64)M) lflags |= kAllRows;
        Events e1 = tm.start(kKindGather, d);
        if constexpr (Lay<W>::G >= 4) {
            if (v2)
            {
                if (lflags & kGatherO5)   // diagnostic A/B (bit 10)
                    hgx_link_gather2_o5<W, MODE == kSym><<<gather_grid, block, 0, s>>>(
                        M, g->tgt_off, g->tgt_idx, g->link_type, want_type, fa, full, lvl, lf, la, c, fm, lflags);
                else
                    hgx_link_gather2<W, MODE == kSym><<<gather_grid, block, 0, s>>>(
                        M, g->tgt_off, g->tgt_idx, g->link_type, want_type, fa, full, lvl, lf, la, c, fm, lflags);
            }
        }
        if (!v2)
            hgx_link_gather<W, MODE == kSym><<<gather_grid, block, 0, s>>>(M, g->tgt_off, g->tgt_idx, g->link_type,
                                                                          want_type, fa, full, lvl, lf, la, c, fm,
                                                                          lflags, lc, cd);
        HGX_CHECK_LAUNCH();
        tm.stop(e1);
        if (sparse && MODE == kSym) {
            // push direction: candidates are few, hubs must not be re-scanned
            Events e2 = tm.start(kKindPull, d);
            hgx_push_zero<<<grid_for(ceil_div(A, 64) * 64, 256, 4096), 256, 0, s>>>(A, W, cand, full, lvl_next);
            HGX_CHECK_LAUNCH();
            hgx_push_rows<<<grid_for(ceil_div(M, 64) * 64, 256, 4096), 256, 0, s>>>(M, W, la, g->tgt_off, g->tgt_idx,
                                                                                 lf, full, lvl_next);
            HGX_CHECK_LAUNCH();
            hgx_push_finalize<W><<<pull_grid, block, 0, s>>>(A, g->inc_off, cand, vis, ever, full, lvl_next, fa_next,
                                                             c, fm);
            HGX_CHECK_LAUNCH();
            tm.stop(e2);
        } else {
        Events e2 = tm.start(kKindPull, d);
        if constexpr (Lay<W>::G >= 4 && MODE == kSym) {
            if (v2)
            {
                // two atoms of a group interleaved (152 VGPRs, 3 waves/SIMD): config 2 pull 5.73 -> 5.23 ms
                // a step against four (184 VGPRs, 2 waves/SIMD, dropped in r02); a tile's atoms placed in
                // descending degree order (5.20 -> 5.13 ms, profiles/r02r_ab_pull_sort.log).  Bit 11 (A/B):
                // half of a group's rows in flight at once (fewer VGPRs, more waves per SIMD).
                if (lflags & 2048)
                    hgx_atom_pull2<W, 2, true, Lay<W>::G / 2><<<pull_grid, block, 0, s>>>(
                        A, g->inc_off, g->inc_row, la, lf, vis, ever, full, lvl_next, fa_next, c, fm, lflags, own_bm);
                else
                    hgx_atom_pull2<W, 2, true, Lay<W>::G><<<pull_grid, block, 0, s>>>(
                        A, g->inc_off, g->inc_row, la, lf, vis, ever, full, lvl_next, fa_next, c, fm, lflags, own_bm);
            }
        }
        if (!(v2 && MODE == kSym))
            hgx_atom_pull<W, MODE><<<pull_grid, block, 0, s>>>(A, g->inc_off, g->inc_row, la, lf, g->tgt_off,
                                                               g->tgt_idx, fa, lvl, vis, ever, full, lvl_next,
                                                               fa_next, c, fm, lflags, cd);
        HGX_CHECK_LAUNCH();
        tm.stop(e2);
        if (g->n_chunks > 0) {
            Events e3 = tm.start(kKindHeavy, d);
            hgx_atom_pull_heavy<W, MODE><<<(unsigned)g->n_chunks, block, 0, s>>>(
                    g->chunks, g->inc_row, la, lf, g->tgt_off, g->tgt_idx, fa, lvl, vis, ever, full, hubacc, c, fm,
                    lflags, cd);
            HGX_CHECK_LAUNCH();
            tm.stop(e3);
            Events e4 = tm.start(kKindHub, d);
            hgx_hub_finalize<W><<<hub_grid, block, 0, s>>>(g->n_heavy, g->heavy_atom, g->inc_off, hubacc, vis, ever,
                                                           full, lvl_next, fa_next, c, fm);
            HGX_CHECK_LAUNCH();
            tm.stop(e4);
        }
        }
        }   // not an ordered push level
        u64 new_global = 0, part_push = 0;
        if (ex) {
            double lb = 0, pm = 0;
            new_global = ex->template level<W>(lvl_next, fa_next, vis, ever, full, fm, &part_push, &lb, &pm, tm, d,
                                               d + 1 >= maxd);
            if (d < 64) {
                res->stats.level_xbytes[d] += lb;
                res->stats.level_xpair_max[d] = std::max(res->stats.level_xpair_max[d], pm);
                res->stats.level_xtrips[d] = std::max(res->stats.level_xtrips[d], (int32_t)ex->trips);
            }
        }
        Pend& pn = pend[d & 1];
        pn.d = d;
        pn.lvl_next = lvl_next;
        pn.fa_next = fa_next;
        pn.kind = fcp ? 4 : nfp ? 3 : sparse ? (opush ? 2 : 1) : 0;
        pn.allrows = (lflags & kAllRows) ? 1 : 0;
        pn.new_global = new_global;
        pn.part_push = part_push;
        pn.flag = flag_level;
        pn.seq = flag_seq;
        pn.slot = flag_slot;
        if (!flag_level) {
            tm.break_chain();
            HGX_HIP(hipMemcpyAsync(pn.h, c, sizeof(u64) * kCtrBlock, hipMemcpyDeviceToHost, s));
            HGX_HIP(hipEventRecord(pn.ev, s));
        }
        ++npend;
        cur_lvl = lvl_next;
        cur_fa = fa_next;
        // Pipelined push levels: while this level runs, the next one is issued as a push level when this
        // level ran on a frontier below the sparse limit (a push is exact on any frontier, so a wrong
        // guess only costs speed); an empty frontier costs it three near-empty launches, so the
        // counters are read one level late.
        for (;;) {
            const bool can_spec = pipe_ok && npend == 1 && opush && push_volume < sparse_limit && d + 1 < maxd &&
                                  d + 1 < max_levels_cap - 1;
            if (npend == 0 || can_spec) break;
            Pend& p = pend[(d - npend + 1) & 1];   // the oldest unread level
            --npend;
            if (!read_level(p)) {
                stop = true;
                for (; npend > 0; --npend) {   // a level issued after the last frontier: its rows are empty
                    Pend& q = pend[(d - npend + 1) & 1];
                    if (q.flag) spin_sync(s);
                    else wait_event(q.ev);
                    g->release(q.lvl_next, row_bytes);
                    g->release(q.fa_next, bm_bytes);
                }
                break;
            }
        }
    }
    if (ex) {
        res->stats.bytes_exchanged += ex->bytes_sent;
        res->stats.xwords_nonzero += ex->nz_words;
        res->stats.xwords_total += ex->words;
    }
    g->release(vis, row_bytes);
    if (lf) g->release(lf, sizeof(u64) * (size_t)std::max<int64_t>(M, 1) * W);
    g->release(hubacc, sizeof(u64) * (size_t)std::max<int64_t>(g->n_heavy, 1) * W);
    g->release(ever, bm_bytes);
    g->release(full, bm_bytes);
    g->release(la, la_bytes);
    if (lcand) g->release(lcand, la_bytes);
    if (cand) g->release(cand, bm_bytes);
    if (flist) g->release(flist, flist_bytes);
    if (clist) g->release(clist, flist_bytes);
    g->release(ctr, sizeof(u64) * kCtrBlock * max_levels_cap);
    g->release(d_atoms, sizeof(int32_t) * seed_atoms.size());
    g->release(d_rows, sizeof(u64) * seed_rows.size());
}

template <int W>
void run_mode(int mode, hgx_graph* g, hgx_bfs_result* res, BfsBatch& bt, int32_t max_depth, int32_t want_type,
              const std::vector<int32_t>& sa, const std::vector<u64>& sr, Timer& tm,
              std::vector<std::vector<u64>>& lc, Transport* tr) {
    switch (mode) {
        case kSym: run_levels<W, kSym>(g, res, bt, max_depth, want_type, sa, sr, tm, lc, tr); break;
        case kAfterFirst: run_levels<W, kAfterFirst>(g, res, bt, max_depth, want_type, sa, sr, tm, lc, tr); break;
        case kBeforeFirst: run_levels<W, kBeforeFirst>(g, res, bt, max_depth, want_type, sa, sr, tm, lc, tr); break;
        case kBeforeLast: run_levels<W, kBeforeLast>(g, res, bt, max_depth, want_type, sa, sr, tm, lc, tr); break;
        default: run_levels<W, kAfterLast>(g, res, bt, max_depth, want_type, sa, sr, tm, lc, tr); break;
    }
}

int words_for(int S) {
    int w = (S + 63) / 64;
    int W = 1;
    while (W < w) W <<= 1;
    return W;
}

template <int W>
void count_level(hgx_graph* g, const u64* fa, const u64* lvl, u64* counts, u64* trav) {
    const int per_block = 256 / W;
    int64_t blocks = ceil_div(g->A, per_block);
    int grid = (int)std::min<int64_t>(blocks, 8192);   // keeps atoms per thread < 2^22
    hgx_level_count<W><<<std::max(grid, 1), 256, 0, g->stream>>>(g->A, fa, lvl, g->inc_off, counts, trav);
    HGX_CHECK_LAUNCH();
}

void count_level_dispatch(int W, hgx_graph* g, const u64* fa, const u64* lvl, u64* counts, u64* trav) {
    switch (W) {
        case 1: count_level<1>(g, fa, lvl, counts, trav); break;
        case 2: count_level<2>(g, fa, lvl, counts, trav); break;
        case 4: count_level<4>(g, fa, lvl, counts, trav); break;
        case 8: count_level<8>(g, fa, lvl, counts, trav); break;
        default: count_level<16>(g, fa, lvl, counts, trav); break;
    }
}



// The result readout: res->counts (per seed, per depth) from the device rows -- one counting launch
// per level (block partials), one reduce launch, one D2H, one synchronisation (first call only).
void ensure_counts(hgx_bfs_result* r) {
    if (r->counts_ready) return;
    hgx_graph* g = r->g;
    HGX_HIP(hipSetDevice(g->device));
    r->counts.assign((size_t)r->n_seeds * r->n_levels, 0);
    if (r->blk) {   // the workgroup engine's seeds: V_0 = {seed}, then the level counts it wrote
        const BlockSet& b = *r->blk;
        for (int32_t i = 0; i < r->n_seeds; ++i) {
            if (b.pairs[i] < 0) continue;
            int64_t* c = &r->counts[(size_t)i * r->n_levels];
            c[0] = 1;
            for (int32_t d = 0; d < b.levels[i]; ++d) c[d + 1] = b.lcnt[i][d];
        }
        if (r->batches.empty()) {
            r->counts_ready = true;
            return;
        }
    }
    // Traversals made of push levels (config 5's closures): every level past the seeds was counted by
    // its push finalise, and level 0 of a whole-graph batch is {seed} (count 1 each) -- the readout is
    // one copy of the count rows, no counting pass and no reduce launch.
    bool all_direct = !g->shard;
    size_t rows = 0;
    for (auto& bt : r->batches) {
        all_direct = all_direct && bt.cpart.empty() && bt.pcnt;
        for (size_t d = 1; all_direct && d < bt.lvl.size(); ++d) all_direct = d < bt.direct.size() && bt.direct[d];
        rows += bt.lvl.empty() ? 0 : bt.lvl.size() - 1;
    }
    if (all_direct) {
        u64* hc = (u64*)g->pinned_buf(sizeof(u64) * 1024 * std::max<size_t>(rows, 1));
        size_t o = 0;
        for (auto& bt : r->batches) {
            const size_t nl = bt.lvl.size();
            if (nl > 1)
                HGX_HIP(hipMemcpyAsync(hc + o * 1024, bt.pcnt + 1024, sizeof(u64) * 1024 * (nl - 1), hipMemcpyDeviceToHost,
                                       g->stream));
            o += nl > 0 ? nl - 1 : 0;
        }
        spin_sync(g->stream);
        o = 0;
        for (auto& bt : r->batches) {
            const size_t nl = bt.lvl.size();
            for (int s = 0; s < bt.S; ++s) {
                int64_t* c = &r->counts[(size_t)r->orig_of(bt.seed0 + s) * r->n_levels];
                if (nl > 0) c[0] = 1;   // V_0 = {seed}
                for (size_t d = 1; d < nl; ++d) c[d] = (int64_t)hc[(o + d - 1) * 1024 + s];
            }
            o += nl > 0 ? nl - 1 : 0;
        }
        r->counts_ready = true;
        return;
    }
    size_t nslots = 0;
    for (auto& bt : r->batches) nslots += bt.lvl.size();
    const int grid = count_grid(g->A);
    std::vector<int32_t> meta(2 * std::max<size_t>(nslots, 1), 0);   // [nblk | width]
    std::vector<int64_t> poff(std::max<size_t>(nslots, 1), 0);
    std::vector<const u64*> fap(std::max<size_t>(nslots, 1), nullptr), lvp(std::max<size_t>(nslots, 1), nullptr),
        dirp(std::max<size_t>(nslots, 1), nullptr);
    int64_t ptot = 0;
    bool any_early = false;
    std::vector<const uint32_t*> early_p(std::max<size_t>(nslots, 1), nullptr), partp(std::max<size_t>(nslots, 1), nullptr);
    {
        size_t k = 0;
        for (auto& bt : r->batches)
            for (size_t d = 0; d < bt.lvl.size(); ++d, ++k) {
                const bool dir = d < bt.direct.size() && bt.direct[d];   // counted by the push finalise
                const bool early = d < bt.cpart.size() && bt.cpart[d];   // counted next to the traversal
                any_early |= early;
                meta[k] = dir ? 0 : early ? bt.cgrid : grid;
                meta[nslots + k] = bt.W * 64;
                poff[k] = ptot;
                fap[k] = (dir || early) ? nullptr : bt.fa[d];
                lvp[k] = bt.lvl[d];
                dirp[k] = dir ? bt.pcnt + d * 1024 : nullptr;
                early_p[k] = early ? bt.cpart[d] : nullptr;
                if (!dir && !early) ptot += (int64_t)grid * bt.W * 64;
            }
    }
    const size_t bytes = sizeof(u64) * 1024 * std::max<size_t>(nslots, 1);
    const size_t pbytes = sizeof(uint32_t) * (size_t)std::max<int64_t>(ptot, 1);
    const size_t o_poff = (sizeof(int32_t) * meta.size() + 15) & ~(size_t)15;
    const size_t o_fap = o_poff + sizeof(int64_t) * poff.size();
    const size_t o_lvp = o_fap + sizeof(u64*) * fap.size();
    const size_t o_dir = o_lvp + sizeof(u64*) * lvp.size();
    const size_t o_pp = o_dir + sizeof(u64*) * dirp.size();
    const size_t mbytes = o_pp + sizeof(uint32_t*) * partp.size();
    u64* dc = (u64*)g->alloc(bytes);
    uint32_t* dp = (uint32_t*)g->alloc(pbytes);
    for (size_t k = 0; k < nslots; ++k) partp[k] = early_p[k] ? early_p[k] : dp + poff[k];
    char* dm = (char*)g->alloc(mbytes);
    // one pinned region: the launch metadata going up, the counts coming back (a copy into pageable
    // memory is staged through a bounce buffer)
    const size_t o_back = (mbytes + 255) & ~(size_t)255;
    char* hm = (char*)g->pinned_buf(o_back + bytes);
    std::memcpy(hm, meta.data(), sizeof(int32_t) * meta.size());
    std::memcpy(hm + o_poff, poff.data(), sizeof(int64_t) * poff.size());
    std::memcpy(hm + o_fap, fap.data(), sizeof(u64*) * fap.size());
    std::memcpy(hm + o_lvp, lvp.data(), sizeof(u64*) * lvp.size());
    std::memcpy(hm + o_dir, dirp.data(), sizeof(u64*) * dirp.size());
    std::memcpy(hm + o_pp, partp.data(), sizeof(uint32_t*) * partp.size());
    HGX_HIP(hipMemcpyAsync(dm, hm, mbytes, hipMemcpyHostToDevice, g->stream));
    const u64* own = g->shard ? (const u64*)g->shard->own_bm : nullptr;
    size_t k = 0;
    for (auto& bt : r->batches) {   // one launch per batch: blockIdx.y = its level slots
        const int nl = (int)bt.lvl.size();
        if (nl > 0) {
            const dim3 gr((unsigned)grid, (unsigned)nl);
            const u64* const* fa_d = (const u64* const*)(dm + o_fap);
            const u64* const* lv_d = (const u64* const*)(dm + o_lvp);
            const int64_t* po_d = (const int64_t*)(dm + o_poff);
            hipStream_t s = g->stream;
            switch (bt.W) {
                case 1: hgx_count_rows_multi<1><<<gr, 256, 0, s>>>(g->A, fa_d, own, lv_d, po_d, (int)k, dp); break;
                case 2: hgx_count_rows_multi<2><<<gr, 256, 0, s>>>(g->A, fa_d, own, lv_d, po_d, (int)k, dp); break;
                case 4: hgx_count_rows_multi<4><<<gr, 256, 0, s>>>(g->A, fa_d, own, lv_d, po_d, (int)k, dp); break;
                case 8: hgx_count_rows_multi<8><<<gr, 256, 0, s>>>(g->A, fa_d, own, lv_d, po_d, (int)k, dp); break;
                default: hgx_count_rows_multi<16><<<gr, 256, 0, s>>>(g->A, fa_d, own, lv_d, po_d, (int)k, dp); break;
            }
            HGX_CHECK_LAUNCH();
        }
        k += (size_t)nl;
    }
    HGX_HIP(hipMemsetAsync(dc, 0, bytes, g->stream));
    if (any_early) {   // the passes already launched on stream2 come first
        HGX_HIP(hipEventRecord(g->ev_count, g->stream2));
        HGX_HIP(hipStreamWaitEvent(g->stream, g->ev_count, 0));
    }
    if (nslots) {
        hgx_count_reduce<<<(unsigned)ceil_div((int64_t)nslots * 1024 * (kCountBlocks / kReduceSpan), 256), 256, 0,
                           g->stream>>>(
            (int)nslots, (const int32_t*)dm, (const int32_t*)dm + nslots, (const uint32_t* const*)(dm + o_pp),
            (const u64* const*)(dm + o_dir), dc);
        HGX_CHECK_LAUNCH();
    }
    const u64* hc = (const u64*)(hm + o_back);
    HGX_HIP(hipMemcpyAsync(hm + o_back, dc, bytes, hipMemcpyDeviceToHost, g->stream));
    spin_sync(g->stream);
    g->release(dc, bytes);
    g->release(dp, pbytes);
    g->release(dm, mbytes);
    for (auto& bt : r->batches) {   // stream2's passes were ordered before the synchronised reduce
        for (auto& p : bt.cpart)
            if (p) g->release(p, bt.cpart_bytes);
        bt.cpart.clear();
    }
    k = 0;
    for (auto& bt : r->batches)
        for (size_t d = 0; d < bt.lvl.size(); ++d, ++k)
            for (int s = 0; s < bt.S; ++s)
                r->counts[(size_t)r->orig_of(bt.seed0 + s) * r->n_levels + d] = (int64_t)hc[k * 1024 + s];
    for (auto& kv : r->isolated) r->counts[(size_t)kv.first * r->n_levels] += 1;
    r->counts_ready = true;
}

// The TEPS numerator, the survey-model bytes, |U_d| and the minimum-bytes model (first call only;
// reads every level and scans the links once per level -- not part of a timed step).
void ensure_accounting(hgx_bfs_result* r) {
    if (r->accounting_ready) return;
    ensure_counts(r);
    hgx_graph* g = r->g;
    HGX_HIP(hipSetDevice(g->device));
    double trav_total = 0;
    u64* dc = (u64*)g->alloc(sizeof(u64) * (1024 + 1));
    std::vector<u64> hc(1025);
    const double typed = r->typed ? 1.0 : 0.0;
    const double dense_min = 8.0 * (g->A + 1) + 4.0 * g->I + 8.0 * (g->M + 1) + 4.0 * g->P;
    for (auto& bt : r->batches) {
        int nl = (int)bt.lvl.size();
        const double mask = (double)((bt.S + 7) / 8);
        std::vector<double> U(nl + 1, 0.0);
        for (int d = 0; d < nl; ++d) {
            HGX_HIP(hipMemsetAsync(dc, 0, sizeof(u64) * 1025, g->stream));
            count_level_dispatch(bt.W, g, bt.fa[d], bt.lvl[d], dc, dc + 1024);
            HGX_HIP(hipMemcpyAsync(hc.data(), dc, sizeof(u64) * 1025, hipMemcpyDeviceToHost, g->stream));
            HGX_HIP(hipStreamSynchronize(g->stream));
            HGX_HIP(hipMemsetAsync(dc, 0, sizeof(u64) * 4, g->stream));
            hgx_level_survey<<<grid_for(std::max(g->A, g->M), 256, 8192), 256, 0, g->stream>>>(
                g->A, g->M, bt.fa[d], g->tgt_off, g->tgt_idx, dc);
            HGX_CHECK_LAUNCH();
            u64 sv[3];
            HGX_HIP(hipMemcpyAsync(sv, dc, sizeof(sv), hipMemcpyDeviceToHost, g->stream));
            HGX_HIP(hipStreamSynchronize(g->stream));
            U[d] = (double)sv[0];
            if (d < bt.n_expanded) {
                trav_total += (double)hc[1024];
                const double sdeg = (double)sv[1], Pd = (double)sv[2];
                r->stats.bytes_survey += 16.0 * U[d] + 4.0 * sdeg + (16.0 + 4.0 * typed) * sdeg + 4.0 * Pd +
                                         mask * (U[d] + 2.0 * Pd);
                if (d < 64) r->stats.union_frontier[d] += (int64_t)sv[0];
                // minimum bytes of the level: the CSR slices of the frontier (or every column once,
                // whichever is less), one S/8-byte row per frontier atom read and per new atom written
                const double sparse_min = 16.0 * U[d] + 4.0 * sdeg + (16.0 + 4.0 * typed) * sdeg + 4.0 * Pd;
                r->stats.bytes_min += std::min(dense_min, sparse_min) + mask * U[d];
            }
        }
        for (int d = 1; d < nl; ++d)
            if (d <= bt.n_expanded) r->stats.bytes_min += mask * U[d];   // rows of the new atoms written
    }
    g->release(dc, sizeof(u64) * 1025);
    // the workgroup engine's seeds counted their own items (|U_d|, the survey and minimum-bytes
    // models above cover the rows engine's seeds only)
    if (r->blk) trav_total += r->blk->traversed;
    r->stats.traversed_edges = trav_total;
    r->accounting_ready = true;
}

void bfs_batch_impl(hgx_graph* g, Transport* tr, const int32_t* seeds, int32_t n_seeds, int32_t max_depth,
                    const hgx_algen_opts* opts, hgx_bfs_result** out);

}  // namespace

extern "C" {

int hgx_bfs_batch(hgx_graph* g, const int32_t* seeds, int32_t n_seeds, int32_t max_depth,
                  const hgx_algen_opts* opts, hgx_bfs_result** out) {
    HGX_API_BEGIN
    if (!g || !out || n_seeds < 0 || (n_seeds > 0 && !seeds)) fail(HGX_E_INVALID, "hgx_bfs_batch: bad argument");
    *out = nullptr;
    if (g->shard) fail(HGX_E_INVALID, "hgx_bfs_batch: a partition shard needs hgx_pbfs_batch (a transport)");
    for (int32_t i = 0; i < n_seeds; ++i)
        if (seeds[i] < 0 || seeds[i] >= g->A) fail(HGX_E_INVALID, "hgx_bfs_batch: seed out of range");
    if (max_depth < -1) fail(HGX_E_INVALID, "hgx_bfs_batch: bad max_depth");
    bfs_batch_impl(g, nullptr, seeds, n_seeds, max_depth, opts, out);
    HGX_API_END
}

}  // extern "C"

// Partitioned batched BFS: seeds are GLOBAL atom ids; this shard seeds the ones it owns.
void hgx::pbfs_run(hgx_graph* g, Transport* tr, const int32_t* seeds, int32_t n_seeds, int32_t max_depth,
                   const hgx_algen_opts* opts, hgx_bfs_result** out) {
    if (!g->shard) fail(HGX_E_INVALID, "hgx_pbfs_batch: not a partition shard");
    const ShardInfo& sh = *g->shard;
    if (tr->world != sh.n_parts || tr->rank != sh.part)
        fail(HGX_E_INVALID, "hgx_pbfs_batch: transport rank/world does not match the shard's part/n_parts");
    for (int32_t i = 0; i < n_seeds; ++i)
        if (seeds[i] < 0 || seeds[i] >= sh.A_global) fail(HGX_E_INVALID, "hgx_pbfs_batch: seed out of range");
    if (max_depth < -1) fail(HGX_E_INVALID, "hgx_pbfs_batch: bad max_depth");
    // The call is collective: every part must run the same exchange format (each mode issues a
    // different sequence of collectives) on the same seeds, depth and generator.  One all-gather
    // before any exchange; every part sees the same table, so a mismatch fails on all of them.
    {
        hgx_algen_opts o = opts ? *opts : hgx_algen_opts{HGX_NO_TYPE, 1, 1, 0, 0};
        uint64_t h = 1469598103934665603ull;   // FNV-1a over seeds + depth + generator flags
        auto mix = [&](uint64_t v) {
            for (int b = 0; b < 8; ++b) h = (h ^ ((v >> (8 * b)) & 0xff)) * 1099511628211ull;
        };
        for (int32_t i = 0; i < n_seeds; ++i) mix((uint32_t)seeds[i]);
        mix((uint32_t)max_depth);
        mix((uint32_t)o.link_type);
        mix(o.return_preceding | o.return_succeeding << 1 | o.reverse_order << 2 | o.return_source << 3);
        const int NP = sh.n_parts;
        int64_t mine[3] = {sh.xmode, n_seeds, (int64_t)h};
        std::vector<int64_t> all(3 * (size_t)NP);
        HGX_HIP(hipSetDevice(g->device));
        tr->allgather_i64(mine, 3, all.data(), g->stream);
        for (int q = 0; q < NP; ++q) {
            if (all[3 * (size_t)q] != mine[0])
                fail(HGX_E_INVALID, "hgx_pbfs_batch: HGX_OPT_PART_EXCHANGE differs between the parts of the group (part " +
                                        std::to_string(q) + ")");
            if (all[3 * (size_t)q + 1] != mine[1] || all[3 * (size_t)q + 2] != mine[2])
                fail(HGX_E_INVALID, "hgx_pbfs_batch: the parts were called with different seeds, depth or generator (part " +
                                        std::to_string(q) + ")");
        }
    }
    bfs_batch_impl(g, tr, seeds, n_seeds, max_depth, opts, out);
}

namespace {

void bfs_batch_impl(hgx_graph* g, Transport* tr, const int32_t* seeds, int32_t n_seeds, int32_t max_depth,
                    const hgx_algen_opts* opts, hgx_bfs_result** out) {
    hgx_algen_opts o = opts ? *opts : hgx_algen_opts{HGX_NO_TYPE, 1, 1, 0, 0};
    const ShardInfo* shp = g->shard;
    std::lock_guard<std::mutex> lk(g->mu);
    HGX_HIP(hipSetDevice(g->device));
    const int mode = mode_of(o);

    hgx_bfs_result* r = new hgx_bfs_result();
    struct Guard {   // error path: the graph mutex is held here, so release without re-locking
        hgx_bfs_result* r;
        ~Guard() {
            if (!r) return;
            if (r->g->stream2) (void)hipStreamSynchronize(r->g->stream2);   // counting passes read the rows
            for (auto& bt : r->batches) {
                for (auto p : bt.lvl) r->g->release(p, r->row_bytes(bt));
                for (auto p : bt.fa) r->g->release(p, r->bm_bytes());
                if (bt.pcnt) r->g->release(bt.pcnt, sizeof(u64) * 1024 * kDirectLevels);
                for (auto p : bt.cpart)
                    if (p) r->g->release(p, bt.cpart_bytes);
            }
            if (r->blk) block_release(r->g, *r->blk);
            r->g->refs.fetch_sub(1);   // the caller still holds its own reference
            delete r;
        }
    } guard{r};
    r->g = g;
    g->refs.fetch_add(1);
    r->n_seeds = n_seeds;
    r->typed = o.link_type >= 0;

    Timer tm(g);
    if (tm.on) HGX_HIP(hipEventRecord(tm.all.a, g->stream));
    std::vector<std::vector<u64>> level_ctr;
    int max_expanded = 0;
    // Whole-graph batches: every seed first runs in one workgroup (hgx_bfs_block); the rows engine
    // below takes the seeds that outgrew it, compacted.
    std::vector<int32_t> rseeds;
    if (!shp && !tr && g->bfs_block && n_seeds > 0) {
        r->blk.reset(new BlockSet());
        bfs_block(g, seeds, n_seeds, max_depth, o, *r->blk);
        const BlockSet& b = *r->blk;
        max_expanded = b.expanded;
        r->stats.ms_block = b.ms;
        r->stats.bytes_block = b.bytes;
        r->stats.block_seeds = n_seeds - (int64_t)b.rerun.size();
        r->stats.block_rerun = (int64_t)b.rerun.size();
        r->stats.ms_coop = b.co_ms;
        r->stats.bytes_coop = b.co_bytes_alg;
        r->stats.block_coop = b.n_coop;
        r->stats.coop_fallbacks = b.co_fallbacks;
        r->compact.assign((size_t)n_seeds, -1);
        for (size_t k = 0; k < b.rerun.size(); ++k) {
            r->compact[b.rerun[k]] = (int32_t)k;
            r->orig.push_back(b.rerun[k]);
            rseeds.push_back(seeds[b.rerun[k]]);
        }
        seeds = rseeds.data();
        n_seeds = (int32_t)rseeds.size();
    }
    for (int32_t s0 = 0; s0 < n_seeds; s0 += 1024) {
        BfsBatch bt;
        bt.seed0 = s0;
        bt.S = std::min<int32_t>(1024, n_seeds - s0);
        bt.W = words_for(bt.S);
        // unique seed atoms (ascending) and their rows: (atom, source bit) pairs sorted by atom
        std::vector<std::pair<int32_t, int32_t>> at;
        at.reserve((size_t)bt.S);
        for (int32_t i = 0; i < bt.S; ++i) {
            int32_t a = seeds[s0 + i];
            if (shp) {   // every part holding the seed starts from it (its links are spread over them)
                const int32_t l = shp->local_of(a);
                if (l < 0) {   // not here; no incidence anywhere: V_0 = {seed}, recorded by part a % n_parts
                    if (!shp->present(a) && a % shp->n_parts == shp->part) r->isolated[s0 + i] = seeds[s0 + i];
                    continue;
                }
                a = l;
            }
            at.emplace_back(a, i);
        }
        std::sort(at.begin(), at.end());
        std::vector<int32_t> sa;
        std::vector<u64> sr;
        sa.reserve(at.size());
        sr.reserve(at.size() * (size_t)bt.W);
        for (size_t k = 0; k < at.size(); ++k) {
            if (k == 0 || at[k].first != at[k - 1].first) {
                sa.push_back(at[k].first);
                sr.insert(sr.end(), (size_t)bt.W, 0ull);
            }
            sr[(sa.size() - 1) * (size_t)bt.W + (at[k].second >> 6)] |= 1ull << (at[k].second & 63);
        }
        size_t before = level_ctr.size();
        switch (bt.W) {
            case 1: run_mode<1>(mode, g, r, bt, max_depth, o.link_type, sa, sr, tm, level_ctr, tr); break;
            case 2: run_mode<2>(mode, g, r, bt, max_depth, o.link_type, sa, sr, tm, level_ctr, tr); break;
            case 4: run_mode<4>(mode, g, r, bt, max_depth, o.link_type, sa, sr, tm, level_ctr, tr); break;
            case 8: run_mode<8>(mode, g, r, bt, max_depth, o.link_type, sa, sr, tm, level_ctr, tr); break;
            default: run_mode<16>(mode, g, r, bt, max_depth, o.link_type, sa, sr, tm, level_ctr, tr); break;
        }
        // algorithmic bytes of every launch of this batch
        const int64_t A = g->A, M = g->M, P = g->P, I = g->I;
        const double rowb = 8.0 * bt.W;
        const bool typed = o.link_type >= 0;
        const int nexp = (int)(level_ctr.size() - before);
        bt.n_expanded = nexp;
        max_expanded = std::max(max_expanded, nexp);
        const double I_light = (double)(I - g->I_heavy), I_heavy = (double)g->I_heavy;
        for (int d = 0; d < nexp; ++d) {
            const auto& c = level_ctr[before + d];
            // hgx_link_gather: tgt_off + tgt_idx (+ link_type) + frontier/full bitmaps + gathered rows
            //                  + lf writes + la words
            const bool fc_level = c[cDirRows] == 4;   // frontier-code pull (its hub chunks ran)
            const bool sparse_level = c[cDirRows] != 0 && !fc_level;
            const double scan_links = sparse_level ? (double)c[cActiveLinks] : (double)M;
            const double scan_pins = sparse_level ? (double)c[cActivePins] : (double)P;
            double b_gather = 8.0 * (scan_links + 1) + 4.0 * scan_pins + (typed ? 4.0 * scan_links : 0.0) +
                                    A / 4.0 + rowb * c[cActivePins] +
                                    (mode == kSym ? rowb * c[cActiveLinks] : 0.0) + M / 8.0;
            // hgx_atom_pull: inc_off + light inc_row + la bitmap + pulled rows + vis reads + lvl/vis writes
            //                + ever/full/fa_next words (sparse levels: candidate words + pushed rows)
            double b_pull = (sparse_level ? 8.0 * (A / 64.0) : 8.0 * (A + 1) + 4.0 * I_light) + M / 8.0 +
                                  rowb * c[cIncLight] + rowb * c[cVisLight] + 2.0 * rowb * c[cNewLight] +
                                  3.0 * A / 8.0;
            const bool opush_level = c[cDirRows] == 2 || c[cDirRows] == 3;
            if (c[cDirRows] == 3) {   // non-full pull: no gather
                b_gather = 0.0;
                // full bitmap + inc_off of the listed atoms + list write/read + entries (inc_row, inc_type,
                // tgt_off pair) + pins + frontier bitmap + frontier rows + vis reads + lvl/vis writes + bitmaps
                b_pull = A / 8.0 + 24.0 * c[cCand] + 4.0 * A / 64.0 + (8.0 + (typed ? 4.0 : 0.0) + 16.0) * c[cIncLight] +
                         4.0 * c[cActivePins] + A / 8.0 + rowb * c[cNfRows] + rowb * c[cVisLight] +
                         2.0 * rowb * c[cNewLight] + 3.0 * A / 8.0;
            } else if (fc_level) {   // frontier-code pull: no gather, no lf
                b_gather = 0.0;
                // codes: frontier bitmap (twice) + prefixes + the frontier atoms' rows + their codes;
                // pull: inc_off + full bitmap + light records (+ inc_type) + frontier words / prefixes / codes of
                // the frontier targets + dense frontier rows + vis reads + lvl/vis writes + bitmap words
                const double n_front = (double)(d == 0 ? bt.S : level_ctr[before + d - 1][cNewAtoms]);
                const double e_light = (double)c[cIncLight], e_all = e_light + (double)c[cIncHeavy];
                b_pull = 2.0 * A / 8.0 + 4.0 * A / 64.0 + n_front * (rowb + 8.0) +
                         8.0 * (A + 1) + A / 8.0 + e_light * (32.0 + (typed ? 4.0 : 0.0)) +
                         (8.0 + 4.0 + 8.0) * c[cActivePins] * e_light / std::max(e_all, 1.0) +
                         rowb * c[cNfRows] * e_light / std::max(e_all, 1.0) + rowb * c[cVisLight] +
                         2.0 * rowb * c[cNewLight] + 3.0 * A / 8.0;
            } else if (opush_level) {   // frontier push: no gather; two frontier passes + finalise
                b_gather = 0.0;
                // frontier scan + scanned entries (inc_type + yield flag) + links (inc_row, tgt_off pair) + pins
                // + one word RMW per pair + candidates (acc read + re-zero) + vis reads + lvl/vis writes
                // + cleared bitmaps
                b_pull = 8.0 * (A / 64.0) + 5.0 * c[cScanned] + 20.0 * c[cActiveLinks] + 4.0 * c[cActivePins] +
                         16.0 * c[cIncLight] +
                         2.0 * rowb * c[cCand] + rowb * c[cVisLight] + 2.0 * rowb * c[cNewLight] + 2.0 * A / 8.0;
            }
            const int pull_kind = fc_level ? HGX_K_FC_PULL : c[cDirRows] == 3 ? HGX_K_NF_PULL
                                  : c[cDirRows] == 2 ? HGX_K_FRONTIER_PUSH : HGX_K_ATOM_PULL;
            r->stats.bytes_kernel[HGX_K_LINK_GATHER] += b_gather;
            r->stats.bytes_kernel[pull_kind] += b_pull;
            double b_heavy = 0, b_hub = 0;
            if (g->n_chunks > 0 && !sparse_level) {
                if (fc_level) {   // chunk table + the streamed records of the chunks that ran + code lookups
                    const double e_all = (double)c[cIncLight] + (double)c[cIncHeavy];
                    const double share = (double)c[cIncHeavy] / std::max(e_all, 1.0);
                    b_heavy = 24.0 * g->n_chunks + rowb * g->n_chunks +
                              c[cIncHeavy] * (32.0 + (typed ? 4.0 : 0.0)) + 20.0 * c[cActivePins] * share +
                              rowb * c[cNfRows] * share + rowb * g->n_chunks;
                } else {
                    b_heavy = 24.0 * g->n_chunks + 4.0 * I_heavy + rowb * c[cIncHeavy] + rowb * g->n_chunks;
                }
                b_hub = 4.0 * g->n_heavy + 2.0 * rowb * g->n_heavy + rowb * c[cAccHub] + 2.0 * rowb * c[cNewHub];
                const int heavy_kind = fc_level ? HGX_K_FC_HEAVY : HGX_K_PULL_HEAVY;
                r->stats.bytes_kernel[heavy_kind] += b_heavy;
                r->stats.bytes_kernel[HGX_K_HUB_FINALIZE] += b_hub;
                r->stats.launches[heavy_kind] += 1;
                r->stats.launches[HGX_K_HUB_FINALIZE] += 1;
            }
            if (d < 64) {
                for (int k = 0; k < 8; ++k) r->stats.level_rows[d][k] += (int64_t)c[k];
                r->stats.level_bytes[d] += b_gather + b_pull + b_heavy + b_hub;
                r->stats.level_sparse[d] = (int32_t)c[cDirRows];
            }
            if (!opush_level && !fc_level) r->stats.launches[HGX_K_LINK_GATHER] += 1;
            r->stats.launches[pull_kind] += 1;
            if (d < 64) r->stats.level_new[d] += (int64_t)c[cNewAtoms];
        }
        r->batches.push_back(std::move(bt));
    }
    if (tm.on) HGX_HIP(hipEventRecord(tm.all.b, g->stream));
    spin_sync(g->stream);
    int nl = 1;
    for (auto& bt : r->batches) nl = std::max(nl, (int)bt.lvl.size());
    if (r->blk)
        for (int32_t lv : r->blk->levels) nl = std::max(nl, lv + 1);
    r->n_levels = nl;
    r->stats.n_levels_expanded = max_expanded;
    r->stats.n_batches = (int32_t)r->batches.size();
    if (tm.on) {
        float ms = 0;
        HGX_HIP(hipEventElapsedTime(&ms, tm.all.a, tm.all.b));
        r->stats.ms_total = ms;
        tm.collect(r->stats);
    }
    guard.r = nullptr;
    *out = r;
}

}  // namespace

extern "C" {

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
    return hgx_bfs_result_visited_range(r, seed_index, depth, 0, out, cap, n_out);
}

int hgx_bfs_result_visited_range(hgx_bfs_result* r, int32_t seed_index, int32_t depth, int64_t first, int32_t* out,
                                 int64_t cap, int64_t* n_out) {
    HGX_API_BEGIN
    if (!r || !n_out || (cap > 0 && !out) || first < 0 || cap < 0)
        fail(HGX_E_INVALID, "hgx_bfs_result_visited: bad argument");
    if (seed_index < 0 || seed_index >= r->n_seeds) fail(HGX_E_NOTFOUND, "no such seed index");
    if (depth < 0) fail(HGX_E_NOTFOUND, "no such depth");
    hgx_graph* g = r->g;
    std::lock_guard<std::mutex> lk(g->mu);
    *n_out = 0;
    if (r->blk && r->blk->pairs[seed_index] >= 0) {   // a workgroup seed: its level, sorted on the host
        block_materialize(g, *r->blk);
        const BlockSet& b = *r->blk;
        if (depth > b.levels[seed_index]) return HGX_OK;
        if (depth == 0) {
            *n_out = 1;
            if (cap > 0 && first == 0) out[0] = b.seeds[seed_index];
            return HGX_OK;
        }
        int64_t beg = 0;
        for (int32_t d = 0; d < depth - 1; ++d) beg += b.lcnt[seed_index][d];
        const int64_t n = b.lcnt[seed_index][depth - 1];
        std::vector<int32_t> v(b.atoms[seed_index] + beg, b.atoms[seed_index] + beg + n);
        std::sort(v.begin(), v.end());
        *n_out = n;
        const int64_t k = std::min(std::max<int64_t>(n - first, 0), cap);
        if (k > 0) std::memcpy(out, v.data() + first, sizeof(int32_t) * (size_t)k);
        return HGX_OK;
    }
    HGX_HIP(hipSetDevice(g->device));
    if (r->blk) seed_index = r->compact[seed_index];
    const BfsBatch& bt = r->batches[seed_index / 1024];
    const int s = seed_index % 1024;
    auto iso = r->isolated.find(seed_index);
    if (iso != r->isolated.end()) {   // an isolated seed: only itself, at distance 0
        if (depth == 0) {
            *n_out = 1;
            if (cap > 0 && first == 0) out[0] = iso->second;
        }
        return HGX_OK;
    }
    if (depth >= (int32_t)bt.lvl.size()) return HGX_OK;
    const int nblk = (int)std::min<int64_t>(2048, std::max<int64_t>(1, ceil_div(g->A, 4096)));
    const int64_t span = ceil_div(std::max<int64_t>(g->A, 1), nblk);
    int64_t* dcnt = (int64_t*)g->alloc(sizeof(int64_t) * nblk * 2);
    int64_t* doff = dcnt + nblk;
    const u64* own = g->shard ? (const u64*)g->shard->own_bm : nullptr;   // a part reports its owned atoms
    hgx_extract<<<nblk, 256, 0, g->stream>>>(g->A, span, bt.W, s, bt.fa[depth], own, bt.lvl[depth], doff, dcnt, nullptr,
                                              0, false);
    HGX_CHECK_LAUNCH();
    std::vector<int64_t> hc(nblk), ho(nblk);
    HGX_HIP(hipMemcpyAsync(hc.data(), dcnt, sizeof(int64_t) * nblk, hipMemcpyDeviceToHost, g->stream));
    HGX_HIP(hipStreamSynchronize(g->stream));
    int64_t tot = 0;
    for (int i = 0; i < nblk; ++i) {
        ho[i] = tot - first;   // positions relative to the range's first entry
        tot += hc[i];
    }
    *n_out = tot;
    int64_t k = std::min(std::max<int64_t>(tot - first, 0), cap);
    if (k > 0) {
        int32_t* dout = (int32_t*)g->alloc(sizeof(int32_t) * k);
        HGX_HIP(hipMemcpyAsync(doff, ho.data(), sizeof(int64_t) * nblk, hipMemcpyHostToDevice, g->stream));
        hgx_extract<<<nblk, 256, 0, g->stream>>>(g->A, span, bt.W, s, bt.fa[depth], own, bt.lvl[depth], doff, dcnt, dout,
                                                  k, true);
        HGX_CHECK_LAUNCH();
        HGX_HIP(hipMemcpyAsync(out, dout, sizeof(int32_t) * k, hipMemcpyDeviceToHost, g->stream));
        HGX_HIP(hipStreamSynchronize(g->stream));
        g->release(dout, sizeof(int32_t) * k);
        if (g->shard)   // local ids are in global order: the mapped list stays ascending
            for (int64_t i = 0; i < k; ++i) out[i] = g->shard->l2g_host[out[i]];
    }
    g->release(dcnt, sizeof(int64_t) * nblk * 2);
    HGX_API_END
}

int hgx_bfs_result_depth_of(hgx_bfs_result* r, int32_t seed_index, int32_t atom, int32_t* depth_out) {
    HGX_API_BEGIN
    if (!r || !depth_out) fail(HGX_E_INVALID, "hgx_bfs_result_depth_of: bad argument");
    if (seed_index < 0 || seed_index >= r->n_seeds) fail(HGX_E_NOTFOUND, "no such seed index");
    hgx_graph* g = r->g;
    if (g->shard) {   // global id of an atom this shard owns
        const ShardInfo& sh = *g->shard;
        if (atom < 0 || atom >= sh.A_global) fail(HGX_E_INVALID, "atom id out of range");
        if (!sh.present(atom)) {   // no incidence anywhere: reached only as its own seed (part atom % n_parts)
            if (atom % sh.n_parts != sh.part) fail(HGX_E_NOTFOUND, "atom is owned by another part");
            auto iso = r->isolated.find(seed_index);
            *depth_out = (iso != r->isolated.end() && iso->second == atom) ? 0 : -1;
            return HGX_OK;
        }
        const int32_t loc = sh.local_of(atom);
        if (loc < 0 || !sh.owns_local(loc)) fail(HGX_E_NOTFOUND, "atom is owned by another part");
        atom = loc;
    }
    if (atom < 0 || atom >= g->A) fail(HGX_E_INVALID, "atom id out of range");
    std::lock_guard<std::mutex> lk(g->mu);
    if (r->blk && r->blk->pairs[seed_index] >= 0) {   // a workgroup seed: scan its levels
        block_materialize(g, *r->blk);
        const BlockSet& b = *r->blk;
        *depth_out = -1;
        if (b.seeds[seed_index] == atom) {
            *depth_out = 0;
            return HGX_OK;
        }
        int64_t k = 0;
        for (int32_t d = 0; d < b.levels[seed_index] && *depth_out < 0; ++d)
            for (int64_t e = k + b.lcnt[seed_index][d]; k < e; ++k)
                if (b.atoms[seed_index][k] == atom) {
                    *depth_out = d + 1;
                    break;
                }
        return HGX_OK;
    }
    HGX_HIP(hipSetDevice(g->device));
    if (r->blk) seed_index = r->compact[seed_index];
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
    hgx_depth_probe<<<1, 64, 0, g->stream>>>(nl, (const u64* const*)tab, (const u64* const*)(tab + nl), bt.W,
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
    if (with_accounting) ensure_accounting(r);
    *st = r->stats;
    HGX_API_END
}

void hgx_bfs_result_free(hgx_bfs_result* r) {
    if (!r) return;
    hgx_graph* g = r->g;
    if (g) {
        std::lock_guard<std::mutex> lk(g->mu);
        (void)hipSetDevice(g->device);
        if (g->stream2) (void)hipStreamSynchronize(g->stream2);   // counting passes may still read the rows
        for (auto& bt : r->batches) {
            for (auto p : bt.lvl) g->release(p, r->row_bytes(bt));
            for (auto p : bt.fa) g->release(p, r->bm_bytes());
            if (bt.pcnt) g->release(bt.pcnt, sizeof(u64) * 1024 * kDirectLevels);
            for (auto p : bt.cpart)
                if (p) g->release(p, bt.cpart_bytes);
        }
        if (r->blk) block_release(g, *r->blk);
    }
    delete r;
    if (g) graph_release(g);
}

}  // extern "C"

// The read-only tables the BFS otherwise builds on first use -- the has-incidence bitmap (non-full
// pull levels), the ordered-mode yield flags and the frontier-push chunk table -- built now on the
// snapshot so that its execution contexts (hgx_graph_context) share one copy.  Caller holds g->mu.
void hgx::bfs_shared_tables(hgx_graph* g) {
    hipStream_t s = g->stream;
    const int64_t A = g->A;
    if (!g->hasinc) {
        HGX_HIP(hipMalloc(&g->hasinc, sizeof(u64) * (size_t)(ceil_div(A, 64) + 1)));
        hgx_hasinc<<<grid_for(ceil_div(A, 64) * 64, 256, 4096), 256, 0, s>>>(A, g->inc_off, (u64*)g->hasinc);
        HGX_CHECK_LAUNCH();
    }
    if (!g->inc_yf) ensure_inc_yield(g);
    if (g->n_pchunks < 0) build_push_chunks(g);
    HGX_HIP(hipStreamSynchronize(s));
}

void hgx::ensure_inc_yield(hgx_graph* g) {
    if (g->inc_yf) return;
    HGX_HIP(hipMalloc(&g->inc_yf, (size_t)g->I + 64));   // + padding: 16-byte loads of the last entries
    HGX_HIP(hipMemsetAsync(g->inc_yf + g->I, 0, 64, g->stream));
    hgx_inc_yield<<<grid_for(g->A * 64, 256, 8192), 256, 0, g->stream>>>(g->A, g->inc_off, g->inc_row, g->tgt_off,
                                                                         g->tgt_idx, g->inc_yf);
    HGX_CHECK_LAUNCH();
}
