// hgx_part.hip -- vertex-cut partition of a snapshot over n_parts devices and the transports of
// the partitioned BFS.
//
// The reference keeps one incidence index per store (HGStore.getIncidenceResultSet,
// C/HGStore.java:253; BJEStorageImplementation.java:405-439) and walks it one atom at a time
// (HGBreadthFirstTraversal.java:49-66).  Config 4 (1B incidences) is split by LINK: every link row
// lives on exactly one part (its target row is stored once), so a part's gather and pull touch
// 1/n_parts of the pins.  An atom is present on every part holding one of its links (its holders);
// one holder owns it.  A BFS level then needs two exchanges of S-bit rows (hgx_bfs.hip, Exchange):
//   reduce    each holder ships its partial news for an atom to the owner, which ORs them;
//   broadcast the owner ships the atom's final news back to the other holders,
// so every holder's frontier row and visited row stay identical to the whole-graph engine's.
//
// Placement (hgx_partition_plan): greedy streaming vertex cut -- a link goes to the part that
// already holds the most of its targets, each target weighted 1/deg (low-degree atoms decide, hubs
// are everywhere anyway), within a pin-balance cap.  Config 4 at 2-10% scale: 1.0 remote holder
// per present atom against 2.0 for a random placement (tools/vcut_quality.py).  Decisions are taken in
// batches of plan_batch(M) links against the hold state at the batch start, in kPlanChunks fixed
// chunks, so the plan is deterministic whatever the thread count -- every rank of a multi-process
// run computes the same plan from the same snapshot.
// Owner of a present atom: one of its holders, chosen by a hash of its id (balances owned atoms).
// Local ids follow global id order, so ascending local lists are ascending global lists and the
// on-device incidence build of hgx_graph_create applies unchanged.
//
// Transports: RCCL (grouped ncclSend/ncclRecv over xGMI, one process per GPU), an in-process
// group (one host thread per part, device-to-device copies) used by hgx_pbfs_batch_group, and a
// host-staged transport whose collectives are callbacks into the caller (e.g. a gloo group).
#include <rccl/rccl.h>

#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <memory>
#include <numeric>
#include <thread>

#include "hgx_internal.h"

using namespace hgx;

struct hgx_shard {
    int32_t n_parts = 1, part = 0;
    int64_t A_global = 0, n_owned = 0;
    std::vector<int32_t> l2g;                 // [A_local] global id, ascending
    std::vector<int32_t> link_atom, link_type, tgt_idx;
    std::vector<int64_t> tgt_off;
    std::vector<uint64_t> own_bm;             // [A_local/64 + 2] owned local atoms
    std::vector<int32_t> xo_part, xo_lid;     // [A_local] ghosts: owner part / local id there (-1: owned)
    std::vector<int64_t> bc_off;              // [A_local + 1] owned atoms: other holders
    std::vector<int32_t> bc_part, bc_lid;     //   (part, local id there)
    std::vector<int64_t> ghost_count, bc_count;   // [n_parts] reduce / broadcast records per peer
    std::vector<uint64_t> present;            // [A_global/64 + 1] atoms present on some part
};

namespace {

int host_threads() {
    unsigned n = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(n, 16u));
}

// fn(lo, hi, t) over [0, n) split into contiguous chunks, one per thread.
template <class F>
void parallel_for(int64_t n, F fn) {
    const int T = (int)std::min<int64_t>(host_threads(), std::max<int64_t>(1, n / 65536));
    if (T <= 1) {
        fn((int64_t)0, n, 0);
        return;
    }
    std::vector<std::thread> th;
    const int64_t per = (n + T - 1) / T;
    for (int t = 0; t < T; ++t) {
        const int64_t lo = std::min(n, t * per), hi = std::min(n, lo + per);
        th.emplace_back([=] { fn(lo, hi, t); });
    }
    for (auto& x : th) x.join();
}

// T worker threads started once; run(fn) executes fn(t) on every worker and returns when all are
// done (a generation barrier), so thousands of short phases cost no thread launches.
struct WorkerPool {
    int T;
    std::vector<std::thread> th;
    std::mutex mu;
    std::condition_variable cv_go, cv_done;
    std::function<void(int)> job;
    int64_t gen = 0;
    int running = 0;
    bool quit = false;
    explicit WorkerPool(int t) : T(t) {
        for (int i = 0; i < T; ++i)
            th.emplace_back([this, i] {
                int64_t seen = 0;
                for (;;) {
                    std::function<void(int)> f;
                    {
                        std::unique_lock<std::mutex> lk(mu);
                        cv_go.wait(lk, [&] { return quit || gen != seen; });
                        if (quit) return;
                        seen = gen;
                        f = job;
                    }
                    f(i);
                    std::lock_guard<std::mutex> lk(mu);
                    if (--running == 0) cv_done.notify_all();
                }
            });
    }
    ~WorkerPool() {
        {
            std::lock_guard<std::mutex> lk(mu);
            quit = true;
        }
        cv_go.notify_all();
        for (auto& x : th) x.join();
    }
    void run(std::function<void(int)> f) {
        std::unique_lock<std::mutex> lk(mu);
        job = std::move(f);
        running = T;
        ++gen;
        cv_go.notify_all();
        cv_done.wait(lk, [&] { return running == 0; });
    }
};

void check_rows(const hgx_graph_desc* d) {
    const int64_t A = d->num_atoms, M = d->num_links;
    if (A < 0 || M < 0 || A >= (int64_t)INT32_MAX) fail(HGX_E_INVALID, "partition: bad sizes");
    if (M > 0 && (!d->tgt_off || !d->tgt_idx || !d->link_atom)) fail(HGX_E_INVALID, "partition: null link arrays");
    const int64_t* off = d->tgt_off;
    const int32_t* tg = d->tgt_idx;
    if (M > 0 && off[0] != 0) fail(HGX_E_INVALID, "partition: tgt_off[0] != 0");
    std::vector<int> bad(64, 0);
    parallel_for(M, [&](int64_t lo, int64_t hi, int t) {
        for (int64_t r = lo; r < hi; ++r) {
            if (off[r + 1] < off[r]) {
                bad[t] = 1;
                continue;
            }
            for (int64_t p = off[r]; p < off[r + 1]; ++p)
                if (tg[p] < 0 || tg[p] >= A) {
                    bad[t] = 2;
                    break;
                }
        }
    });
    for (int b : bad)
        if (b == 1) fail(HGX_E_INVALID, "partition: tgt_off not monotone");
        else if (b == 2) fail(HGX_E_INVALID, "partition: target id out of range");
}

// Links placed against one hold-state snapshot: M/512 clamped to [1K, 64K] (a function of M only,
// so the plan stays deterministic); the first batch of a placement sees an empty state.
inline int64_t plan_batch(int64_t M) { return std::min<int64_t>(std::max<int64_t>(M / 512, 1024), 1 << 16); }
constexpr int kPlanChunks = 16;   // fixed chunks per batch (determinism)

void plan_links(const hgx_graph_desc* d, int NP, int32_t* link_part, double slack) {
    const int64_t A = d->num_atoms, M = d->num_links;
    const int64_t* off = d->tgt_off;
    const int32_t* tg = d->tgt_idx;
    const int64_t P = M > 0 ? off[M] : 0;
    if (NP == 1) {
        std::fill(link_part, link_part + M, 0);
        return;
    }
    std::vector<int32_t> deg((size_t)A, 0);
    parallel_for(P, [&](int64_t lo, int64_t hi, int) {
        for (int64_t p = lo; p < hi; ++p) __atomic_fetch_add(&deg[tg[p]], 1, __ATOMIC_RELAXED);
    });
    std::vector<float> wt((size_t)A);
    parallel_for(A, [&](int64_t lo, int64_t hi, int) {
        for (int64_t v = lo; v < hi; ++v) wt[v] = deg[v] > 0 ? 1.0f / (float)deg[v] : 0.0f;
    });
    std::vector<int32_t>().swap(deg);
    std::vector<uint64_t> hold((size_t)A, 0);
    std::vector<int64_t> load(NP, 0);
    const int64_t cap = (int64_t)((1.0 + slack) * (double)P / NP) + 64;
    std::vector<std::vector<int64_t>> delta(kPlanChunks, std::vector<int64_t>(NP, 0));
    WorkerPool pool(std::min(host_threads(), kPlanChunks));
    const int64_t batch = plan_batch(M);
    for (int64_t b0 = 0; b0 < M; b0 += batch) {
        const int64_t b1 = std::min(M, b0 + batch);
        const int64_t per = (b1 - b0 + kPlanChunks - 1) / kPlanChunks;
        // decide: every chunk reads the hold state of the batch start and its own load deltas
        pool.run([&](int t) {
            for (int c = t; c < kPlanChunks; c += pool.T) {
                std::vector<int64_t>& dl = delta[c];
                std::fill(dl.begin(), dl.end(), 0);
                const int64_t lo = std::min(b1, b0 + c * per), hi = std::min(b1, lo + per);
                float score[64];
                for (int64_t L = lo; L < hi; ++L) {
                    for (int q = 0; q < NP; ++q) score[q] = 0.0f;
                    for (int64_t p = off[L]; p < off[L + 1]; ++p) {
                        uint64_t m = hold[tg[p]];
                        const float w = wt[tg[p]];
                        while (m) {
                            score[__builtin_ctzll(m)] += w;
                            m &= m - 1;
                        }
                    }
                    const int64_t n = off[L + 1] - off[L];
                    int best = -1;
                    for (int q = 0; q < NP; ++q) {
                        // each chunk of the batch may fill 1/kPlanChunks of a part's room under the cap
                        // (the chunks decide concurrently against the batch-start loads)
                        if ((dl[q] + n) * kPlanChunks > cap - load[q]) continue;
                        if (best < 0 || score[q] > score[best] ||
                            (score[q] == score[best] && load[q] + dl[q] < load[best] + dl[best]))
                            best = q;
                    }
                    if (best < 0) {   // every part at the cap: the least loaded
                        best = 0;
                        for (int q = 1; q < NP; ++q)
                            if (load[q] + dl[q] < load[best] + dl[best]) best = q;
                    }
                    link_part[L] = best;
                    dl[best] += n;
                }
            }
        });
        for (int c = 0; c < kPlanChunks; ++c)
            for (int q = 0; q < NP; ++q) load[q] += delta[c][q];
        // apply the batch's placements to the hold state
        pool.run([&](int t) {
            const int64_t per2 = (b1 - b0 + pool.T - 1) / pool.T;
            const int64_t lo = std::min(b1, b0 + t * per2), hi = std::min(b1, lo + per2);
            for (int64_t L = lo; L < hi; ++L) {
                const uint64_t bitq = 1ull << link_part[L];
                for (int64_t p = off[L]; p < off[L + 1]; ++p) {
                    uint64_t* h = &hold[tg[p]];
                    if (!(__atomic_load_n(h, __ATOMIC_RELAXED) & bitq)) __atomic_fetch_or(h, bitq, __ATOMIC_RELAXED);
                }
            }
        });
    }
}

inline uint64_t mix64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

// owner of a present atom: holder number mix(v) % |holders| in part order
inline int owner_of(int64_t v, uint64_t hold) {
    int k = (int)(mix64((uint64_t)v) % (uint64_t)__builtin_popcountll(hold));
    while (k--) hold &= hold - 1;
    return __builtin_ctzll(hold);
}

hgx_shard* shard_build(const hgx_graph_desc* d, int32_t NP, int32_t part, const int32_t* link_part) {
    const int64_t A = d->num_atoms, M = d->num_links;
    if (NP < 1 || NP > 64 || part < 0 || part >= NP) fail(HGX_E_INVALID, "hgx_shard_build: bad part / n_parts (1..64)");
    if (M > 0 && !link_part) fail(HGX_E_INVALID, "hgx_shard_build: null link placement");
    check_rows(d);
    const int64_t* off = d->tgt_off;
    const int32_t* tg = d->tgt_idx;
    for (int64_t r = 0; r < M; ++r)
        if (link_part[r] < 0 || link_part[r] >= NP) fail(HGX_E_INVALID, "hgx_shard_build: link placement out of range");
    std::unique_ptr<hgx_shard> s(new hgx_shard());
    s->n_parts = NP;
    s->part = part;
    s->A_global = A;

    // 1. holders of every atom
    std::vector<uint64_t> hold((size_t)A, 0);
    parallel_for(M, [&](int64_t lo, int64_t hi, int) {
        for (int64_t r = lo; r < hi; ++r) {
            const uint64_t bq = 1ull << link_part[r];
            for (int64_t p = off[r]; p < off[r + 1]; ++p) {
                uint64_t* h = &hold[tg[p]];
                if (!(__atomic_load_n(h, __ATOMIC_RELAXED) & bq)) __atomic_fetch_or(h, bq, __ATOMIC_RELAXED);
            }
        }
    });
    // 2. per-part presence bitmaps and their block prefix counts: lid_q(v) in O(1)
    const int64_t nw = A / 64 + 1;
    std::vector<uint64_t> bm((size_t)NP * nw, 0);
    std::vector<int32_t> cnt((size_t)NP * nw, 0);
    s->present.assign((size_t)nw, 0);
    parallel_for(nw, [&](int64_t lo, int64_t hi, int) {
        for (int64_t w = lo; w < hi; ++w) {
            uint64_t pres = 0;
            for (int64_t i = 0; i < 64 && w * 64 + i < A; ++i) {
                uint64_t m = hold[w * 64 + i];
                if (m) pres |= 1ull << i;
                while (m) {
                    bm[(size_t)__builtin_ctzll(m) * nw + w] |= 1ull << i;
                    m &= m - 1;
                }
            }
            s->present[w] = pres;
        }
    });
    parallel_for(NP, [&](int64_t lo, int64_t hi, int) {
        for (int64_t q = lo; q < hi; ++q) {
            int64_t run = 0;
            for (int64_t w = 0; w < nw; ++w) {
                cnt[(size_t)q * nw + w] = (int32_t)run;
                run += __builtin_popcountll(bm[(size_t)q * nw + w]);
            }
        }
    });
    auto lid = [&](int q, int64_t v) -> int32_t {
        const int64_t w = v >> 6;
        return cnt[(size_t)q * nw + w] + __builtin_popcountll(bm[(size_t)q * nw + w] & ((1ull << (v & 63)) - 1ull));
    };
    // 3. local atoms of this part (ascending global ids) and their exchange partners
    int64_t AL = 0;
    for (int64_t w = 0; w < nw; ++w) AL += __builtin_popcountll(bm[(size_t)part * nw + w]);
    s->l2g.resize((size_t)AL);
    parallel_for(nw, [&](int64_t lo, int64_t hi, int) {
        for (int64_t w = lo; w < hi; ++w) {
            uint64_t m = bm[(size_t)part * nw + w];
            int64_t k = cnt[(size_t)part * nw + w];
            while (m) {
                s->l2g[k++] = (int32_t)(w * 64 + __builtin_ctzll(m));
                m &= m - 1;
            }
        }
    });
    s->own_bm.assign((size_t)(AL / 64 + 2), 0);
    s->xo_part.assign((size_t)AL, -1);
    s->xo_lid.assign((size_t)AL, -1);
    s->bc_off.assign((size_t)AL + 1, 0);
    std::vector<int32_t> nbc((size_t)AL, 0);
    parallel_for(AL, [&](int64_t lo, int64_t hi, int) {
        for (int64_t i = lo; i < hi; ++i) {
            const int64_t v = s->l2g[i];
            const uint64_t h = hold[v];
            const int o = owner_of(v, h);
            if (o == part) nbc[i] = __builtin_popcountll(h) - 1;
            else {
                s->xo_part[i] = o;
                s->xo_lid[i] = lid(o, v);
            }
        }
    });
    for (int64_t i = 0; i < AL; ++i) {
        s->bc_off[i + 1] = s->bc_off[i] + nbc[i];
        if (s->xo_part[i] < 0) s->own_bm[i >> 6] |= 1ull << (i & 63);
    }
    s->bc_part.resize((size_t)s->bc_off[AL]);
    s->bc_lid.resize((size_t)s->bc_off[AL]);
    parallel_for(AL, [&](int64_t lo, int64_t hi, int) {
        for (int64_t i = lo; i < hi; ++i) {
            if (!nbc[i]) continue;
            const int64_t v = s->l2g[i];
            uint64_t m = hold[v] & ~(1ull << part);
            int64_t k = s->bc_off[i];
            while (m) {
                const int q = __builtin_ctzll(m);
                m &= m - 1;
                s->bc_part[k] = q;
                s->bc_lid[k++] = lid(q, v);
            }
        }
    });
    s->ghost_count.assign(NP, 0);
    s->bc_count.assign(NP, 0);
    for (int64_t i = 0; i < AL; ++i)
        if (s->xo_part[i] >= 0) s->ghost_count[s->xo_part[i]]++;
    for (int32_t q : s->bc_part) s->bc_count[q]++;
    s->n_owned = AL - std::accumulate(s->ghost_count.begin(), s->ghost_count.end(), (int64_t)0);

    // 4. local link rows (ascending global row order) with targets in local ids
    std::vector<int64_t> lrow;
    lrow.reserve((size_t)(M / std::max(NP, 1) + 16));
    for (int64_t r = 0; r < M; ++r)
        if (link_part[r] == part) lrow.push_back(r);
    const int64_t ML = (int64_t)lrow.size();
    s->tgt_off.resize((size_t)ML + 1);
    s->link_atom.resize((size_t)ML);
    s->link_type.resize((size_t)ML);
    s->tgt_off[0] = 0;
    for (int64_t i = 0; i < ML; ++i) s->tgt_off[i + 1] = s->tgt_off[i] + (off[lrow[i] + 1] - off[lrow[i]]);
    s->tgt_idx.resize((size_t)s->tgt_off[ML]);
    parallel_for(ML, [&](int64_t lo, int64_t hi, int) {
        for (int64_t i = lo; i < hi; ++i) {
            const int64_t r = lrow[i];
            s->link_atom[i] = d->link_atom[r];
            s->link_type[i] = d->link_type ? d->link_type[r] : 0;
            int64_t o = s->tgt_off[i];
            for (int64_t p = off[r]; p < off[r + 1]; ++p) s->tgt_idx[o++] = lid(part, tg[p]);
        }
    });
    return s.release();
}

// ---------------------------------------------------------------------------------------------
// Transports
// ---------------------------------------------------------------------------------------------

#define HGX_NCCL(x)                                                                                    \
    do {                                                                                               \
        ncclResult_t r_ = (x);                                                                         \
        if (r_ != ncclSuccess) ::hgx::fail(HGX_E_DEVICE, std::string(#x) + ": " + ncclGetErrorString(r_)); \
    } while (0)

}  // namespace

int hgx::Transport::allgather_dev(const int64_t* din, int64_t n, int64_t* out, hipStream_t s, int64_t* pin) {
    HGX_HIP(hipMemcpyAsync(pin, din, sizeof(int64_t) * n, hipMemcpyDeviceToHost, s));
    spin_sync(s);
    allgather_i64(pin, n, out, s);
    return 2;
}

namespace {

struct RcclTransport : Transport {
    ncclComm_t comm = nullptr;
    int device = 0;
    int64_t* scratch = nullptr;   // device staging of the small all-gathers
    int64_t scratch_n = 0;
    ~RcclTransport() override {
        if (scratch) (void)hipFree(scratch);
        if (comm) (void)ncclCommDestroy(comm);
    }
    const char* kind() const override { return "rccl"; }
    void allgather_i64(const int64_t* in, int64_t n, int64_t* out, hipStream_t s) override {
        const int64_t need = n * world;
        if (need > scratch_n) {
            if (scratch) HGX_HIP(hipFree(scratch));
            scratch = nullptr;
            HGX_HIP(hipMalloc(&scratch, sizeof(int64_t) * need));
            scratch_n = need;
        }
        HGX_HIP(hipMemcpyAsync(scratch + (int64_t)rank * n, in, sizeof(int64_t) * n, hipMemcpyHostToDevice, s));
        HGX_NCCL(ncclAllGather(scratch + (int64_t)rank * n, scratch, (size_t)n, ncclInt64, comm, s));
        HGX_HIP(hipMemcpyAsync(out, scratch, sizeof(int64_t) * need, hipMemcpyDeviceToHost, s));
        spin_sync(s);
    }
    // the counts never leave the device before the gather: one collective, one read-back
    int allgather_dev(const int64_t* din, int64_t n, int64_t* out, hipStream_t s, int64_t* pin) override {
        const int64_t need = n * world;
        if (need > scratch_n) {
            if (scratch) HGX_HIP(hipFree(scratch));
            scratch = nullptr;
            HGX_HIP(hipMalloc(&scratch, sizeof(int64_t) * need));
            scratch_n = need;
        }
        HGX_NCCL(ncclAllGather(din, scratch, (size_t)n, ncclInt64, comm, s));
        HGX_HIP(hipMemcpyAsync(pin, scratch, sizeof(int64_t) * need, hipMemcpyDeviceToHost, s));
        spin_sync(s);
        std::memcpy(out, pin, sizeof(int64_t) * need);
        return 1;
    }
    void alltoallv(const void* send, const int64_t* send_off, const int64_t* send_bytes, void* recv,
                   const int64_t* recv_off, const int64_t* recv_bytes, hipStream_t s) override {
        HGX_NCCL(ncclGroupStart());
        for (int p = 0; p < world; ++p) {
            if (p == rank) continue;
            if (send_bytes[p] > 0)
                HGX_NCCL(ncclSend((const char*)send + send_off[p], (size_t)send_bytes[p], ncclUint8, p, comm, s));
            if (recv_bytes[p] > 0)
                HGX_NCCL(ncclRecv((char*)recv + recv_off[p], (size_t)recv_bytes[p], ncclUint8, p, comm, s));
        }
        HGX_NCCL(ncclGroupEnd());
        if (send_bytes[rank] > 0)   // never produced by the BFS (own atoms are not ghosts); kept general
            HGX_HIP(hipMemcpyAsync((char*)recv + recv_off[rank], (const char*)send + send_off[rank],
                                   (size_t)send_bytes[rank], hipMemcpyDeviceToDevice, s));
    }
};

// In-process group: one host thread per part; a generation barrier with an abort flag so one
// failing part releases the others instead of leaving them waiting.
struct LocalHub {
    int world;
    bool serial = false;   // rehearsal: one part's device work at a time (clean per-part device times)
    std::mutex gate;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    int64_t gen = 0;
    bool aborted = false;
    std::vector<const int64_t*> ag_in;
    std::vector<const void*> send;
    std::vector<const int64_t*> send_off;
    std::vector<int> dev;
    explicit LocalHub(int w) : world(w), ag_in(w), send(w), send_off(w), dev(w) {}
    void barrier() {
        std::unique_lock<std::mutex> lk(mu);
        if (aborted) fail(HGX_E_DEVICE, "partition group aborted by another part");
        const int64_t my = gen;
        if (++arrived == world) {
            arrived = 0;
            ++gen;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return gen != my || aborted; });
            if (gen == my) fail(HGX_E_DEVICE, "partition group aborted by another part");
        }
    }
    void abort() {
        std::lock_guard<std::mutex> lk(mu);
        aborted = true;
        cv.notify_all();
    }
};

struct LocalTransport : Transport {
    std::shared_ptr<LocalHub> hub;
    int device = 0;
    const char* kind() const override { return "local"; }
    bool held = false;
    void compute_begin(hipStream_t) override {
        if (hub->serial && !held) {
            hub->gate.lock();
            held = true;
        }
    }
    void compute_end(hipStream_t s) override {
        if (!held) return;
        hipError_t e = hipStreamSynchronize(s);   // this part's kernels have finished
        held = false;
        hub->gate.unlock();
        HGX_HIP(e);
    }
    void compute_release(hipStream_t s) override {
        if (!held) return;
        (void)hipStreamSynchronize(s);
        held = false;
        hub->gate.unlock();
    }
    void allgather_i64(const int64_t* in, int64_t n, int64_t* out, hipStream_t) override {
        hub->ag_in[rank] = in;
        hub->barrier();
        for (int r = 0; r < world; ++r) std::memcpy(out + (int64_t)r * n, hub->ag_in[r], sizeof(int64_t) * n);
        hub->barrier();
    }
    void alltoallv(const void* send, const int64_t* send_off, const int64_t* send_bytes, void* recv,
                   const int64_t* recv_off, const int64_t* recv_bytes, hipStream_t s) override {
        HGX_HIP(hipStreamSynchronize(s));   // my send segments are complete
        hub->send[rank] = send;
        hub->send_off[rank] = send_off;
        hub->dev[rank] = device;
        hub->barrier();
        {
            // rehearsal: the copies (the modelled link traffic) run under the gate too, so no
            // part's kernels overlap another part's copies; the gate is given back before the barrier
            struct Ungate {
                LocalHub* h;
                ~Ungate() {
                    if (h) h->gate.unlock();
                }
            } ungate{nullptr};
            if (hub->serial) {
                hub->gate.lock();
                ungate.h = hub.get();
            }
            for (int p = 0; p < world; ++p) {
                if (recv_bytes[p] <= 0) continue;
                const char* src = (const char*)hub->send[p] + hub->send_off[p][rank];
                char* dst = (char*)recv + recv_off[p];
                if (hub->dev[p] == device)
                    HGX_HIP(hipMemcpyAsync(dst, src, (size_t)recv_bytes[p], hipMemcpyDeviceToDevice, s));
                else
                    HGX_HIP(hipMemcpyPeerAsync(dst, device, src, hub->dev[p], (size_t)recv_bytes[p], s));
            }
            HGX_HIP(hipStreamSynchronize(s));
        }
        hub->barrier();   // every part has pulled its segments: send buffers may be reused
        (void)send_bytes;
    }
};

// Host-staged transport: the collectives are the caller's callbacks on host buffers (e.g. a
// torch.distributed gloo group); device segments are staged through pinned host memory.  Used to
// run the partitioned BFS between processes without RCCL (tests on one GPU).
struct HostTransport : Transport {
    hgx_host_allgather_fn ag = nullptr;
    hgx_host_alltoallv_fn a2a = nullptr;
    void* user = nullptr;
    void* hs = nullptr;
    void* hr = nullptr;
    size_t hs_n = 0, hr_n = 0;
    ~HostTransport() override {
        if (hs) (void)hipHostFree(hs);
        if (hr) (void)hipHostFree(hr);
    }
    const char* kind() const override { return "host"; }
    static void grow(void*& p, size_t& n, size_t need) {
        if (need <= n) return;
        if (p) HGX_HIP(hipHostFree(p));
        p = nullptr;
        n = 0;
        HGX_HIP(hipHostMalloc(&p, need));
        n = need;
    }
    void allgather_i64(const int64_t* in, int64_t n, int64_t* out, hipStream_t) override {
        if (ag(user, in, n, out) != 0) fail(HGX_E_DEVICE, "host transport: all-gather callback failed");
    }
    void alltoallv(const void* send, const int64_t* send_off, const int64_t* send_bytes, void* recv,
                   const int64_t* recv_off, const int64_t* recv_bytes, hipStream_t s) override {
        size_t sn = 1, rn = 1;
        for (int p = 0; p < world; ++p) {
            sn = std::max(sn, (size_t)(send_off[p] + send_bytes[p]));
            rn = std::max(rn, (size_t)(recv_off[p] + recv_bytes[p]));
        }
        grow(hs, hs_n, sn);
        grow(hr, hr_n, rn);
        for (int p = 0; p < world; ++p)
            if (send_bytes[p] > 0)
                HGX_HIP(hipMemcpyAsync((char*)hs + send_off[p], (const char*)send + send_off[p], (size_t)send_bytes[p],
                                       hipMemcpyDeviceToHost, s));
        HGX_HIP(hipStreamSynchronize(s));
        if (a2a(user, hs, send_off, send_bytes, hr, recv_off, recv_bytes) != 0)
            fail(HGX_E_DEVICE, "host transport: all-to-all callback failed");
        for (int p = 0; p < world; ++p)
            if (recv_bytes[p] > 0)
                HGX_HIP(hipMemcpyAsync((char*)recv + recv_off[p], (const char*)hr + recv_off[p], (size_t)recv_bytes[p],
                                       hipMemcpyHostToDevice, s));
        HGX_HIP(hipStreamSynchronize(s));
    }
};

}  // namespace

// copy a host table to a caller buffer (an empty table copies nothing: memcpy from a null data()
// would be undefined even at size 0)
template <class T>
static void copy_out(T* dst, const std::vector<T>& v) {
    if (dst && !v.empty()) std::memcpy(dst, v.data(), sizeof(T) * v.size());
}

extern "C" {

int hgx_partition_plan(const hgx_graph_desc* global, int32_t n_parts, int32_t* link_part) {
    HGX_API_BEGIN
    if (!global || (global->num_links > 0 && !link_part)) fail(HGX_E_INVALID, "hgx_partition_plan: null argument");
    if (n_parts < 1 || n_parts > 64) fail(HGX_E_INVALID, "hgx_partition_plan: n_parts must be 1..64");
    check_rows(global);
    plan_links(global, n_parts, link_part, 0.02);
    HGX_API_END
}

int hgx_shard_build(const hgx_graph_desc* global, int32_t n_parts, int32_t part, const int32_t* link_part,
                    hgx_shard** out) {
    HGX_API_BEGIN
    if (!global || !out) fail(HGX_E_INVALID, "hgx_shard_build: null argument");
    *out = nullptr;
    *out = shard_build(global, n_parts, part, link_part);
    HGX_API_END
}

int hgx_shard_info(const hgx_shard* s, int64_t* n_local, int64_t* n_owned, int64_t* n_local_links,
                   int64_t* n_local_pins) {
    HGX_API_BEGIN
    if (!s) fail(HGX_E_INVALID, "null shard");
    if (n_local) *n_local = (int64_t)s->l2g.size();
    if (n_owned) *n_owned = s->n_owned;
    if (n_local_links) *n_local_links = (int64_t)s->link_atom.size();
    if (n_local_pins) *n_local_pins = (int64_t)s->tgt_idx.size();
    HGX_API_END
}

int hgx_shard_export(const hgx_shard* s, int32_t* l2g, int32_t* link_atom, int32_t* link_type, int64_t* tgt_off,
                     int32_t* tgt_idx, int64_t* ghost_count) {
    HGX_API_BEGIN
    if (!s) fail(HGX_E_INVALID, "null shard");
    copy_out(l2g, s->l2g);
    copy_out(link_atom, s->link_atom);
    copy_out(link_type, s->link_type);
    copy_out(tgt_off, s->tgt_off);
    copy_out(tgt_idx, s->tgt_idx);
    copy_out(ghost_count, s->ghost_count);
    HGX_API_END
}

int hgx_shard_exchange_tables(const hgx_shard* s, int32_t* xo_part, int32_t* xo_lid, int64_t* bc_off,
                              int32_t* bc_part, int32_t* bc_lid, int64_t* bc_count) {
    HGX_API_BEGIN
    if (!s) fail(HGX_E_INVALID, "null shard");
    copy_out(xo_part, s->xo_part);
    copy_out(xo_lid, s->xo_lid);
    copy_out(bc_off, s->bc_off);
    copy_out(bc_part, s->bc_part);
    copy_out(bc_lid, s->bc_lid);
    copy_out(bc_count, s->bc_count);
    HGX_API_END
}

void hgx_shard_free(hgx_shard* s) { delete s; }

int hgx_shard_graph_create(const hgx_shard* s, int32_t device, hgx_graph** out) {
    HGX_API_BEGIN
    if (!s || !out) fail(HGX_E_INVALID, "hgx_shard_graph_create: null argument");
    *out = nullptr;
    const int64_t AL = (int64_t)s->l2g.size(), ML = (int64_t)s->link_atom.size();
    hgx_graph_desc d{AL, ML, s->link_atom.data(), s->tgt_off.data(), s->tgt_idx.data(), s->link_type.data()};
    hgx_graph* g = graph_create(&d, device, false);
    struct Guard {
        hgx_graph* g;
        ~Guard() { if (g) graph_release(g); }
    } guard{g};
    ShardInfo* sh = new ShardInfo();
    g->shard = sh;
    sh->n_parts = s->n_parts;
    sh->part = s->part;
    sh->A_global = s->A_global;
    sh->n_owned = s->n_owned;
    sh->l2g_host = s->l2g;
    sh->present_host = s->present;
    sh->own_bm_host = s->own_bm;
    sh->ghost_count = s->ghost_count;
    sh->bc_count = s->bc_count;
    auto up = [&](auto*& dst, const auto& v, size_t min_n) {
        using T = typename std::remove_reference<decltype(v)>::type::value_type;
        const size_t n = std::max(v.size(), min_n);
        HGX_HIP(hipMalloc(&dst, sizeof(T) * std::max<size_t>(n, 1)));
        if (!v.empty())
            HGX_HIP(hipMemcpyAsync(dst, v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice, g->stream));
    };
    up(sh->own_bm, s->own_bm, 1);
    up(sh->xo_part, s->xo_part, 1);
    up(sh->xo_lid, s->xo_lid, 1);
    up(sh->bc_off, s->bc_off, 1);
    up(sh->bc_part, s->bc_part, 1);
    up(sh->bc_lid, s->bc_lid, 1);
    {   // static broadcast slots: rank of an owned atom among my owned atoms held by a holder (ascending
        // local ids = ascending global ids on every part); the ghost counts are checked with them
        std::vector<int32_t> bc_slot(s->bc_part.size(), -1),
            bc_atom(s->bc_part.size(), -1);
        std::vector<int64_t> c1((size_t)s->n_parts, 0), c2((size_t)s->n_parts, 0);
        for (size_t i = 0; i < s->xo_part.size(); ++i) {
            const int32_t q = s->xo_part[i];
            if (q >= 0) ++c1[(size_t)q];
            for (int64_t k = s->bc_off[i]; k < s->bc_off[i + 1]; ++k) {
                bc_slot[(size_t)k] = (int32_t)c2[(size_t)s->bc_part[(size_t)k]]++;
                bc_atom[(size_t)k] = (int32_t)i;
            }
        }
        for (int q = 0; q < s->n_parts; ++q)
            if (c1[(size_t)q] != s->ghost_count[(size_t)q] || c2[(size_t)q] != s->bc_count[(size_t)q])
                fail(HGX_E_INVALID, "hgx_shard_graph_create: inconsistent exchange tables");
        up(sh->bc_slot, bc_slot, 1);
        up(sh->bc_atom, bc_atom, 1);
    }
    HGX_HIP(hipStreamSynchronize(g->stream));
    guard.g = nullptr;
    *out = g;
    HGX_API_END
}

int hgx_comm_rccl_unique_id(uint8_t id[128]) {
    HGX_API_BEGIN
    if (!id) fail(HGX_E_INVALID, "null id");
    static_assert(sizeof(ncclUniqueId) == 128, "RCCL unique id size");
    ncclUniqueId u;
    HGX_NCCL(ncclGetUniqueId(&u));
    std::memcpy(id, &u, 128);
    HGX_API_END
}

int hgx_comm_rccl_create(const uint8_t id[128], int32_t world, int32_t rank, int32_t device, hgx_comm** out) {
    HGX_API_BEGIN
    if (!id || !out || world < 1 || rank < 0 || rank >= world) fail(HGX_E_INVALID, "hgx_comm_rccl_create: bad argument");
    *out = nullptr;
    HGX_HIP(hipSetDevice(device));
    std::unique_ptr<RcclTransport> t(new RcclTransport());
    t->world = world;
    t->rank = rank;
    t->device = device;
    ncclUniqueId u;
    std::memcpy(&u, id, 128);
    HGX_NCCL(ncclCommInitRank(&t->comm, world, u, rank));
    hgx_comm* c = new hgx_comm();
    c->t = t.release();
    *out = c;
    HGX_API_END
}

int hgx_comm_host_create(int32_t world, int32_t rank, hgx_host_allgather_fn allgather, hgx_host_alltoallv_fn alltoallv,
                         void* user, hgx_comm** out) {
    HGX_API_BEGIN
    if (!out || !allgather || !alltoallv || world < 1 || rank < 0 || rank >= world)
        fail(HGX_E_INVALID, "hgx_comm_host_create: bad argument");
    *out = nullptr;
    std::unique_ptr<HostTransport> t(new HostTransport());
    t->world = world;
    t->rank = rank;
    t->ag = allgather;
    t->a2a = alltoallv;
    t->user = user;
    hgx_comm* c = new hgx_comm();
    c->t = t.release();
    *out = c;
    HGX_API_END
}

int hgx_comm_check_allgather(hgx_comm* c, int32_t device, const int64_t* values, int64_t n, int64_t* out_dev,
                             int64_t* out_base, int64_t* out_host) {
    HGX_API_BEGIN
    if (!c || !c->t || n < 1 || !values || !out_dev || !out_base || !out_host)
        fail(HGX_E_INVALID, "hgx_comm_check_allgather: bad argument");
    HGX_HIP(hipSetDevice(device));
    Transport* tr = c->t;
    const int64_t need = n * tr->world;
    hipStream_t s = nullptr;
    int64_t* din = nullptr;
    int64_t* pin = nullptr;
    struct Cleanup {
        hipStream_t& s;
        int64_t*& din;
        int64_t*& pin;
        ~Cleanup() {
            if (din) (void)hipFree(din);
            if (pin) (void)hipHostFree(pin);
            if (s) (void)hipStreamDestroy(s);
        }
    } cleanup{s, din, pin};
    HGX_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    HGX_HIP(hipMalloc(&din, sizeof(int64_t) * (size_t)n));
    HGX_HIP(hipHostMalloc(&pin, sizeof(int64_t) * (size_t)need, hipHostMallocDefault));
    HGX_HIP(hipMemcpyAsync(din, values, sizeof(int64_t) * (size_t)n, hipMemcpyHostToDevice, s));
    tr->allgather_dev(din, n, out_dev, s, pin);               // the transport's own (RCCL: device gather)
    tr->Transport::allgather_dev(din, n, out_base, s, pin);   // the default: read back + host all-gather
    tr->allgather_i64(values, n, out_host, s);
    HGX_HIP(hipStreamSynchronize(s));
    HGX_API_END
}

void hgx_comm_destroy(hgx_comm* c) {
    if (!c) return;
    delete c->t;
    delete c;
}

int hgx_pbfs_batch(hgx_graph* shard, hgx_comm* comm, const int32_t* seeds, int32_t n_seeds, int32_t max_depth,
                   const hgx_algen_opts* opts, hgx_bfs_result** out) {
    HGX_API_BEGIN
    if (!shard || !comm || !comm->t || !out || n_seeds < 0 || (n_seeds > 0 && !seeds))
        fail(HGX_E_INVALID, "hgx_pbfs_batch: bad argument");
    *out = nullptr;
    pbfs_run(shard, comm->t, seeds, n_seeds, max_depth, opts, out);
    HGX_API_END
}

int hgx_pbfs_batch_group(hgx_graph* const* shards, int32_t n_parts, const int32_t* seeds, int32_t n_seeds,
                         int32_t max_depth, const hgx_algen_opts* opts, hgx_bfs_result** outs) {
    HGX_API_BEGIN
    if (!shards || !outs || n_parts < 1 || n_seeds < 0 || (n_seeds > 0 && !seeds))
        fail(HGX_E_INVALID, "hgx_pbfs_batch_group: bad argument");
    for (int p = 0; p < n_parts; ++p) {
        outs[p] = nullptr;
        if (!shards[p] || !shards[p]->shard || shards[p]->shard->part != p || shards[p]->shard->n_parts != n_parts)
            fail(HGX_E_INVALID, "hgx_pbfs_batch_group: shards[p] must be part p of n_parts");
    }
    auto hub = std::make_shared<LocalHub>(n_parts);
    for (int p = 0; p < n_parts; ++p) hub->serial |= shards[p]->shard->serial;
    std::vector<std::unique_ptr<LocalTransport>> tr(n_parts);
    for (int p = 0; p < n_parts; ++p) {
        tr[p].reset(new LocalTransport());
        tr[p]->world = n_parts;
        tr[p]->rank = p;
        tr[p]->device = shards[p]->device;
        tr[p]->hub = hub;
    }
    std::vector<int> rc(n_parts, HGX_OK);
    std::vector<std::string> msg(n_parts);
    std::vector<std::thread> th;
    for (int p = 0; p < n_parts; ++p)
        th.emplace_back([&, p] {
            try {
                pbfs_run(shards[p], tr[p].get(), seeds, n_seeds, max_depth, opts, &outs[p]);
            } catch (const Error& e) {
                rc[p] = e.code;
                msg[p] = e.msg;
                hub->abort();
            } catch (const std::exception& e) {
                rc[p] = HGX_E_DEVICE;
                msg[p] = e.what();
                hub->abort();
            }
        });
    for (auto& x : th) x.join();
    for (int p = 0; p < n_parts; ++p)
        if (rc[p] != HGX_OK) {
            for (int q = 0; q < n_parts; ++q) {
                hgx_bfs_result_free(outs[q]);
                outs[q] = nullptr;
            }
            // report the root failure, not the secondary "aborted by another part"
            int k = p;
            for (int q = 0; q < n_parts; ++q)
                if (rc[q] != HGX_OK && msg[q].find("aborted by another part") == std::string::npos) {
                    k = q;
                    break;
                }
            fail(rc[k], "part " + std::to_string(k) + ": " + msg[k]);
        }
    HGX_API_END
}

}  // extern "C"
