// hgx_part.hip -- hash partition of a snapshot over n_parts devices and the transports of the
// partitioned BFS.
//
// The reference keeps one incidence index per store (HGStore.getIncidenceResultSet,
// C/HGStore.java:253; BJEStorageImplementation.java:405-439).  Config 4 (1B incidences) is split
// by atom: owner(a) = a % n_parts.  Part p keeps
//   * every atom it owns (the incidence rows of owned atoms are complete on p),
//   * every link with at least one owned target (target rows replicated, at most arity copies),
//   * the ghosts: atoms owned elsewhere that are targets of a local link.
// Owned atoms with no incidence (no link targets them, e.g. the link atoms of config 4) get no
// local id and no device rows: they are reachable only as seeds.
// Local ids follow global id order, so ascending local lists are ascending global lists and the
// on-device incidence build of hgx_graph_create applies unchanged.
//
// Transports: RCCL (grouped ncclSend/ncclRecv over xGMI, one process per GPU) and an in-process
// group (one host thread per part, device-to-device copies) used by hgx_pbfs_batch_group.
#include <rccl/rccl.h>

#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <memory>
#include <thread>

#include "hgx_internal.h"

using namespace hgx;

struct hgx_shard {
    int32_t n_parts = 1, part = 0;
    int64_t A_global = 0, n_owned = 0;
    std::vector<int32_t> l2g, own_l;
    std::vector<int32_t> link_atom, link_type, tgt_idx;
    std::vector<int64_t> tgt_off, ghost_count;
};

namespace {

int host_threads() {
    unsigned n = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(n, 16u));
}

// fn(lo, hi) over [0, n) split into contiguous chunks, one per thread.
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

hgx_shard* shard_build(const hgx_graph_desc* d, int32_t NP, int32_t part) {
    const int64_t A = d->num_atoms, M = d->num_links;
    if (A < 0 || M < 0 || A >= (int64_t)INT32_MAX) fail(HGX_E_INVALID, "hgx_shard_build: bad sizes");
    if (M > 0 && (!d->tgt_off || !d->tgt_idx || !d->link_atom)) fail(HGX_E_INVALID, "hgx_shard_build: null link arrays");
    if (NP < 1 || NP > 64 || part < 0 || part >= NP) fail(HGX_E_INVALID, "hgx_shard_build: bad part / n_parts (1..64)");
    const int64_t* off = d->tgt_off;
    const int32_t* tg = d->tgt_idx;
    if (M > 0 && off[0] != 0) fail(HGX_E_INVALID, "hgx_shard_build: tgt_off[0] != 0");
    std::unique_ptr<hgx_shard> s(new hgx_shard());
    s->n_parts = NP;
    s->part = part;
    s->A_global = A;

    // 1. local links (an owned target) and the atoms they touch
    std::vector<uint8_t> loc((size_t)M), mark((size_t)A, 0);
    std::vector<int> bad(64, 0);
    parallel_for(M, [&](int64_t lo, int64_t hi, int t) {
        for (int64_t r = lo; r < hi; ++r) {
            const int64_t b = off[r], e = off[r + 1];
            if (e < b) {
                bad[t] = 1;
                continue;
            }
            bool any = false;
            for (int64_t p = b; p < e; ++p) {
                const int32_t v = tg[p];
                if (v < 0 || v >= A) {
                    bad[t] = 2;
                    break;
                }
                any |= (v % NP) == part;
            }
            loc[r] = any;
        }
    });
    for (int b : bad)
        if (b == 1) fail(HGX_E_INVALID, "hgx_shard_build: tgt_off not monotone");
        else if (b == 2) fail(HGX_E_INVALID, "hgx_shard_build: target id out of range");
    // Owned atoms that no link targets are left out of the local space: BFS can reach them only
    // as seeds (V_0 = {seed}), which the result records on the host (bfs_batch_impl).
    parallel_for(M, [&](int64_t lo, int64_t hi, int) {
        for (int64_t r = lo; r < hi; ++r)
            if (loc[r])
                for (int64_t p = off[r]; p < off[r + 1]; ++p) mark[tg[p]] = 1;   // benign same-value races
    });

    // 2. global -> local ids (prefix over the marks, in global order)
    std::vector<int32_t> g2l((size_t)A);
    {
        const int T = host_threads();
        std::vector<int64_t> cnt(T + 1, 0);
        const int64_t per = (A + T - 1) / std::max(T, 1);
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
            th.emplace_back([&, t] {
                int64_t c = 0;
                for (int64_t a = t * per; a < std::min(A, (t + 1) * per); ++a) c += mark[a];
                cnt[t + 1] = c;
            });
        for (auto& x : th) x.join();
        th.clear();
        for (int t = 0; t < T; ++t) cnt[t + 1] += cnt[t];
        s->l2g.resize((size_t)cnt[T]);
        for (int t = 0; t < T; ++t)
            th.emplace_back([&, t] {
                int64_t k = cnt[t];
                for (int64_t a = t * per; a < std::min(A, (t + 1) * per); ++a) {
                    if (mark[a]) {
                        g2l[a] = (int32_t)k;
                        s->l2g[k++] = (int32_t)a;
                    } else {
                        g2l[a] = -1;
                    }
                }
            });
        for (auto& x : th) x.join();
    }
    const int64_t AL = (int64_t)s->l2g.size();
    s->n_owned = A > part ? (A - part + NP - 1) / NP : 0;
    s->own_l.resize((size_t)s->n_owned);
    for (int64_t k = 0; k < s->n_owned; ++k) s->own_l[k] = g2l[part + k * NP];   // -1: isolated
    s->ghost_count.assign(NP, 0);
    for (int64_t i = 0; i < AL; ++i) {
        const int o = s->l2g[i] % NP;
        if (o != part) s->ghost_count[o]++;
    }

    // 3. local link rows (ascending global row order) with targets in local ids
    std::vector<int64_t> lrow;
    lrow.reserve((size_t)(M / std::max(NP, 1) + 16));
    for (int64_t r = 0; r < M; ++r)
        if (loc[r]) lrow.push_back(r);
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
            for (int64_t p = off[r]; p < off[r + 1]; ++p) s->tgt_idx[o++] = g2l[tg[p]];
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
        HGX_HIP(hipStreamSynchronize(s));
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
        hub->barrier();   // every part has pulled its segments: send buffers may be reused
        (void)send_bytes;
    }
};

}  // namespace

extern "C" {

int hgx_shard_build(const hgx_graph_desc* global, int32_t n_parts, int32_t part, hgx_shard** out) {
    HGX_API_BEGIN
    if (!global || !out) fail(HGX_E_INVALID, "hgx_shard_build: null argument");
    *out = nullptr;
    *out = shard_build(global, n_parts, part);
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
    if (l2g) std::memcpy(l2g, s->l2g.data(), sizeof(int32_t) * s->l2g.size());
    if (link_atom) std::memcpy(link_atom, s->link_atom.data(), sizeof(int32_t) * s->link_atom.size());
    if (link_type) std::memcpy(link_type, s->link_type.data(), sizeof(int32_t) * s->link_type.size());
    if (tgt_off) std::memcpy(tgt_off, s->tgt_off.data(), sizeof(int64_t) * s->tgt_off.size());
    if (tgt_idx) std::memcpy(tgt_idx, s->tgt_idx.data(), sizeof(int32_t) * s->tgt_idx.size());
    if (ghost_count) std::memcpy(ghost_count, s->ghost_count.data(), sizeof(int64_t) * s->ghost_count.size());
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
    sh->own_l_host = s->own_l;
    sh->ghost_count = s->ghost_count;
    sh->ghost_start.assign(s->n_parts + 1, 0);
    for (int p = 0; p < s->n_parts; ++p) sh->ghost_start[p + 1] = sh->ghost_start[p] + s->ghost_count[p];
    sh->n_ghost = sh->ghost_start[s->n_parts];
    std::vector<uint64_t> own((size_t)(AL / 64 + 2), 0);
    for (int64_t i = 0; i < AL; ++i)
        if (s->l2g[i] % s->n_parts == s->part) own[i >> 6] |= 1ull << (i & 63);
    HGX_HIP(hipMalloc(&sh->l2g, sizeof(int32_t) * std::max<int64_t>(AL, 1)));
    HGX_HIP(hipMalloc(&sh->own_l, sizeof(int32_t) * std::max<int64_t>(s->n_owned, 1)));
    HGX_HIP(hipMalloc(&sh->own_bm, sizeof(uint64_t) * own.size()));
    if (AL) HGX_HIP(hipMemcpyAsync(sh->l2g, s->l2g.data(), sizeof(int32_t) * AL, hipMemcpyHostToDevice, g->stream));
    if (s->n_owned)
        HGX_HIP(hipMemcpyAsync(sh->own_l, s->own_l.data(), sizeof(int32_t) * s->n_owned, hipMemcpyHostToDevice,
                               g->stream));
    HGX_HIP(hipMemcpyAsync(sh->own_bm, own.data(), sizeof(uint64_t) * own.size(), hipMemcpyHostToDevice, g->stream));
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
