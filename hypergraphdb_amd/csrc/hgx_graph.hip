// hgx_graph.hip -- snapshot upload and on-device incidence-index build.
//
// Replaces the reference's per-call incidence materialisation
// (HyperGraph.getIncidenceSet C/HyperGraph.java:1415-1418 -> ISRefResolver C/ISRefResolver.java:72-105
//  -> BJEStorageImplementation.getIncidenceResultSet storage/bdb-je/.../BJEStorageImplementation.java:405-439)
// with one device-resident CSR built once per snapshot: pins are keyed (target << 32 | link row),
// radix-sorted on the GPU, de-duplicated (putNoDupData, :300-307) and cut into rows.
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <cstring>
#include <new>

#include "hgx_internal.h"

namespace hgx {

static thread_local std::string t_last_error;

void set_last_error(const std::string& msg) { t_last_error = msg; }
[[noreturn]] void fail(int code, const std::string& msg) { throw Error{code, msg}; }

void graph_release(hgx_graph* g) {
    if (!g) return;
    if (g->refs.fetch_sub(1) != 1) return;
    (void)hipSetDevice(g->device);
    if (g->stream) (void)hipStreamSynchronize(g->stream);
    for (auto& b : g->pool) (void)hipFree(b.p);
    g->pool.clear();
    for (auto e : g->ev_pool) (void)hipEventDestroy(e);
    g->ev_pool.clear();
    for (auto e : g->pend_ev)
        if (e) (void)hipEventDestroy(e);
    // a context (hgx_graph_context) frees what it built itself, never an array borrowed from its base
    hgx_graph* const b = g->base;
#define HGX_FREE_OWN(f) \
    if (g->f && (!b || (const void*)g->f != (const void*)b->f)) (void)hipFree(g->f)
    HGX_FREE_OWN(link_atom); HGX_FREE_OWN(tgt_off); HGX_FREE_OWN(tgt_idx); HGX_FREE_OWN(link_type);
    HGX_FREE_OWN(inc_off); HGX_FREE_OWN(inc_row); HGX_FREE_OWN(inc_type); HGX_FREE_OWN(inc_ts_row);
    HGX_FREE_OWN(inc_ts_type); HGX_FREE_OWN(inc_ts_tgt); HGX_FREE_OWN(heavy_atom); HGX_FREE_OWN(chunks);
    HGX_FREE_OWN(hasinc); HGX_FREE_OWN(inc_yf); HGX_FREE_OWN(pchunks);
#undef HGX_FREE_OWN
    if (g->zacc) (void)hipFree(g->zacc);
    if (g->q_ticket) (void)hipFree(g->q_ticket);
    if (g->co_vis) (void)hipFree(g->co_vis);
    if (g->sc_tab) (void)hipFree(g->sc_tab);
    free_yield_lists(g);
    for (auto& b : g->seq_hbufs) (void)hipHostFree(b.p);
    g->seq_hbufs.clear();
    if (g->pinned) (void)hipHostFree(g->pinned);
    if (g->ctr_host) (void)hipHostFree(g->ctr_host);
    if (g->seq_flag) (void)hipHostFree(g->seq_flag);
    for (hipEvent_t& e : g->ls_ev)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t& e : g->ls_cev)
        if (e) (void)hipEventDestroy(e);
    if (g->mapped) (void)hipHostFree(g->mapped);
    if (g->zc_in) (void)hipHostFree(g->zc_in);
    if (g->stream2) (void)hipStreamSynchronize(g->stream2);
    if (g->stream3) (void)hipStreamSynchronize(g->stream3);
    if (g->ev_count) (void)hipEventDestroy(g->ev_count);
    if (g->stream2) (void)hipStreamDestroy(g->stream2);
    if (g->stream3) (void)hipStreamDestroy(g->stream3);
    if (g->stream) (void)hipStreamDestroy(g->stream);
    if (g->shard) {
        (void)hipFree(g->shard->own_bm); (void)hipFree(g->shard->xo_part); (void)hipFree(g->shard->xo_lid);
        (void)hipFree(g->shard->bc_off); (void)hipFree(g->shard->bc_part); (void)hipFree(g->shard->bc_lid);
        (void)hipFree(g->shard->bc_slot);
        (void)hipFree(g->shard->bc_atom);
        delete g->shard;
    }
    delete g;
    if (b) graph_release(b);   // the context's reference on its snapshot
}

// ---------------------------------------------------------------------------------------------
// Kernels
// ---------------------------------------------------------------------------------------------

// One key per (target, link row); a target repeated inside one link keeps its first
// position only (putNoDupData).  Repeats become UINT64_MAX and sort to the end.
__global__ void __launch_bounds__(256) k_pin_keys(int64_t M, const int64_t* __restrict__ tgt_off,
                                                  const int32_t* __restrict__ tgt_idx,
                                                  uint64_t* __restrict__ keys,
                                                  unsigned long long* __restrict__ n_dup) {
    unsigned long long dups = 0;
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < M;
         r += (int64_t)gridDim.x * blockDim.x) {
        int64_t b = tgt_off[r], e = tgt_off[r + 1];
        for (int64_t p = b; p < e; ++p) {
            int32_t t = tgt_idx[p];
            bool dup = false;
            for (int64_t q = b; q < p; ++q) dup |= (tgt_idx[q] == t);
            keys[p] = dup ? ~0ull : (((uint64_t)(uint32_t)t << 32) | (uint32_t)r);
            dups += dup;
        }
    }
    if (dups) atomicAdd(n_dup, dups);
}

// inc_type[i] = link_type[inc_row[i]]
__global__ void __launch_bounds__(256) k_inc_type(int64_t I, const int32_t* __restrict__ inc_row,
                                                  const int32_t* __restrict__ link_type, int32_t* __restrict__ inc_type) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < I; i += (int64_t)gridDim.x * blockDim.x)
        inc_type[i] = link_type[inc_row[i]];
}

// inc_row[i] = low word of key i.
__global__ void __launch_bounds__(256) k_cut_rows(int64_t I, const uint64_t* __restrict__ keys,
                                                  int32_t* __restrict__ inc_row) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < I; i += (int64_t)gridDim.x * blockDim.x)
        inc_row[i] = (int32_t)(uint32_t)keys[i];
}

// inc_off[a] = first i with (keys[i] >> 32) >= a  (binary search per atom; a in [0, A])
__global__ void __launch_bounds__(256) k_row_offsets(int64_t I, int64_t A, const uint64_t* __restrict__ keys,
                                                     int64_t* __restrict__ inc_off) {
    for (int64_t a = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; a <= A; a += (int64_t)gridDim.x * blockDim.x) {
        int64_t lo = 0, hi = I;
        const uint64_t key = (uint64_t)a << 32;
        while (lo < hi) {
            int64_t mid = (lo + hi) >> 1;
            if (keys[mid] < key) lo = mid + 1; else hi = mid;
        }
        inc_off[a] = lo;
    }
}

__global__ void __launch_bounds__(256) k_validate(int64_t A, int64_t M, const int32_t* __restrict__ link_atom,
                                                  const int64_t* __restrict__ tgt_off,
                                                  const int32_t* __restrict__ tgt_idx, int64_t P,
                                                  unsigned int* __restrict__ bad, int links_are_atoms) {
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < M;
         r += (int64_t)gridDim.x * blockDim.x) {
        int32_t la = link_atom[r];
        if (la < 0 || (links_are_atoms && la >= A) || (r > 0 && link_atom[r - 1] >= la)) atomicOr(bad, 1u);
        if (tgt_off[r] > tgt_off[r + 1] || tgt_off[r + 1] > P) atomicOr(bad, 2u);
    }
    for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < P;
         p += (int64_t)gridDim.x * blockDim.x) {
        int32_t t = tgt_idx[p];
        if (t < 0 || t >= A) atomicOr(bad, 4u);
    }
}

__global__ void k_degrees(int32_t n, const int32_t* __restrict__ atoms, const int64_t* __restrict__ inc_off,
                          int64_t A, int64_t* __restrict__ out) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        int32_t a = atoms[i];
        out[i] = (a >= 0 && a < A) ? inc_off[a + 1] - inc_off[a] : -1;
    }
}

__global__ void k_rows_to_atoms(int64_t n, const int32_t* __restrict__ rows, const int32_t* __restrict__ link_atom,
                                int32_t* __restrict__ out) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = link_atom[rows[i]];
}

// heavy atoms: deg > kHeavyDegree (order-free compaction; the chunk table is rebuilt on host)
__global__ void __launch_bounds__(256) k_find_heavy(int64_t A, const int64_t* __restrict__ inc_off, int64_t thr,
                                                    int32_t* __restrict__ out, unsigned int* __restrict__ n) {
    for (int64_t a = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; a < A; a += (int64_t)gridDim.x * blockDim.x)
        if (inc_off[a + 1] - inc_off[a] > thr) out[atomicAdd(n, 1u)] = (int32_t)a;
}

// out[i] = inc_off[atoms[i]], out[n + i] = deg(atoms[i])
__global__ void k_ranges(int32_t n, const int32_t* __restrict__ atoms, const int64_t* __restrict__ inc_off,
                         int64_t* __restrict__ out) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        int64_t b = inc_off[atoms[i]];
        out[i] = b;
        out[n + i] = inc_off[atoms[i] + 1] - b;
    }
}

}  // namespace hgx

using namespace hgx;

// ---------------------------------------------------------------------------------------------
// Pool
// ---------------------------------------------------------------------------------------------

void* hgx_graph::alloc(size_t bytes) {
    if (bytes == 0) bytes = 256;
    bytes = (bytes + 255) & ~(size_t)255;
    size_t best = (size_t)-1;
    for (size_t i = 0; i < pool.size(); ++i)
        if (pool[i].n >= bytes && pool[i].n <= 2 * bytes && (best == (size_t)-1 || pool[i].n < pool[best].n))
            best = i;
    if (best != (size_t)-1) {
        void* p = pool[best].p;
        pool.erase(pool.begin() + best);
        return p;
    }
    void* p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipStreamSynchronize(stream);
        for (auto& b : pool) (void)hipFree(b.p);
        pool.clear();
        if (hipMalloc(&p, bytes) != hipSuccess) {
            (void)hipGetLastError();
            fail(HGX_E_NOMEM, "hipMalloc of " + std::to_string(bytes) + " bytes failed");
        }
    }
    return p;
}

void hgx_graph::release(void* p, size_t bytes) {
    if (!p) return;
    if (bytes == 0) bytes = 256;
    bytes = (bytes + 255) & ~(size_t)255;
    pool.push_back({p, bytes});
}

void* hgx_graph::pinned_buf(size_t bytes) {
    if (bytes > pinned_bytes) {
        if (pinned) (void)hipHostFree(pinned);
        pinned = nullptr;
        size_t n = std::max<size_t>(bytes, 1 << 16);
        HGX_HIP(hipHostMalloc(&pinned, n, hipHostMallocDefault));
        pinned_bytes = n;
    }
    return pinned;
}

void* hgx_graph::mapped_buf(size_t bytes) {
    if (bytes > mapped_bytes) {
        if (mapped) (void)hipHostFree(mapped);
        mapped = nullptr;
        mapped_bytes = 0;
        const size_t n = std::max<size_t>(bytes + bytes / 4, 1 << 16);
        HGX_HIP(hipHostMalloc(&mapped, n, hipHostMallocMapped));
        mapped_bytes = n;
    }
    return mapped;
}

void* hgx_graph::zc_in_buf(size_t bytes) {
    if (bytes > zc_in_bytes) {
        if (zc_in) (void)hipHostFree(zc_in);
        zc_in = zc_in_dev = nullptr;
        zc_in_bytes = 0;
        const size_t n = std::max<size_t>(bytes + bytes / 4, 1 << 16);
        HGX_HIP(hipHostMalloc(&zc_in, n, hipHostMallocMapped | hipHostMallocCoherent));
        zc_in_bytes = n;
        HGX_HIP(hipHostGetDevicePointer(&zc_in_dev, zc_in, 0));
    }
    return zc_in;
}

// ---------------------------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------------------------

extern "C" {

const char* hgx_version(void) { return "hgx 0.1.0 (gfx950)"; }

const char* hgx_last_error(void) { return t_last_error.c_str(); }

int hgx_device_synchronize(int32_t device) {
    HGX_API_BEGIN
    HGX_HIP(hipSetDevice(device));
    HGX_HIP(hipDeviceSynchronize());
    HGX_API_END
}

int hgx_device_count(int32_t* n) {
    HGX_API_BEGIN
    if (!n) fail(HGX_E_INVALID, "hgx_device_count: null argument");
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;   // no GPU / no driver: zero devices
    *n = (int32_t)c;
    HGX_API_END
}

int hgx_graph_create(const hgx_graph_desc* d, int32_t device, hgx_graph** out) {
    HGX_API_BEGIN
    if (!d || !out) fail(HGX_E_INVALID, "hgx_graph_create: null argument");
    *out = nullptr;
    *out = graph_create(d, device, true);
    HGX_API_END
}

int hgx_graph_context(hgx_graph* g, hgx_graph** out) {
    HGX_API_BEGIN
    if (!g || !out) fail(HGX_E_INVALID, "hgx_graph_context: null argument");
    *out = nullptr;
    if (g->base) g = g->base;   // a context of a context is another context of the snapshot
    if (g->shard)
        fail(HGX_E_UNSUPPORTED, "hgx_graph_context: a partition shard runs one collective traversal at a time");
    std::lock_guard<std::mutex> lk(g->mu);
    HGX_HIP(hipSetDevice(g->device));
    bfs_shared_tables(g);   // built once on the snapshot, read by every context
    hgx_graph* c = new hgx_graph();
    c->base = g;
    g->refs.fetch_add(1);
    struct Guard {
        hgx_graph* c;
        ~Guard() { if (c) graph_release(c); }
    } guard{c};
    c->device = g->device;
    HGX_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    // the snapshot (borrowed)
    c->A = g->A; c->M = g->M; c->P = g->P; c->I = g->I;
    c->link_atom = g->link_atom; c->tgt_off = g->tgt_off; c->tgt_idx = g->tgt_idx; c->link_type = g->link_type;
    c->inc_off = g->inc_off; c->inc_row = g->inc_row; c->inc_type = g->inc_type;
    c->inc_ts_row = g->inc_ts_row; c->inc_ts_type = g->inc_ts_type; c->inc_ts_tgt = g->inc_ts_tgt;
    c->n_heavy = g->n_heavy; c->I_heavy = g->I_heavy; c->n_chunks = g->n_chunks;
    c->heavy_atom = g->heavy_atom; c->chunks = g->chunks;
    c->hasinc = g->hasinc; c->inc_yf = g->inc_yf; c->pchunks = g->pchunks; c->n_pchunks = g->n_pchunks;
    c->max_arity = g->max_arity; c->max_deg = g->max_deg;
    // the snapshot's options at this point (set separately on the context afterwards)
    c->timing = g->timing; c->bfs_flags = g->bfs_flags; c->seq_budget_bytes = g->seq_budget_bytes;
    c->seq_engine = g->seq_engine;
    c->bfs_block = g->bfs_block;
    c->co_timeout = g->co_timeout;
    c->seq_pull = g->seq_pull;
    c->seq_small = g->seq_small;
    c->seq_tlimit = g->seq_tlimit;
    c->seq_pack_min = g->seq_pack_min;
    c->xb_flat = g->xb_flat;
    c->xb_static = g->xb_static;
    c->ranks_ordered = g->ranks_ordered; c->q_inline = g->q_inline;
    c->q_coalesce = g->q_coalesce; c->q_coalesce_max = g->q_coalesce_max;
    guard.c = nullptr;
    *out = c;
    HGX_API_END
}

}  // extern "C"

hgx_graph* hgx::graph_create(const hgx_graph_desc* d, int32_t device, bool links_are_atoms) {
    if (d->num_atoms < 0 || d->num_links < 0 || (links_are_atoms && d->num_links > d->num_atoms))
        fail(HGX_E_INVALID, "hgx_graph_create: bad sizes");
    if (d->num_atoms >= (int64_t)INT32_MAX) fail(HGX_E_INVALID, "hgx_graph_create: more than 2^31-1 atoms");
    if (d->num_links > 0 && (!d->link_atom || !d->tgt_off || !d->tgt_idx))
        fail(HGX_E_INVALID, "hgx_graph_create: null link arrays");
    int ndev = 0;
    HGX_HIP(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) fail(HGX_E_INVALID, "hgx_graph_create: no such device");
    HGX_HIP(hipSetDevice(device));

    hgx_graph* g = new hgx_graph();
    struct Guard {
        hgx_graph* g;
        ~Guard() { if (g) graph_release(g); }
    } guard{g};
    g->device = device;
    HGX_HIP(hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking));
    const int64_t A = d->num_atoms, M = d->num_links;
    const int64_t P = M > 0 ? d->tgt_off[M] : 0;
    if (M > 0 && d->tgt_off[0] != 0) fail(HGX_E_INVALID, "hgx_graph_create: tgt_off[0] != 0");
    if (P < 0 || P >= ((int64_t)1 << 40)) fail(HGX_E_INVALID, "hgx_graph_create: bad pin count");
    g->A = A; g->M = M; g->P = P;
    hipStream_t s = g->stream;

    HGX_HIP(hipMalloc(&g->link_atom, sizeof(int32_t) * std::max<int64_t>(M, 1)));
    HGX_HIP(hipMalloc(&g->tgt_off, sizeof(int64_t) * (M + 1)));
    HGX_HIP(hipMalloc(&g->tgt_idx, sizeof(int32_t) * std::max<int64_t>(P, 1)));
    HGX_HIP(hipMalloc(&g->link_type, sizeof(int32_t) * std::max<int64_t>(M, 1)));
    HGX_HIP(hipMalloc(&g->inc_off, sizeof(int64_t) * (A + 1)));
    if (M > 0) {
        HGX_HIP(hipMemcpyAsync(g->link_atom, d->link_atom, sizeof(int32_t) * M, hipMemcpyHostToDevice, s));
        HGX_HIP(hipMemcpyAsync(g->tgt_off, d->tgt_off, sizeof(int64_t) * (M + 1), hipMemcpyHostToDevice, s));
        if (P > 0)
            HGX_HIP(hipMemcpyAsync(g->tgt_idx, d->tgt_idx, sizeof(int32_t) * P, hipMemcpyHostToDevice, s));
        if (d->link_type)
            HGX_HIP(hipMemcpyAsync(g->link_type, d->link_type, sizeof(int32_t) * M, hipMemcpyHostToDevice, s));
        else
            HGX_HIP(hipMemsetAsync(g->link_type, 0, sizeof(int32_t) * M, s));
    } else {
        int64_t z = 0;
        HGX_HIP(hipMemcpyAsync(g->tgt_off, &z, sizeof(int64_t), hipMemcpyHostToDevice, s));
    }
    // validation on device (ids in range, strictly ascending link ranks, monotone offsets)
    unsigned int* bad = (unsigned int*)g->alloc(sizeof(unsigned int) + sizeof(unsigned long long));
    unsigned long long* ndup = (unsigned long long*)((char*)bad + 8);
    HGX_HIP(hipMemsetAsync(bad, 0, 16, s));
    if (M > 0) {
        k_validate<<<grid_for(std::max(M, P), 256), 256, 0, s>>>(A, M, g->link_atom, g->tgt_off, g->tgt_idx, P, bad,
                                                                 links_are_atoms ? 1 : 0);
        HGX_CHECK_LAUNCH();
    }
    unsigned int hbad = 0;
    HGX_HIP(hipMemcpyAsync(&hbad, bad, sizeof(hbad), hipMemcpyDeviceToHost, s));
    HGX_HIP(hipStreamSynchronize(s));
    if (hbad & 1u) fail(HGX_E_INVALID, "hgx_graph_create: link_atom not strictly ascending / out of range");
    if (hbad & 2u) fail(HGX_E_INVALID, "hgx_graph_create: tgt_off not monotone");
    if (hbad & 4u) fail(HGX_E_INVALID, "hgx_graph_create: target id out of range");

    // incidence index: key sort on the device
    int64_t I = 0;
    if (P > 0) {
        uint64_t* keys = (uint64_t*)g->alloc(sizeof(uint64_t) * P);
        uint64_t* sorted = (uint64_t*)g->alloc(sizeof(uint64_t) * P);
        k_pin_keys<<<grid_for(M, 256), 256, 0, s>>>(M, g->tgt_off, g->tgt_idx, keys, ndup);
        HGX_CHECK_LAUNCH();
        int end_bit = 64;
        {
            int ab = 1;
            while (((int64_t)1 << ab) <= A) ab++;
            end_bit = 32 + ab;            // UINT64_MAX sentinels still sort last
            if (end_bit > 64) end_bit = 64;
        }
        size_t tmp_bytes = 0;   // rocPRIM takes 64-bit sizes: no 2^31-1 pin limit
        HGX_HIP(rocprim::radix_sort_keys(nullptr, tmp_bytes, keys, sorted, (size_t)P, 0u, (unsigned)end_bit, s));
        void* tmp = g->alloc(tmp_bytes);
        HGX_HIP(rocprim::radix_sort_keys(tmp, tmp_bytes, keys, sorted, (size_t)P, 0u, (unsigned)end_bit, s));
        unsigned long long hdup = 0;
        HGX_HIP(hipMemcpyAsync(&hdup, ndup, sizeof(hdup), hipMemcpyDeviceToHost, s));
        HGX_HIP(hipStreamSynchronize(s));
        I = P - (int64_t)hdup;
        HGX_HIP(hipMalloc(&g->inc_row, sizeof(int32_t) * std::max<int64_t>(I, 1)));
        k_cut_rows<<<grid_for(I, 256), 256, 0, s>>>(I, sorted, g->inc_row);
        HGX_CHECK_LAUNCH();
        k_row_offsets<<<grid_for(A + 1, 256), 256, 0, s>>>(I, A, sorted, g->inc_off);
        HGX_CHECK_LAUNCH();
        HGX_HIP(hipStreamSynchronize(s));
        g->release(tmp, tmp_bytes);
        g->release(keys, sizeof(uint64_t) * P);
        g->release(sorted, sizeof(uint64_t) * P);
    } else {
        HGX_HIP(hipMalloc(&g->inc_row, sizeof(int32_t)));
        HGX_HIP(hipMemsetAsync(g->inc_off, 0, sizeof(int64_t) * (A + 1), s));
    }
    g->I = I;
    HGX_HIP(hipMalloc(&g->inc_type, sizeof(int32_t) * std::max<int64_t>(I, 1)));
    if (I > 0) {
        k_inc_type<<<grid_for(I, 256), 256, 0, s>>>(I, g->inc_row, g->link_type, g->inc_type);
        HGX_CHECK_LAUNCH();
    }

    // heavy atoms + chunk table (load balance for power-law incidence rows)
    {
        int32_t* dheavy = (int32_t*)g->alloc(sizeof(int32_t) * std::max<int64_t>(A, 1));
        HGX_HIP(hipMemsetAsync(bad, 0, 4, s));
        k_find_heavy<<<grid_for(A, 256), 256, 0, s>>>(A, g->inc_off, kHeavyDegree, dheavy, bad);
        HGX_CHECK_LAUNCH();
        unsigned int nh = 0;
        HGX_HIP(hipMemcpyAsync(&nh, bad, 4, hipMemcpyDeviceToHost, s));
        HGX_HIP(hipStreamSynchronize(s));
        std::vector<int32_t> heavy(nh);
        if (nh) HGX_HIP(hipMemcpyAsync(heavy.data(), dheavy, sizeof(int32_t) * nh, hipMemcpyDeviceToHost, s));
        HGX_HIP(hipStreamSynchronize(s));
        std::sort(heavy.begin(), heavy.end());
        std::vector<int64_t> hb(nh), hd(nh);
        if (nh) {
            int32_t* dh = (int32_t*)g->alloc(sizeof(int32_t) * nh);
            int64_t* dr = (int64_t*)g->alloc(sizeof(int64_t) * 2 * nh);
            HGX_HIP(hipMemcpyAsync(dh, heavy.data(), sizeof(int32_t) * nh, hipMemcpyHostToDevice, s));
            k_ranges<<<grid_for(nh, 256), 256, 0, s>>>((int32_t)nh, dh, g->inc_off, dr);
            HGX_CHECK_LAUNCH();
            HGX_HIP(hipMemcpyAsync(hb.data(), dr, sizeof(int64_t) * nh, hipMemcpyDeviceToHost, s));
            HGX_HIP(hipMemcpyAsync(hd.data(), dr + nh, sizeof(int64_t) * nh, hipMemcpyDeviceToHost, s));
            HGX_HIP(hipStreamSynchronize(s));
            g->release(dh, sizeof(int32_t) * nh);
            g->release(dr, sizeof(int64_t) * 2 * nh);
        }
        std::vector<HeavyChunk> ch;
        for (unsigned int h = 0; h < nh; ++h)
            for (int64_t b = hb[h]; b < hb[h] + hd[h]; b += kChunkEntries)
                ch.push_back({b, std::min(hb[h] + hd[h], b + kChunkEntries), heavy[h], (int32_t)h});
        g->n_heavy = nh;
        g->I_heavy = 0;
        for (unsigned int h = 0; h < nh; ++h) g->I_heavy += hd[h];
        g->n_chunks = (int64_t)ch.size();
        HGX_HIP(hipMalloc(&g->heavy_atom, sizeof(int32_t) * std::max<int64_t>(nh, 1)));
        HGX_HIP(hipMalloc(&g->chunks, sizeof(HeavyChunk) * std::max<int64_t>(g->n_chunks, 1)));
        if (nh) HGX_HIP(hipMemcpyAsync(g->heavy_atom, heavy.data(), sizeof(int32_t) * nh, hipMemcpyHostToDevice, s));
        if (!ch.empty())
            HGX_HIP(hipMemcpyAsync(g->chunks, ch.data(), sizeof(HeavyChunk) * ch.size(), hipMemcpyHostToDevice, s));
        HGX_HIP(hipStreamSynchronize(s));
        g->release(dheavy, sizeof(int32_t) * std::max<int64_t>(A, 1));
    }
    g->release(bad, 16);
    guard.g = nullptr;
    return g;
}

extern "C" {

void hgx_graph_destroy(hgx_graph* g) { graph_release(g); }

int hgx_graph_info(const hgx_graph* g, int64_t* num_atoms, int64_t* num_links, int64_t* num_incidences) {
    HGX_API_BEGIN
    if (!g) fail(HGX_E_INVALID, "null graph");
    if (num_atoms) *num_atoms = g->A;
    if (num_links) *num_links = g->M;
    if (num_incidences) *num_incidences = g->I;
    HGX_API_END
}

int hgx_set_timing(hgx_graph* g, int32_t enabled) {
    HGX_API_BEGIN
    if (!g) fail(HGX_E_INVALID, "null graph");
    std::lock_guard<std::mutex> lk(g->mu);
    g->timing = enabled != 0;
    HGX_API_END
}

int hgx_set_option(hgx_graph* g, int32_t option, int64_t value) {
    HGX_API_BEGIN
    if (!g) fail(HGX_E_INVALID, "null graph");
    std::lock_guard<std::mutex> lk(g->mu);
    if (option == HGX_OPT_BFS_FLAGS) {
        // bit 16 is the engine's per-level internal flag (kAllRows): never settable; bit 17 = frontier-code pull
        if (value < 0 || value > 0x3FFFF || (value & 0x10000))
            fail(HGX_E_INVALID, "hgx_set_option: BFS flags outside bits 0-15 and 17");
        g->bfs_flags = (int32_t)value;
    } else if (option == HGX_OPT_RANKS_ORDERED) {
        g->ranks_ordered = value != 0;
    } else if (option == HGX_OPT_PART_SERIAL) {
        if (!g->shard) fail(HGX_E_INVALID, "hgx_set_option: HGX_OPT_PART_SERIAL applies to partition shards");
        g->shard->serial = value != 0;
    } else if (option == HGX_OPT_QUERY_FUSED) {
        // removed in round 5 (measured slower): only "off" is accepted
        if (value != 0) fail(HGX_E_UNSUPPORTED, "hgx_set_option: HGX_OPT_QUERY_FUSED was removed (measured slower)");
    } else if (option == HGX_OPT_QUERY_INLINE) {
        g->q_inline = value != 0;
    } else if (option == HGX_OPT_PART_EXCHANGE) {
        if (!g->shard) fail(HGX_E_INVALID, "hgx_set_option: HGX_OPT_PART_EXCHANGE applies to partition shards");
        // 2 (static slots) was removed in round 5 (measured slower)
        if (value == 2) fail(HGX_E_UNSUPPORTED, "hgx_set_option: the static-slot exchange (2) was removed");
        if (value < 0 || value > 1) fail(HGX_E_INVALID, "hgx_set_option: exchange mode outside 0..1");
        g->shard->xmode = (int32_t)value;
    } else if (option == HGX_OPT_QUERY_FLAT) {
        // 0 and 1 were removed in round 5 (measured slower): only the single-pass path (2)
        if (value != 2) fail(HGX_E_UNSUPPORTED, "hgx_set_option: only HGX_OPT_QUERY_FLAT 2 remains");
    } else if (option == HGX_OPT_CODED) {
        // removed in round 5 (measured slower): only "off" is accepted
        if (value != 0) fail(HGX_E_UNSUPPORTED, "hgx_set_option: HGX_OPT_CODED was removed (coded levels measured slower)");
    } else if (option == HGX_OPT_PUSH_BATCH) {
        // removed in round 5 (slower on the sum of config 5's directions): only 0
        if (value != 0) fail(HGX_E_UNSUPPORTED, "hgx_set_option: HGX_OPT_PUSH_BATCH was removed (measured slower)");
    } else if (option == HGX_OPT_SEQ_BUDGET) {
        if (value < (1 << 20)) fail(HGX_E_INVALID, "hgx_set_option: sequence budget below 1 MiB");
        g->seq_budget_bytes = value;
    } else if (option == HGX_OPT_SEQ_ENGINE) {
        if (value < 0 || value > 2) fail(HGX_E_INVALID, "hgx_set_option: sequence engine outside 0..2");
        g->seq_engine = (int32_t)value;
    } else if (option == HGX_OPT_BFS_BLOCK) {
        if (value < 0 || value > 2) fail(HGX_E_INVALID, "hgx_set_option: BFS block mode outside 0..2");
        g->bfs_block = (int32_t)value;
    } else if (option == HGX_OPT_PUSH_INLINE) {
        // removed in round 5 (measured no faster): only "off" is accepted
        if (value != 0) fail(HGX_E_UNSUPPORTED, "hgx_set_option: HGX_OPT_PUSH_INLINE was removed (measured no faster)");
    } else if (option == HGX_OPT_QUERY_COALESCE) {
        if (value < 0 || value > (1 << 24)) fail(HGX_E_INVALID, "hgx_set_option: coalesce cap outside 0..2^24");
        g->q_coalesce = value != 0;
        if (value > 1) g->q_coalesce_max = value;
    } else if (option == HGX_OPT_CO_TIMEOUT) {
        if (value < 0) fail(HGX_E_INVALID, "hgx_set_option: grid-stage timeout below 0");
        g->co_timeout = value;
    } else if (option == HGX_OPT_SEQ_PULL) {
        if (value < 0 || value > 2) fail(HGX_E_INVALID, "hgx_set_option: sequence pull mode outside 0..2");
        g->seq_pull = (int32_t)value;
    } else if (option == HGX_OPT_SEQ_SMALL) {
        g->seq_small = value != 0;
    } else if (option == HGX_OPT_SEQ_TLIMIT) {
        if (value < 0) fail(HGX_E_INVALID, "hgx_set_option: stream-key limit below 0");
        g->seq_tlimit = value;
    } else if (option == HGX_OPT_SEQ_PACK_MIN) {
        if (value < 0) fail(HGX_E_INVALID, "hgx_set_option: packed-transfer threshold below 0");
        g->seq_pack_min = value;
    } else if (option == HGX_OPT_XB_FLAT) {
        if (!g->shard) fail(HGX_E_INVALID, "hgx_set_option: HGX_OPT_XB_FLAT applies to partition shards");
        if (value < -1 || value > 2) fail(HGX_E_INVALID, "hgx_set_option: broadcast pack mode outside -1..2");
        g->xb_flat = (int32_t)value;
    } else if (option == HGX_OPT_XB_STATIC) {
        if (!g->shard) fail(HGX_E_INVALID, "hgx_set_option: HGX_OPT_XB_STATIC applies to partition shards");
        if (value < -1 || value > 2) fail(HGX_E_INVALID, "hgx_set_option: static broadcast mode outside -1..2");
        g->xb_static = (int32_t)value;
    } else fail(HGX_E_INVALID, "hgx_set_option: unknown option");
    HGX_API_END
}

int hgx_graph_degree(hgx_graph* g, const int32_t* atoms, int32_t n, int64_t* out_deg) {
    HGX_API_BEGIN
    if (!g || (n > 0 && (!atoms || !out_deg)) || n < 0) fail(HGX_E_INVALID, "hgx_graph_degree: bad argument");
    if (n == 0) return HGX_OK;
    std::lock_guard<std::mutex> lk(g->mu);
    HGX_HIP(hipSetDevice(g->device));
    int32_t* da = (int32_t*)g->alloc(sizeof(int32_t) * n);
    int64_t* dd = (int64_t*)g->alloc(sizeof(int64_t) * n);
    HGX_HIP(hipMemcpyAsync(da, atoms, sizeof(int32_t) * n, hipMemcpyHostToDevice, g->stream));
    k_degrees<<<grid_for(n, 256, 1 << 20), 256, 0, g->stream>>>(n, da, g->inc_off, g->A, dd);
    HGX_CHECK_LAUNCH();
    HGX_HIP(hipMemcpyAsync(out_deg, dd, sizeof(int64_t) * n, hipMemcpyDeviceToHost, g->stream));
    HGX_HIP(hipStreamSynchronize(g->stream));
    g->release(da, sizeof(int32_t) * n);
    g->release(dd, sizeof(int64_t) * n);
    for (int32_t i = 0; i < n; ++i)
        if (out_deg[i] < 0) fail(HGX_E_INVALID, "hgx_graph_degree: atom id out of range");
    HGX_API_END
}

int hgx_graph_incidence(hgx_graph* g, int32_t atom, int32_t* out, int64_t cap, int64_t* n_out) {
    HGX_API_BEGIN
    if (!g || !n_out || (cap > 0 && !out)) fail(HGX_E_INVALID, "hgx_graph_incidence: bad argument");
    if (g->shard) fail(HGX_E_UNSUPPORTED, "hgx_graph_incidence: not available on a partition shard");
    if (atom < 0 || atom >= g->A) fail(HGX_E_INVALID, "hgx_graph_incidence: atom id out of range");
    std::lock_guard<std::mutex> lk(g->mu);
    HGX_HIP(hipSetDevice(g->device));
    int64_t off[2];
    HGX_HIP(hipMemcpyAsync(off, g->inc_off + atom, sizeof(off), hipMemcpyDeviceToHost, g->stream));
    HGX_HIP(hipStreamSynchronize(g->stream));
    int64_t n = off[1] - off[0];
    *n_out = n;
    int64_t k = std::min(n, cap);
    if (k > 0) {
        int32_t* tmp = (int32_t*)g->alloc(sizeof(int32_t) * k);
        k_rows_to_atoms<<<grid_for(k, 256), 256, 0, g->stream>>>(k, g->inc_row + off[0], g->link_atom, tmp);
        HGX_CHECK_LAUNCH();
        HGX_HIP(hipMemcpyAsync(out, tmp, sizeof(int32_t) * k, hipMemcpyDeviceToHost, g->stream));
        HGX_HIP(hipStreamSynchronize(g->stream));
        g->release(tmp, sizeof(int32_t) * k);
    }
    HGX_API_END
}

}  // extern "C"
