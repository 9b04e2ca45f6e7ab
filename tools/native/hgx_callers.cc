// hgx_callers.cc -- a native load generator for the C ABI: T application threads issuing calls on
// one graph at once, the way JVM threads call the JNI shim (TC/query/QueryCompilation.java:76-122
// runs one compiled query from a 20-thread pool).  MEASUREMENT INFRASTRUCTURE (bench.py,
// tools/bench_callers.py): Python threads would serialise on the interpreter lock between calls.
//
// hgxc_pattern_threads: thread t issues the packed queries t*per_call, (t+T)*per_call, ... in calls of
// per_call queries each (per_call = 1: single And queries); per-query hit counts go to hits[].
// hgxc_sequence_threads: thread t issues hgx_bfs_sequence for single seeds t, t+T, ...; per-seed pair
// counts go to pairs[] (contexts != 0: each thread on its own execution context of the graph).  Both return the wall seconds from the start barrier to the last call's end.
#include <atomic>
#include <chrono>
#include <cstring>
#include <thread>
#include <vector>

#include "hgx.h"

namespace {

struct Start {
    std::atomic<int> ready{0};
    std::atomic<bool> go{false};
    void arrive_and_wait() {
        ready.fetch_add(1);
        while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
    }
};

template <class Body>
int run_threads(int32_t threads, Body body, double* seconds) {
    std::vector<std::thread> th;
    std::vector<int> rc((size_t)threads, HGX_OK);
    Start st;
    for (int t = 0; t < threads; ++t)
        th.emplace_back([&, t] {
            st.arrive_and_wait();
            rc[(size_t)t] = body(t);
        });
    while (st.ready.load() < threads) std::this_thread::yield();
    const auto t0 = std::chrono::steady_clock::now();
    st.go.store(true, std::memory_order_release);
    for (auto& x : th) x.join();
    *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    for (int r : rc)
        if (r != HGX_OK) return r;
    return HGX_OK;
}

}  // namespace

extern "C" {

int hgxc_pattern_threads(hgx_graph* g, int32_t threads, int32_t n, const int32_t* type, const int64_t* inc_off,
                         const int32_t* inc, const int32_t* has_ordered, const int64_t* pat_off, const int32_t* pat,
                         int32_t per_call, int64_t* hits, double* seconds) {
    if (!g || threads < 1 || n < 1 || per_call < 1 || !seconds) return HGX_E_INVALID;
    return run_threads(
        threads,
        [&](int t) -> int {
            std::vector<int64_t> io((size_t)per_call + 1), po((size_t)per_call + 1), off((size_t)per_call + 1);
            for (int64_t b = (int64_t)t * per_call; b < n; b += (int64_t)threads * per_call) {
                const int32_t k = (int32_t)std::min<int64_t>(per_call, n - b);
                for (int32_t i = 0; i <= k; ++i) {   // the call's own offsets start at 0
                    io[(size_t)i] = inc_off[b + i] - inc_off[b];
                    po[(size_t)i] = pat_off[b + i] - pat_off[b];
                }
                hgx_query_result* r = nullptr;
                int rc = hgx_pattern_batch_packed(g, k, type + b, io.data(), inc + inc_off[b], has_ordered + b, po.data(),
                                                  pat + pat_off[b], &r);
                if (rc != HGX_OK) return rc;
                rc = hgx_query_result_offsets(r, off.data());
                if (rc == HGX_OK && hits)
                    for (int32_t i = 0; i < k; ++i) hits[b + i] = off[(size_t)i + 1] - off[(size_t)i];
                hgx_query_result_free(r);
                if (rc != HGX_OK) return rc;
            }
            return HGX_OK;
        },
        seconds);
}

int hgxc_sequence_threads(hgx_graph* g, int32_t threads, int32_t n, const int32_t* seeds, int32_t max_depth,
                          const hgx_algen_opts* opts, int64_t* pairs, double* seconds, int32_t contexts) {
    if (!g || threads < 1 || n < 1 || !seeds || !seconds) return HGX_E_INVALID;
    // contexts != 0: every thread runs on its own execution context of g (hgx_graph_context, made before
    // the start barrier), as HGGpuSnapshot.acquireContext gives each Java caller one
    std::vector<hgx_graph*> ctx((size_t)threads, g);
    if (contexts)
        for (int t = 0; t < threads; ++t) {
            const int rc = hgx_graph_context(g, &ctx[(size_t)t]);
            if (rc != HGX_OK) {
                for (int k = 0; k < t; ++k) hgx_graph_destroy(ctx[(size_t)k]);
                return rc;
            }
        }
    const int rc_all = run_threads(
        threads,
        [&](int t) -> int {
            hgx_graph* gt = ctx[(size_t)t];
            for (int32_t i = t; i < n; i += threads) {
                hgx_seq_result* r = nullptr;
                int rc = hgx_bfs_sequence(gt, seeds + i, 1, max_depth, opts, &r);
                if (rc != HGX_OK) return rc;
                int32_t ns = 0, nl = 0;
                int64_t np = 0;
                rc = hgx_seq_result_info(r, &ns, &np, &nl);
                if (pairs) pairs[i] = np;
                hgx_seq_result_free(r);
                if (rc != HGX_OK) return rc;
            }
            return HGX_OK;
        },
        seconds);
    if (contexts)
        for (hgx_graph* c : ctx) hgx_graph_destroy(c);
    return rc_all;
}

}  // extern "C"
