// hgx_internal.h -- shared definitions of the MI355X engine (libhgx.so).
//
// Device layout of a snapshot:
//   link_atom [M]   int32   atom id of link row r (ascending)
//   tgt_off   [M+1] int64   target row offsets
//   tgt_idx   [P]   int32   target atom ids, layout order t0..tk-1
//   link_type [M]   int32   type key of link row r
//   inc_off   [A+1] int64   incidence row offsets
//   inc_row   [I]   int32   incident LINK ROWS, ascending (row order == atom rank order)
//   inc_type  [I]   int32   type key of inc_row[i] (denormalised for the pattern filter)
// plus the heavy-atom chunk table used to balance power-law incidence rows.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/hgx.h"

namespace hgx {

// Engine knobs.  The product library reads no tuning setting from the environment (a library loaded into
// a JVM must not change behaviour with whichever call read the environment first, and getenv racing a
// setenv is undefined in a multi-threaded host): tunables that callers and tests set go through
// hgx_set_option (per graph).  The measured-negative A/B variants of DESIGN.md are reachable only in A/B
// builds (tools/build_variant.sh compiles with -DHGX_AB_KNOBS), where ab_env reads them; tracing
// (trace_env: HGX_BFS_TRACE, HGX_SEQ_TRACE, HGX_CO_TRACE, HGX_LS_PROF, HGX_QUERY_PROFILE) stays
// environment-driven and only adds output.
inline const char* ab_env(const char* name) {
#ifdef HGX_AB_KNOBS
    return std::getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}
inline bool trace_env(const char* name) { return std::getenv(name) != nullptr; }
inline int ab_int(const char* name, int dflt) {
    const char* e = ab_env(name);
    return e ? std::atoi(e) : dflt;
}

struct Error {
    int code;
    std::string msg;
};

[[noreturn]] void fail(int code, const std::string& msg);
void set_last_error(const std::string& msg);

#define HGX_HIP(x)                                                                              \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess)                                                                   \
            ::hgx::fail(HGX_E_DEVICE, std::string(#x) + ": " + hipGetErrorString(e_));          \
    } while (0)

#define HGX_CHECK_LAUNCH() HGX_HIP(hipGetLastError())

#define HGX_API_BEGIN try {
// As HGX_API_END without the final `return HGX_OK` (a body that falls through to more code).
#define HGX_API_END_NORETURN                                                                    \
    }                                                                                           \
    catch (const ::hgx::Error& e) {                                                             \
        ::hgx::set_last_error(e.msg);                                                           \
        return e.code;                                                                          \
    }                                                                                           \
    catch (const std::bad_alloc&) {                                                             \
        ::hgx::set_last_error("host allocation failed");                                        \
        return HGX_E_NOMEM;                                                                     \
    }                                                                                           \
    catch (const std::exception& e) {                                                           \
        ::hgx::set_last_error(e.what());                                                        \
        return HGX_E_DEVICE;                                                                    \
    }                                                                                           \
    catch (...) {                                                                               \
        ::hgx::set_last_error("unknown error");                                                 \
        return HGX_E_DEVICE;                                                                    \
    }

#define HGX_API_END                                                                             \
    }                                                                                           \
    catch (const ::hgx::Error& e) {                                                             \
        ::hgx::set_last_error(e.msg);                                                           \
        return e.code;                                                                          \
    }                                                                                           \
    catch (const std::bad_alloc&) {                                                             \
        ::hgx::set_last_error("host allocation failed");                                        \
        return HGX_E_NOMEM;                                                                     \
    }                                                                                           \
    catch (const std::exception& e) {                                                           \
        ::hgx::set_last_error(e.what());                                                        \
        return HGX_E_DEVICE;                                                                    \
    }                                                                                           \
    catch (...) {                                                                               \
        ::hgx::set_last_error("unknown error");                                                 \
        return HGX_E_DEVICE;                                                                    \
    }                                                                                           \
    return HGX_OK;

// Incidence rows longer than this are split into chunks processed by whole workgroups.
constexpr int64_t kHeavyDegree = 512;
constexpr int64_t kChunkEntries = 4096;

struct HeavyChunk {
    int64_t beg, end;   // incidence entry range
    int32_t atom;       // atom id
    int32_t slot;       // heavy-atom slot (accumulator row)
};

struct PoolBuf {
    void* p;
    size_t n;
};

// A yield list (yield_list below): the links of each atom's incidence entries that pass one link type
// and can yield in one generator mode, in entry order.
struct YieldList {
    int32_t mode, type;
    int64_t* off;   // [A + 1]
    int32_t* row;   // [n] link ids
    int64_t n;
};
constexpr size_t kMaxYieldLists = 8;

// A yield adjacency (yield_adj below): per atom, the generator's output itself -- every (target, link
// atom) pair its incidence entries yield in one mode for one link type and minimum arity, in stream
// order (entry order, then yield rank).  off == nullptr: refused (more than kYieldAdjBudget bytes).
struct YieldAdj {
    int32_t mode, type, min_arity, rev;
    int64_t* off;   // [A + 1]
    int32_t* tgt;   // [n]
    int32_t* lnk;   // [n] link atom ids
    int64_t n;
};
constexpr int64_t kYieldAdjBudget = (int64_t)4 << 30;

// Vertex-cut partition of a snapshot over n_parts devices (hgx_part.hip):
// every link row lives on one part; an atom is present (local) on every part holding one of its
// links and owned by one of them.  Local ids are assigned in global id order, so every ascending
// local list is an ascending global list.
struct ShardInfo {
    int32_t n_parts = 1, part = 0;
    int64_t A_global = 0, n_owned = 0;
    std::vector<int32_t> l2g_host;       // [A_local] global id of local atom (ascending)
    std::vector<uint64_t> present_host;  // [A_global/64 + 1] atoms present on some part
    std::vector<uint64_t> own_bm_host;   // [A_local/64 + 2] bit set <=> local atom is owned here
    std::vector<int64_t> ghost_count;    // [n_parts] my ghosts owned by part q = reduce records to q (max)
    std::vector<int64_t> bc_count;       // [n_parts] my owned atoms held by part q = broadcast records to q (max)
    bool serial = false;                 // in-process rehearsal: parts run their kernels one at a time
    // device copies
    uint64_t* own_bm = nullptr;          // [A_local/64 + 2]
    int32_t* xo_part = nullptr;          // [A_local] ghost: owner part (-1 owned)
    int32_t* xo_lid = nullptr;           // [A_local] ghost: its local id on the owner
    int64_t* bc_off = nullptr;           // [A_local + 1] owned atom: its other holders ...
    int32_t* bc_part = nullptr;          //   ... their parts
    int32_t* bc_lid = nullptr;           //   ... and its local id there
    // Static exchange slots (dense levels): the j-th of my ghosts owned by q (ascending ids) sends to
    // slot j of q's receive segment from me, and q's j-th owned atom held by me (ascending ids: the
    // same atom) answers in slot j of my receive segment from q.
    int32_t* bc_slot = nullptr;          // [bc entries] its slot in the (me -> holder) segment
    int32_t* bc_atom = nullptr;          // [bc entries] the owned atom of the entry (flat broadcast pack)
    int32_t xmode = 1;                   // HGX_OPT_PART_EXCHANGE: 0 / 1 compressed records (static slots removed in round 5)
    // the global -> local id of an atom present here, or -1 (binary search of l2g_host)
    int32_t local_of(int64_t v) const {
        auto it = std::lower_bound(l2g_host.begin(), l2g_host.end(), (int32_t)v);
        return (it != l2g_host.end() && *it == v) ? (int32_t)(it - l2g_host.begin()) : -1;
    }
    bool owns_local(int64_t l) const { return (own_bm_host[l >> 6] >> (l & 63)) & 1ull; }
    bool present(int64_t v) const { return (present_host[v >> 6] >> (v & 63)) & 1ull; }
};

// Transport of the per-level frontier exchange: RCCL between processes (one GPU each), an
// in-process group of shard threads, or host-staged callbacks.  Every call is collective.
struct Transport {
    int32_t world = 1, rank = 0;
    virtual ~Transport() {}
    // out[r * n + i] = in[i] of rank r (host buffers)
    virtual void allgather_i64(const int64_t* in, int64_t n, int64_t* out, hipStream_t s) = 0;
    // The same for a DEVICE input written by work ordered on s: out (host) = every rank's n values;
    // pin = pinned host scratch of n * world int64.  Returns the host round trips it took.  The
    // default reads the values back and runs the host all-gather (two); RCCL gathers on the device
    // and reads the gathered block back once (hgx_part.hip).
    virtual int allgather_dev(const int64_t* din, int64_t n, int64_t* out, hipStream_t s, int64_t* pin);
    // rank p receives send_bytes[p] bytes from send + send_off[p]; this rank receives recv_bytes[p]
    // bytes from rank p at recv + recv_off[p] (device buffers, ordered on stream s)
    virtual void alltoallv(const void* send, const int64_t* send_off, const int64_t* send_bytes, void* recv,
                           const int64_t* recv_off, const int64_t* recv_bytes, hipStream_t s) = 0;
    // brackets of a part's device work between two exchanges (the in-process rehearsal runs the
    // parts' kernels one part at a time so their device times are clean)
    virtual void compute_begin(hipStream_t) {}
    virtual void compute_end(hipStream_t) {}
    virtual void compute_release(hipStream_t) {}   // end of the work or an error path: give the gate back
    virtual const char* kind() const = 0;
};

// Cross-thread coalescing of pattern batches (hgx_pattern_batch_packed, HGX_OPT_QUERY_COALESCE):
// a caller that finds the graph's device busy queues its batch; whoever runs next takes every queued
// batch (FIFO, up to a query cap) and runs them as ONE device batch, then splits the result.  The
// reference's usage is many threads each executing small compiled queries
// (TC/query/QueryCompilation.java:76-122); one device batch per caller would serialise them on the
// per-graph mutex at the full fixed cost of a batch each.
struct PackedReq {
    int32_t n = 0;
    const int32_t* type = nullptr;
    const int64_t* inc_off = nullptr;
    const int32_t* inc = nullptr;
    const int32_t* has_ordered = nullptr;
    const int64_t* pat_off = nullptr;
    const int32_t* pat = nullptr;
    hgx_query_result* r = nullptr;   // set when done and rc == HGX_OK
    int rc = HGX_OK;
    std::string err;
    bool done = false;
};
struct QueryCombiner {
    std::mutex mu;
    std::condition_variable cv;
    std::deque<PackedReq*> pending;
    bool busy = false;
    int64_t batches = 0, requests = 0;   // device batches run / caller batches served (statistics)
};

}  // namespace hgx

struct hgx_comm {
    hgx::Transport* t = nullptr;
};

struct hgx_graph {
    // Execution context (hgx_graph_context): the snapshot's arrays are borrowed from base (which this
    // context holds a reference on); the stream, lock, scratch pool, accumulator, counters and host
    // staging are its own, so traversals on two contexts of one snapshot run side by side.
    hgx_graph* base = nullptr;
    int device = 0;
    hipStream_t stream = nullptr;
    hipStream_t stream2 = nullptr;      // readout counting next to the traversal (made on first use)
    hipStream_t stream3 = nullptr;      // the order-exact level engine's second copy stream (made on first use)
    hipEvent_t ev_count = nullptr;      //   and its ordering event
    std::mutex mu;
    std::atomic<int> refs{1};
    bool timing = false;
    std::vector<hipEvent_t> ev_pool;   // timing events reused across calls (taken under mu)
    int32_t bfs_flags = 0x3BE;      // HGX_OPT_BFS_FLAGS (see hgx.h)
    int64_t seq_budget_bytes = (int64_t)48 << 30;   // HGX_OPT_SEQ_BUDGET: order-exact traversal working set
    int64_t max_arity = -1, max_deg = -1;           // lazily computed (order-exact stream keys)
    int32_t seq_engine = 0;                         // HGX_OPT_SEQ_ENGINE: 0 workgroup per seed (+ level engine), 1 key-array
                                                    //   level engine only, 2 level engine (hgx_ls_*) only
    unsigned long long* seq_flag = nullptr;         // mapped coherent words: level sizes of the level engine
    hipEvent_t ls_ev[16] = {};                      //   its rank parts' events (2 level parities x 8 parts)
    hipEvent_t ls_cev[2] = {};                      //   a level's pair copies enqueued (by level parity)
    unsigned long long seq_flag_seq = 0;            //   (their sequence numbers)
    int64_t ls_cap = 0, ls_tcap = 0, ls_rcap = 0;   // level-engine capacities grown on demand
    int64_t ls_hcap = 0, ls_fcap = 0;               //   and its two hash tables' slots (push, frontier)
    int32_t* pin_j = nullptr;                       // [P] index of link row L in inc(t) for each pin (t, L):
                                                    //   the level engine's pull levels (snapshot only, made on first use)
    int4* pull_rec = nullptr;                       // [I x 4] per incidence entry (t, L): L's <= 8 targets, then their
                                                    //   pin_j -- the pull walk's link data streamed in entry order
    int2* pull_meta = nullptr;                      // [I] (link atom, arity) per incidence entry
    int32_t pull_rec_state = 0;                     //   0 not built yet, 1 built, -1 over its memory budget
    int4* fc_rec = nullptr;                         // [I x 2] per incidence entry: its link's <= 8 targets (-1 padded),
    int32_t fc_rec_state = 0;                       //   the frontier-code pull's records (snapshot only, made on first
                                                    //   use; 0 not built, 1 built, -1 over budget / arity > 8)
    int32_t* fc_hubs = nullptr;                     //   and its hub atoms (ascending; their slots are in the records)
    int32_t fc_nhubs = 0;
    std::mutex seq_mu;                              // guards seq_hbufs (results hand their buffers back from any thread)
    std::vector<hgx::PoolBuf> seq_hbufs;            // mapped host buffers of order-exact results, free for reuse
    int32_t bfs_block = 1;                          // HGX_OPT_BFS_BLOCK: hgx_bfs_batch seeds first run one workgroup each
    // test / diagnostic options (hgx.h: HGX_OPT_CO_TIMEOUT .. HGX_OPT_XB_STATIC); 0 / -1 = the engine's default
    int64_t co_timeout = 0;                         // grid-stage barrier limit in s_memrealtime ticks (0 = 1 s)
    int32_t seq_pull = 1;                           // level engine pull levels: 0 never, 1 by width, 2 always
    int32_t seq_small = 0;                          // level engine: tiny starting capacities (exercise growth)
    int64_t seq_tlimit = 0;                         // level engine: stream-key limit below the 32-bit one (0 = none)
    int64_t seq_pack_min = 0;                       // level engine: pairs of a level that cross PCIe packed (0 = 2^20)
    int32_t xb_flat = -1, xb_static = -1;           // partition broadcast pack variants (-1 = default)
    unsigned long long* co_vis = nullptr;           // multi-workgroup stage: per-seed visited bitmaps (zero between calls)
    unsigned long long* sc_tab = nullptr;           // order-exact grid stage: level hash, word / key counts (empty between calls)
    int64_t co_vis_seeds = 0, co_pcap = 0;          //   seeds they hold; pair-list capacity (grown on demand)
    int64_t co_fr = 0;                              //   work items a level holds, all segments (likewise)
    int32_t co_ok = -1;                             //   its grid in blocks (0: does not fit; -1: not checked yet)
    int64_t co_timeouts = 0;                        //   launches whose grid barrier timed out (seeds fell back)
    int32_t sc_ok = -1;                             // order-exact grid stage (hgx_seq_coop): its grid (0: does not fit)
    int64_t sc_pcap = 0;                            //   its pair capacity (grown on demand)
    std::deque<hgx::YieldList> ylists;              // yield lists (snapshot only; contexts read their base's)
    std::deque<hgx::YieldAdj> yadjs;                // yield adjacencies (likewise)
    std::mutex ylist_mu;
    // HGX_OPT_RANKS_ORDERED: rank order == persistent-handle order.  Cleared by an hgx_graph_update
    // that extends the rank space (appended ranks need not sort after the existing handles); the
    // order-exact traversal refuses to run until the caller re-asserts it.
    bool ranks_ordered = true;
    // Frontier-push accumulator rows (A x W words), all zero between levels: each push level ORs
    // into it and its finalise re-zeroes exactly the rows it consumed (no per-level clear).
    std::vector<int64_t> inc_off_host;   // host copy of inc_off (pattern planning), made on first use
    uint64_t* zacc = nullptr;
    unsigned long long* ctr_host = nullptr;   // push levels' counters, written by the finalise (mapped host memory)
    unsigned long long ctr_seq = 0;          // sequence numbers of those writes
    hipEvent_t pend_ev[2] = {nullptr, nullptr};   // the batched BFS's two in-flight level events
    uint64_t* hasinc = nullptr;          // [A/64 + 1] bit set <=> inc(atom) non-empty (non-full pull levels)
    uint8_t* inc_yf = nullptr;           // [I] ordered-mode yield flags per incidence (frontier push), made on first use
    hgx::HeavyChunk* pchunks = nullptr;  // frontier push: kPushChunk-entry chunks of atoms with deg > kPushLight
    int64_t n_pchunks = -1;              // -1 = not built yet
    size_t zacc_bytes = 0;
    bool zacc_clean = false;

    int64_t A = 0, M = 0, P = 0, I = 0;
    int32_t* link_atom = nullptr;
    int64_t* tgt_off = nullptr;
    int32_t* tgt_idx = nullptr;
    int32_t* link_type = nullptr;
    int64_t* inc_off = nullptr;
    int32_t* inc_row = nullptr;
    int32_t* inc_type = nullptr;    // [I] link_type[inc_row[i]]: streamed type filter of the query path
    // Type-grouped incidence (built on the first pattern query): inside each atom's segment the link
    // rows ordered by (type, row), so the links of one type incident to an atom are one contiguous,
    // ascending range (found by binary search over inc_ts_type).
    int32_t* inc_ts_row = nullptr;
    int32_t* inc_ts_type = nullptr;
    // Inline target rows of the type-grouped incidence (HGX_OPT_QUERY_INLINE, built with it): entry i
    // holds the <= 8 targets of link inc_ts_row[i] in 32 bytes (-1 padded; slot 0 = -2 for a link of
    // arity > 8, which the match reads through tgt_off).  A typed candidate then costs one streamed
    // 32-byte record instead of two dependent random rows.
    int32_t* inc_ts_tgt = nullptr;
    bool q_inline = true;

    int64_t n_heavy = 0;            // heavy atoms (deg > kHeavyDegree)
    int64_t I_heavy = 0;            // incidence entries of heavy atoms
    int64_t n_chunks = 0;
    int32_t* heavy_atom = nullptr;  // [n_heavy]
    hgx::HeavyChunk* chunks = nullptr;

    hgx::ShardInfo* shard = nullptr;   // set for a partition shard (hgx_shard_graph_create)

    std::vector<hgx::PoolBuf> pool;  // free device buffers for reuse across batches
    void* pinned = nullptr;          // small pinned host staging area
    size_t pinned_bytes = 0;
    void* mapped = nullptr;          // host-mapped result area the pattern kernels write into
    size_t mapped_bytes = 0;
    void* zc_in = nullptr;           // fine-grained pinned staging the pattern front kernel reads directly
    void* zc_in_dev = nullptr;       //   (its device address)
    size_t zc_in_bytes = 0;
    int64_t q_cap_chunks = 0, q_cap_cand = 0;   // pattern workspace capacity (grown on demand)
    int64_t q_hits_guess = 0;                   // result ids copied back with the head of the result area
    int32_t q_coalesce = 1;                     // HGX_OPT_QUERY_COALESCE: concurrent packed batches share device batches
    int64_t q_coalesce_max = 1 << 16;           //   at most this many queries per coalesced device batch
    hgx::QueryCombiner qcomb;
    unsigned long long* q_ticket = nullptr;     // pattern placement: blocks-done ticket (device, zero between batches)
    unsigned long long q_seq = 0;               //   sequence number of the completion flag in the result area

    void* alloc(size_t bytes);
    void release(void* p, size_t bytes);
    void* pinned_buf(size_t bytes);
    void* mapped_buf(size_t bytes);
    void* zc_in_buf(size_t bytes);   // host pointer; zc_in_dev is the kernels' view of it
};

namespace hgx {
void graph_release(hgx_graph* g);
void free_yield_lists(hgx_graph* g);   // (hgx_graph_update: the incidence changed)   // drop a reference; frees at zero
// Builds the BFS's first-use read-only tables (has-incidence bitmap, yield flags, push chunks) on g
// (hgx_bfs.hip; caller holds g->mu).
void bfs_shared_tables(hgx_graph* g);
// Upload + incidence build.  links_are_atoms = false for partition shards: link rows then carry
// their global link atom ids (not local atoms) and are not validated against num_atoms.
hgx_graph* graph_create(const hgx_graph_desc* d, int32_t device, bool links_are_atoms);
// Partitioned batched BFS over one shard; tr is the group's transport (hgx_bfs.hip).
void pbfs_run(hgx_graph* g, Transport* tr, const int32_t* seeds, int32_t n_seeds, int32_t max_depth,
              const hgx_algen_opts* opts, hgx_bfs_result** out);
inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }
// Builds the ordered-mode yield flags (hgx_inc_yield, one byte per incidence entry + 64 bytes of
// padding for 16-byte vector loads) on g if absent; caller holds g->mu (hgx_bfs.hip).
void ensure_inc_yield(hgx_graph* g);
// Per (generator mode, link type): for each atom the links of its incidence entries of that type that
// can yield in that mode, in entry order (off [A + 1], row [n]); built on first use on the snapshot
// (shared by its contexts, freed with it).  nullptr for the symmetric mode without a type (the
// incidence itself) and once kMaxYieldLists lists exist.  Caller holds g->mu (hgx_seq.hip).
const YieldList* yield_list(hgx_graph* g, int mode, int32_t type);
// The generator's (target, link atom) output per atom for (mode, type, minimum arity, reverse order),
// in stream order; built on first use on the snapshot.  nullptr for the symmetric mode without a type,
// when refused (over kYieldAdjBudget) and once kMaxYieldLists exist.  Caller holds g->mu (hgx_seq.hip).
const YieldAdj* yield_adj(hgx_graph* g, int mode, int32_t type, int32_t min_arity, bool rev);
// The set-mode workgroup engine's part of one hgx_bfs_batch (hgx_seq.hip, HGX_OPT_BFS_BLOCK): per seed
// V_1, V_2, ... one after the other (atoms) and |V_d| (lcnt[d - 1]) in mapped host buffers the
// result owns; the seeds whose traversal outgrew a workgroup are listed in rerun (the batched engine
// runs them).
struct BlockSet {
    std::vector<PoolBuf> bufs;
    std::vector<int32_t> seeds;                 // [n seeds] the start atoms (V_0)
    std::vector<const int32_t*> atoms, lcnt;   // [n seeds] (nullptr: rerun)
    std::vector<int32_t> pairs, levels;         // [n seeds] atoms past V_0 (-1: rerun), levels with news
    std::vector<int32_t> rerun;                 // seed indices, ascending
    double traversed = 0, ms = 0, bytes = 0;   // items of the finished seeds; device ms; algorithmic bytes
    int32_t expanded = 0;                       // most levels expanded by one finished seed
    // Seeds the multi-workgroup stage finished (the workgroup stage's overflow, <= kMaxCoSeeds of
    // them): their (atom, seed | level << 8) pairs stay in device pool memory until a reader asks for
    // a set (block_materialize); their level counts are on the host at once.
    void* co_pairs = nullptr;                   // kCoSegs segments of co_pseg pairs, co_segn[q] used in q
    size_t co_bytes = 0;
    int64_t co_n = 0, co_pseg = 0;
    std::vector<int64_t> co_segn;
    std::vector<int32_t> co_idx;                // seed indices
    std::vector<std::vector<int32_t>> co_lcnt, co_atoms;
    bool co_host = false;
    double co_ms = 0, co_bytes_alg = 0;         // device ms of that launch (timing on), its algorithmic bytes
    int32_t n_coop = 0;                         // seeds it finished
    int32_t co_fallbacks = 0;                   // its launches that timed out on a grid barrier (rows engine ran)
};
constexpr int kMaxCoSeeds = 64;
// Runs every seed on the workgroup engine (caller holds g->mu, g's device current; max_depth -1 =
// unbounded); returns when the seeds are done.
void bfs_block(hgx_graph* g, const int32_t* seeds, int32_t n_seeds, int32_t max_depth, const hgx_algen_opts& o,
               BlockSet& out);
// Hands the result's mapped buffers back to the graph's pool (caller holds g->mu).
void block_release(hgx_graph* g, BlockSet& b);
// Per-seed atom lists of the multi-workgroup stage's seeds on the host (first reader; g->mu held).
void block_materialize(hgx_graph* g, BlockSet& b);
// Waits for the work enqueued on s by polling: hipStreamSynchronize sleeps and wakes tens of
// microseconds after the last kernel, a cost per call of the short pattern batches.
inline void spin_sync(hipStream_t s) {
    hipError_t e;
    while ((e = hipStreamQuery(s)) == hipErrorNotReady) {
    }
    HGX_HIP(e);
}
inline int grid_for(int64_t work_items, int block, int max_blocks = 8192) {
    int64_t b = ceil_div(work_items > 0 ? work_items : 1, block);
    return (int)(b < max_blocks ? b : max_blocks);
}
}  // namespace hgx
