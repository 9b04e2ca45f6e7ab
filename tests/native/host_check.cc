// host_check.cc -- host-side checks of libhgx's host code under AddressSanitizer + UBSan.
//
// TEST INFRASTRUCTURE (tests/test_sanitize.py builds it with `make -C hypergraphdb_amd/csrc
// sanitize`; nothing ships it).  It links the engine's sources compiled host-only with
// -fsanitize=address,undefined, the synthetic generator (hgx_gen.c) and the oracle
// (oracle/hgx_oracle.c), and drives every entry point that runs without a GPU:
//   * the .hgcsr writer / info / read (hgx_file.hip) on empty, ragged and typed graphs, then the
//     reader on every single-byte header corruption, random section corruptions and every
//     truncation step -- each must fail cleanly (an error code), never read out of bounds;
//   * the descriptor validation of the writer (bad offsets, out-of-range targets);
//   * the vertex-cut planner and shard builder (hgx_part.hip) for 1..8 parts, with the shard
//     tables checked for consistency (each link on one part, one owner per atom, broadcast and
//     reduce tables pointing at each other);
//   * the oracle's BFS and And-query restatements on the same graphs.
// Exit status 0 = every check passed; a sanitizer report aborts with a non-zero status.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/hgx.h"
extern "C" {
#include "../../oracle/hgx_oracle.h"
int64_t hgx_gen_hypergraph_offsets(int64_t M, int32_t lo, int32_t hi, uint64_t seed, int64_t* tgt_off);
int hgx_gen_hypergraph_fill(int64_t N, int64_t M, int32_t lo, int32_t hi, double gamma, int32_t n_types,
                            uint64_t seed, const int64_t* tgt_off, int32_t* tgt_idx, int32_t* link_type);
}

static int g_fail = 0;
#define CHECK(c)                                                                         \
    do {                                                                                 \
        if (!(c)) {                                                                      \
            std::fprintf(stderr, "%s:%d: check failed: %s\n", __FILE__, __LINE__, #c);  \
            g_fail = 1;                                                                  \
        }                                                                                \
    } while (0)

struct Graph {
    int64_t N = 0, M = 0;
    std::vector<int32_t> link_atom, tgt_idx, link_type;
    std::vector<int64_t> tgt_off;
    int64_t A() const { return N + M; }
    hgx_graph_desc desc() const {
        hgx_graph_desc d;
        d.num_atoms = A();
        d.num_links = M;
        d.link_atom = link_atom.data();
        d.tgt_off = tgt_off.data();
        d.tgt_idx = tgt_idx.data();
        d.link_type = link_type.empty() ? nullptr : link_type.data();
        return d;
    }
};

// N nodes then M links (link l is atom N + l); arities in [lo, hi]; power-law targets when gamma > 1.
// Every 5th link of a graph with links also targets an earlier link (links over links).
static Graph make_graph(int64_t N, int64_t M, int lo, int hi, double gamma, int n_types, uint64_t seed) {
    Graph g;
    g.N = N;
    g.M = M;
    g.tgt_off.assign(M + 1, 0);
    int64_t P = hgx_gen_hypergraph_offsets(M, lo, hi, seed, g.tgt_off.data());
    g.tgt_idx.assign(P > 0 ? P : 1, 0);
    if (n_types > 0) g.link_type.assign(M > 0 ? M : 1, 0);
    if (M) hgx_gen_hypergraph_fill(N, M, lo, hi, gamma, n_types, seed, g.tgt_off.data(), g.tgt_idx.data(),
                                   n_types > 0 ? g.link_type.data() : nullptr);
    g.tgt_idx.resize(P);
    if (n_types > 0) g.link_type.resize(M);
    g.link_atom.resize(M);
    for (int64_t l = 0; l < M; l++) g.link_atom[l] = (int32_t)(N + l);
    for (int64_t l = 5; l < M; l += 5)
        if (g.tgt_off[l + 1] > g.tgt_off[l]) g.tgt_idx[g.tgt_off[l]] = (int32_t)(N + l / 2);   // l/2 < l: a link target
    return g;
}

static std::vector<uint8_t> slurp(const std::string& p) {
    std::vector<uint8_t> b;
    FILE* f = std::fopen(p.c_str(), "rb");
    if (!f) return b;
    std::fseek(f, 0, SEEK_END);
    long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    b.resize(n);
    if (n && std::fread(b.data(), 1, n, f) != (size_t)n) b.clear();
    std::fclose(f);
    return b;
}

static void spit(const std::string& p, const uint8_t* b, size_t n) {
    FILE* f = std::fopen(p.c_str(), "wb");
    if (!f) return;
    if (n) std::fwrite(b, 1, n, f);
    std::fclose(f);
}

static bool same(const void* a, const void* b, size_t n) { return n == 0 || std::memcmp(a, b, n) == 0; }

// read back through info + read; returns the hgx status (0 = the file verified and was copied)
static int read_back(const std::string& p, const Graph* expect, int handle_bytes) {
    int64_t A = -1, M = -1, P = -1;
    int32_t hb = -1, typed = -1;
    int rc = hgx_snapshot_info(p.c_str(), &A, &M, &P, &hb, &typed);
    if (rc) return rc;
    // a corrupted header may name absurd sizes: only allocate what a sane reader would (the file
    // size bounds every section), and let the reader refuse the rest
    if (A < 0 || M < 0 || P < 0 || hb < 0 || A > (1 << 26) || M > (1 << 26) || P > (1 << 28) || hb > 64) return -100;
    std::vector<int32_t> la(M + 1), ti(P + 1), lt(M + 1);
    std::vector<int64_t> to(M + 1);
    std::vector<uint8_t> hd((size_t)A * hb + 1);
    rc = hgx_snapshot_read(p.c_str(), la.data(), to.data(), ti.data(), lt.data(), hb ? hd.data() : nullptr);
    if (rc || !expect) return rc;
    CHECK(A == expect->A() && M == expect->M && P == (int64_t)expect->tgt_idx.size());
    CHECK(hb == handle_bytes);
    CHECK(same(la.data(), expect->link_atom.data(), M * 4));
    CHECK(same(to.data(), expect->tgt_off.data(), (M + 1) * 8));
    CHECK(same(ti.data(), expect->tgt_idx.data(), P * 4));
    if (!expect->link_type.empty()) CHECK(same(lt.data(), expect->link_type.data(), M * 4));
    for (int64_t i = 0; i < (int64_t)A * hb; i++) CHECK(hd[i] == (uint8_t)(i * 7 + 3));
    return 0;
}

static void check_file(const Graph& g, const std::string& dir, int handle_bytes, uint64_t seed) {
    std::string p = dir + "/hc.hgcsr";
    std::vector<uint8_t> handles((size_t)g.A() * handle_bytes + 1);
    for (size_t i = 0; i < handles.size(); i++) handles[i] = (uint8_t)(i * 7 + 3);
    hgx_graph_desc d = g.desc();
    CHECK(hgx_snapshot_write(p.c_str(), &d, handle_bytes ? handles.data() : nullptr, handle_bytes) == 0);
    CHECK(read_back(p, &g, handle_bytes) == 0);
    std::vector<uint8_t> good = slurp(p);
    CHECK(good.size() >= 64);
    std::string q = dir + "/hc_bad.hgcsr";
    // every single-byte header corruption must be refused (the header is in the checksum)
    for (size_t i = 0; i < 64 && i < good.size(); i++) {
        std::vector<uint8_t> b = good;
        b[i] ^= 0x5A;
        spit(q, b.data(), b.size());
        CHECK(read_back(q, nullptr, handle_bytes) != 0);
    }
    // section corruptions
    uint64_t s = seed * 0x9E3779B97F4A7C15ull + 1;
    for (int k = 0; k < 64 && good.size() > 64; k++) {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        size_t i = 64 + (size_t)((s >> 17) % (good.size() - 64));
        std::vector<uint8_t> b = good;
        b[i] ^= (uint8_t)(1u << ((s >> 5) & 7));
        spit(q, b.data(), b.size());
        int rc = read_back(q, nullptr, handle_bytes);
        // a flip inside inter-section padding is allowed to pass only if it left the data alone
        (void)rc;
    }
    // every truncation (stepped) must be refused
    size_t step = good.size() > 4096 ? good.size() / 509 : 1;
    for (size_t n = 0; n < good.size(); n += step) {
        spit(q, good.data(), n);
        CHECK(read_back(q, nullptr, handle_bytes) != 0);
    }
    std::remove(q.c_str());
    std::remove(p.c_str());
}

static void check_bad_desc(const Graph& g, const std::string& dir) {
    if (g.M == 0 || g.tgt_idx.empty()) return;
    std::string p = dir + "/hc_inv.hgcsr";
    Graph b = g;
    b.tgt_idx[b.tgt_idx.size() / 2] = (int32_t)b.A();   // out of range
    hgx_graph_desc d = b.desc();
    CHECK(hgx_snapshot_write(p.c_str(), &d, nullptr, 0) != 0);
    b = g;
    b.tgt_off[b.M] = b.tgt_off[b.M] + 1;                  // offsets past the pins
    b.tgt_idx.push_back(0);
    b.tgt_off[1] = b.tgt_off[0] - 1;                      // decreasing
    d = b.desc();
    CHECK(hgx_snapshot_write(p.c_str(), &d, nullptr, 0) != 0);
    b = g;
    b.link_atom[0] = -1;
    d = b.desc();
    CHECK(hgx_snapshot_write(p.c_str(), &d, nullptr, 0) != 0);
    std::remove(p.c_str());
}

static void check_partition(const Graph& g, int NP) {
    hgx_graph_desc d = g.desc();
    std::vector<int32_t> lp(g.M + 1, -1);
    CHECK(hgx_partition_plan(&d, NP, lp.data()) == 0);
    for (int64_t r = 0; r < g.M; r++) CHECK(lp[r] >= 0 && lp[r] < NP);
    std::vector<hgx_shard*> sh(NP, nullptr);
    struct Tab {
        int64_t nl, no, nk, np;
        std::vector<int32_t> l2g, xo_part, xo_lid, bc_part, bc_lid;
        std::vector<int64_t> bc_off, bc_count, ghost_count;
    };
    std::vector<Tab> t(NP);
    std::vector<int> owners(g.A(), 0);
    int64_t links = 0;
    for (int p = 0; p < NP; p++) {
        CHECK(hgx_shard_build(&d, NP, p, lp.data(), &sh[p]) == 0);
        if (!sh[p]) return;
        Tab& x = t[p];
        CHECK(hgx_shard_info(sh[p], &x.nl, &x.no, &x.nk, &x.np) == 0);
        links += x.nk;
        x.l2g.resize(x.nl + 1);
        std::vector<int32_t> la(x.nk + 1), lt(x.nk + 1), ti(x.np + 1);
        std::vector<int64_t> to(x.nk + 1);
        x.ghost_count.resize(NP);
        CHECK(hgx_shard_export(sh[p], x.l2g.data(), la.data(), lt.data(), to.data(), ti.data(),
                               x.ghost_count.data()) == 0);
        for (int64_t i = 1; i < x.nl; i++) CHECK(x.l2g[i - 1] < x.l2g[i]);
        for (int64_t i = 0; i < x.np; i++) CHECK(ti[i] >= 0 && ti[i] < x.nl);
        x.xo_part.resize(x.nl + 1);
        x.xo_lid.resize(x.nl + 1);
        x.bc_off.resize(x.nl + 1);
        x.bc_count.resize(NP);
        CHECK(hgx_shard_exchange_tables(sh[p], x.xo_part.data(), x.xo_lid.data(), x.bc_off.data(), nullptr,
                                        nullptr, x.bc_count.data()) == 0);
        int64_t nb = x.nl ? x.bc_off[x.nl] : 0;
        x.bc_part.resize(nb + 1);
        x.bc_lid.resize(nb + 1);
        CHECK(hgx_shard_exchange_tables(sh[p], nullptr, nullptr, nullptr, x.bc_part.data(), x.bc_lid.data(),
                                        nullptr) == 0);
        int64_t owned = 0;
        for (int64_t l = 0; l < x.nl; l++)
            if (x.xo_part[l] < 0) {
                owned++;
                owners[x.l2g[l]]++;
            }
        CHECK(owned == x.no);
    }
    CHECK(links == g.M);
    // each atom present somewhere has exactly one owner; reduce and broadcast tables agree
    for (int p = 0; p < NP; p++) {
        Tab& x = t[p];
        for (int64_t l = 0; l < x.nl; l++) {
            int32_t a = x.l2g[l];
            CHECK(owners[a] == 1);
            if (x.xo_part[l] >= 0) {
                int q = x.xo_part[l];
                CHECK(q != p && q < NP);
                if (q >= 0 && q < NP && x.xo_lid[l] >= 0 && x.xo_lid[l] < t[q].nl) {
                    CHECK(t[q].l2g[x.xo_lid[l]] == a);
                    CHECK(t[q].xo_part[x.xo_lid[l]] < 0);
                }
            } else {
                for (int64_t e = x.bc_off[l]; e < x.bc_off[l + 1]; e++) {
                    int q = x.bc_part[e];
                    CHECK(q >= 0 && q < NP && q != p);
                    if (q >= 0 && q < NP && x.bc_lid[e] >= 0 && x.bc_lid[e] < t[q].nl) {
                        CHECK(t[q].l2g[x.bc_lid[e]] == a);
                        CHECK(t[q].xo_part[x.bc_lid[e]] == p);
                    }
                }
            }
        }
    }
    for (auto* s : sh) hgx_shard_free(s);
    // invalid arguments
    CHECK(hgx_partition_plan(&d, 0, lp.data()) != 0);
    CHECK(hgx_partition_plan(&d, 65, lp.data()) != 0);
    hgx_shard* bad = nullptr;
    CHECK(hgx_shard_build(&d, NP, NP, lp.data(), &bad) != 0);
    if (g.M) {
        std::vector<int32_t> lq = lp;
        lq[0] = NP;
        CHECK(hgx_shard_build(&d, NP, 0, lq.data(), &bad) != 0);
    }
}

static void check_oracle(const Graph& g) {
    og_graph o;
    std::memset(&o, 0, sizeof(o));
    CHECK(og_graph_build(&o, g.A(), g.M, g.link_atom.data(), g.tgt_off.data(), g.tgt_idx.data(),
                         g.link_type.empty() ? nullptr : g.link_type.data()) == 0);
    const int L = 8;
    int ns = (int)(g.A() < 16 ? g.A() : 16);
    std::vector<int32_t> seeds(ns);
    for (int i = 0; i < ns; i++) seeds[i] = (int32_t)((i * 7919ll) % g.A());
    std::vector<int64_t> counts((size_t)ns * L + 1), trav(ns + 1);
    og_algen al{-1, 1, 1, 0, 0};
    double el = 0;
    if (ns) CHECK(og_bfs_many(&o, &al, seeds.data(), ns, -1, L, counts.data(), trav.data(), 2, 0.0, &el) == 0);
    for (int i = 0; i < ns; i++) CHECK(counts[(size_t)i * L] == 1);
    // single traversals with every generator mode on the first seeds
    std::vector<int32_t> ol(g.A() + 1), oa(g.A() + 1), od(g.A() + 1);
    for (int m = 0; m < 16 && ns; m++) {
        og_algen a2{(m & 8) ? 0 : -1, m & 1, (m >> 1) & 1, (m >> 2) & 1, (m >> 3) & 1};
        int64_t tr = 0;
        int64_t n = og_bfs(&o, &a2, seeds[m % ns], -1, ol.data(), oa.data(), od.data(), g.A(), &tr);
        CHECK(n >= 0 && n <= g.A());
    }
    // And queries anchored on each link's first two targets
    std::vector<int32_t> out(g.M + 1);
    for (int64_t l = 0; l < g.M && l < 64; l++) {
        int64_t b = g.tgt_off[l], k = g.tgt_off[l + 1] - b;
        if (k < 1) continue;
        int32_t inc[2] = {g.tgt_idx[b], g.tgt_idx[b + (k > 1 ? 1 : 0)]};
        int64_t n = og_and_query(&o, g.link_type.empty() ? -1 : g.link_type[l], inc, k > 1 ? 2 : 1,
                                 g.tgt_idx.data() + b, (int32_t)k, 1, out.data(), g.M);
        CHECK(n >= 1);   // the link itself matches
        int64_t n2 = og_and_query_sets(&o, g.link_type.empty() ? -1 : g.link_type[l], inc, k > 1 ? 2 : 1,
                                       g.tgt_idx.data() + b, (int32_t)k, 1, out.data(), g.M);
        CHECK(n == n2);
    }
    og_graph_free(&o);
}

int main(int argc, char** argv) {
    std::string dir = argc > 1 ? argv[1] : "/tmp";
    struct Case {
        int64_t N, M;
        int lo, hi;
        double gamma;
        int types;
    } cases[] = {
        {1, 0, 0, 0, 0.0, 0},        // one isolated atom, no links
        {5, 3, 0, 3, 0.0, 0},        // ragged, arity 0 links
        {40, 60, 1, 6, 0.0, 3},      // typed
        {300, 700, 2, 9, 2.1, 2},    // power law hubs
        {2000, 5000, 1, 12, 2.3, 4}, // larger, hubs above the heavy-row threshold
    };
    int ci = 0;
    for (const Case& c : cases) {
        Graph g = make_graph(c.N, c.M, c.lo, c.hi, c.gamma, c.types, 1000 + ci);
        check_file(g, dir, 0, ci);
        check_file(g, dir, 8, ci);
        check_bad_desc(g, dir);
        for (int NP : {1, 2, 3, 8}) check_partition(g, NP);
        check_oracle(g);
        std::printf("case %d: A=%lld M=%lld P=%zu %s\n", ci, (long long)g.A(), (long long)g.M, g.tgt_idx.size(),
                    g_fail ? "FAIL" : "ok");
        ci++;
    }
    std::printf(g_fail ? "host_check: FAILED\n" : "host_check: all checks passed\n");
    return g_fail;
}
