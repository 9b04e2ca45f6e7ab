// hgx_file.hip -- the snapshot on disk (.hgcsr) and batched store updates.
//
// The exporter side of SURVEY.md 8(f) rank 1: a Java exporter enumerates
// the store -- every atom handle via IndexScanQuery(indexByType) (C/query/cond2qry/ToQueryMap.java:
// 101-113), every link layout via HGStore.getLink (C/HGStore.java:179-191) -- ranks the handles in
// unsigned byte order and writes the bipartite CSR here; hgx_graph_open maps the file and builds the
// device snapshot.  hgx_graph_update applies a batch of HGAtomAddedEvent / HGAtomRemovedEvent link
// changes (C/event; store side C/HGStore.java:100-170) by rebuilding the device index from the merged rows.
//
// Layout (little-endian), every section 64-byte aligned:
//   header  64 B  magic "HGXCSR1\0", u32 version (2), u32 flags (bit 0 link_type, bit 1 handles),
//                 i64 num_atoms, i64 num_links, i64 num_pins, u32 handle_bytes, u32 reserved,
//                 u64 checksum of the header (checksum field zero) and the sections
//   link_atom i32[M] | tgt_off i64[M+1] | tgt_idx i32[P] | link_type i32[M] (flag 0) |
//   handles u8[A * handle_bytes] (flag 1: the persistent handle of every rank)
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <memory>

#include "hgx_internal.h"

using namespace hgx;

namespace {

constexpr char kMagic[8] = {'H', 'G', 'X', 'C', 'S', 'R', '1', '\0'};
constexpr uint32_t kVersion = 2;   // 2: the checksum also covers the header

struct Header {
    char magic[8];
    uint32_t version, flags;
    int64_t num_atoms, num_links, num_pins;
    uint32_t handle_bytes, reserved;
    uint64_t checksum;
    uint8_t pad[8];
};
static_assert(sizeof(Header) == 64, "header is 64 bytes");

inline size_t align64(size_t x) { return (x + 63) & ~(size_t)63; }

// 64-bit checksum over 8-byte words (multiply-rotate mix; the tail is zero-padded)
uint64_t mix(uint64_t h, const void* p, size_t n) {
    const uint8_t* b = (const uint8_t*)p;
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t w;
        std::memcpy(&w, b + i, 8);
        h = (h ^ w) * 0x9E3779B97F4A7C15ull;
        h = (h << 31) | (h >> 33);
    }
    if (i < n) {
        uint64_t w = 0;
        std::memcpy(&w, b + i, n - i);
        h = (h ^ w) * 0x9E3779B97F4A7C15ull;
        h = (h << 31) | (h >> 33);
    }
    return h;
}

// Checksum of a file: the header with its checksum field zeroed, then every section.  A corrupted
// count or flag in the header fails verification even in a file without a handle table.
uint64_t file_checksum(const Header& h, const void* const ptrs[5], const size_t lens[5]) {
    Header z = h;
    z.checksum = 0;
    uint64_t c = mix(0x243F6A8885A308D3ull, &z, sizeof(z));
    for (int k = 0; k < 5; ++k) c = mix(c, ptrs[k], lens[k]);
    return c;
}

struct Sections {
    size_t off[5] = {0, 0, 0, 0, 0};
    size_t len[5] = {0, 0, 0, 0, 0};
    size_t total = 0;
};

Sections layout(int64_t A, int64_t M, int64_t P, uint32_t flags, uint32_t hb) {
    Sections s;
    size_t at = sizeof(Header);
    const size_t lens[5] = {4 * (size_t)M, 8 * (size_t)(M + 1), 4 * (size_t)P, (flags & 1) ? 4 * (size_t)M : 0,
                            (flags & 2) ? (size_t)A * hb : 0};
    for (int k = 0; k < 5; ++k) {
        s.off[k] = at;
        s.len[k] = lens[k];
        at = align64(at + lens[k]);
    }
    s.total = at;
    return s;
}

// A read-only mapping of a .hgcsr file with its header validated.
struct Mapped {
    int fd = -1;
    void* base = MAP_FAILED;
    size_t size = 0;
    Header h{};
    Sections s;
    ~Mapped() {
        if (base != MAP_FAILED) munmap(base, size);
        if (fd >= 0) close(fd);
    }
    const char* at(int k) const { return (const char*)base + s.off[k]; }
};

std::unique_ptr<Mapped> map_file(const char* path, bool verify) {
    std::unique_ptr<Mapped> m(new Mapped());
    m->fd = open(path, O_RDONLY);
    if (m->fd < 0) fail(HGX_E_NOTFOUND, std::string("hgcsr: cannot open ") + path);
    struct stat st;
    if (fstat(m->fd, &st) != 0 || (size_t)st.st_size < sizeof(Header)) fail(HGX_E_INVALID, "hgcsr: file too short");
    m->size = (size_t)st.st_size;
    m->base = mmap(nullptr, m->size, PROT_READ, MAP_PRIVATE, m->fd, 0);
    if (m->base == MAP_FAILED) fail(HGX_E_NOMEM, "hgcsr: mmap failed");
    std::memcpy(&m->h, m->base, sizeof(Header));
    const Header& h = m->h;
    if (std::memcmp(h.magic, kMagic, 8) != 0) fail(HGX_E_INVALID, "hgcsr: bad magic");
    if (h.version != kVersion) fail(HGX_E_UNSUPPORTED, "hgcsr: unsupported version");
    if (h.num_atoms < 0 || h.num_links < 0 || h.num_pins < 0 || h.num_links > h.num_atoms ||
        h.num_atoms >= (int64_t)INT32_MAX || h.handle_bytes > 64 || (h.flags & ~3u))
        fail(HGX_E_INVALID, "hgcsr: bad header");
    m->s = layout(h.num_atoms, h.num_links, h.num_pins, h.flags, h.handle_bytes);
    if (m->s.total > m->size) fail(HGX_E_INVALID, "hgcsr: truncated file");
    if (verify) {
        const void* ptrs[5];
        for (int k = 0; k < 5; ++k) ptrs[k] = m->at(k);
        if (file_checksum(h, ptrs, m->s.len) != h.checksum) fail(HGX_E_INVALID, "hgcsr: checksum mismatch");
        const int64_t* off = (const int64_t*)m->at(1);
        if (off[0] != 0 || off[h.num_links] != h.num_pins) fail(HGX_E_INVALID, "hgcsr: inconsistent offsets");
    }
    return m;
}

void write_all(FILE* f, const void* p, size_t n) {
    if (n && std::fwrite(p, 1, n, f) != n) fail(HGX_E_DEVICE, "hgcsr: write failed");
}

// D2H of the snapshot rows of a device graph (link_atom, tgt_off, tgt_idx, link_type).
void download(hgx_graph* g, std::vector<int32_t>& la, std::vector<int64_t>& off, std::vector<int32_t>& tg,
              std::vector<int32_t>& ty) {
    la.resize((size_t)g->M);
    off.resize((size_t)g->M + 1);
    tg.resize((size_t)g->P);
    ty.resize((size_t)g->M);
    if (g->M) HGX_HIP(hipMemcpyAsync(la.data(), g->link_atom, 4 * g->M, hipMemcpyDeviceToHost, g->stream));
    HGX_HIP(hipMemcpyAsync(off.data(), g->tgt_off, 8 * (g->M + 1), hipMemcpyDeviceToHost, g->stream));
    if (g->P) HGX_HIP(hipMemcpyAsync(tg.data(), g->tgt_idx, 4 * g->P, hipMemcpyDeviceToHost, g->stream));
    if (g->M) HGX_HIP(hipMemcpyAsync(ty.data(), g->link_type, 4 * g->M, hipMemcpyDeviceToHost, g->stream));
    HGX_HIP(hipStreamSynchronize(g->stream));
}

}  // namespace

// A streaming .hgcsr writer: the rows at begin, the handle table in any number of pieces (an exporter
// walking a store larger than one Java array never holds the whole table), the checksum run alongside;
// end patches the header and renames the file into place, abort removes the partial file.
struct hgx_snapshot_writer {
    std::string path, tmp;
    FILE* f = nullptr;
    Header h{};
    Sections s;
    uint64_t c = 0;           // running checksum
    uint8_t carry[8] = {0};   // handle bytes of a partial checksum word
    size_t carry_n = 0;
    int64_t ranks = 0;        // handles written so far
    bool failed = false;
    ~hgx_snapshot_writer() {
        if (f) std::fclose(f);
        if (!tmp.empty()) std::remove(tmp.c_str());
    }
};

extern "C" {

int hgx_snapshot_writer_begin(const char* path, const hgx_graph_desc* d, int32_t handle_bytes,
                              hgx_snapshot_writer** out) {
    HGX_API_BEGIN
    if (!path || !d || !out || handle_bytes < 0 || handle_bytes > 64)
        fail(HGX_E_INVALID, "hgx_snapshot_write: bad argument");
    *out = nullptr;
    const int64_t A = d->num_atoms, M = d->num_links;
    if (A < 0 || M < 0 || M > A || (M > 0 && (!d->link_atom || !d->tgt_off || !d->tgt_idx)))
        fail(HGX_E_INVALID, "hgx_snapshot_write: bad snapshot");
    const int64_t P = M > 0 ? d->tgt_off[M] : 0;
    if (M > 0 && d->tgt_off[0] != 0) fail(HGX_E_INVALID, "hgx_snapshot_write: tgt_off[0] != 0");
    for (int64_t r = 0; r < M; ++r)
        if (d->link_atom[r] < 0 || d->link_atom[r] >= A || (r && d->link_atom[r - 1] >= d->link_atom[r]) ||
            d->tgt_off[r + 1] < d->tgt_off[r])
            fail(HGX_E_INVALID, "hgx_snapshot_write: link rows not ascending / offsets not monotone");
    for (int64_t p = 0; p < P; ++p)
        if (d->tgt_idx[p] < 0 || d->tgt_idx[p] >= A) fail(HGX_E_INVALID, "hgx_snapshot_write: target out of range");
    std::unique_ptr<hgx_snapshot_writer> w(new hgx_snapshot_writer());
    Header& h = w->h;
    std::memcpy(h.magic, kMagic, 8);
    h.version = kVersion;
    h.flags = (d->link_type ? 1u : 0u) | (handle_bytes > 0 ? 2u : 0u);
    h.num_atoms = A;
    h.num_links = M;
    h.num_pins = P;
    h.handle_bytes = (uint32_t)handle_bytes;
    h.checksum = 0;
    w->s = layout(A, M, P, h.flags, h.handle_bytes);
    w->path = path;
    w->tmp = w->path + ".tmp";
    w->f = std::fopen(w->tmp.c_str(), "wb");
    if (!w->f) fail(HGX_E_DEVICE, std::string("hgx_snapshot_write: cannot create ") + w->tmp);
    // the header (its checksum patched in at the end), then the four row sections; the checksum runs
    // over the header with a zero checksum field and then every section in order (file_checksum)
    write_all(w->f, &h, sizeof(h));
    w->c = mix(0x243F6A8885A308D3ull, &h, sizeof(h));
    const int64_t zero_off = 0;
    const void* ptrs[4] = {d->link_atom, M ? (const void*)d->tgt_off : (const void*)&zero_off, d->tgt_idx, d->link_type};
    size_t at = sizeof(Header);
    static const char zeros[64] = {0};
    for (int k = 0; k < 4; ++k) {
        write_all(w->f, zeros, w->s.off[k] - at);
        write_all(w->f, ptrs[k], w->s.len[k]);
        w->c = mix(w->c, ptrs[k], w->s.len[k]);
        at = w->s.off[k] + w->s.len[k];
    }
    write_all(w->f, zeros, w->s.off[4] - at);
    *out = w.release();
    HGX_API_END
}

int hgx_snapshot_writer_handles(hgx_snapshot_writer* w, const uint8_t* handles, int64_t n_ranks) {
    HGX_API_BEGIN
    if (!w || n_ranks < 0 || (n_ranks > 0 && !handles) || w->failed)
        fail(HGX_E_INVALID, "hgx_snapshot_writer_handles: bad argument");
    const size_t hb = w->h.handle_bytes;
    if (n_ranks > 0 && hb == 0) fail(HGX_E_INVALID, "hgx_snapshot_writer_handles: the snapshot has no handle table");
    if (n_ranks > w->h.num_atoms - w->ranks) fail(HGX_E_INVALID, "hgx_snapshot_writer_handles: more ranks than num_atoms");
    const size_t n = (size_t)n_ranks * hb;
    try {
        write_all(w->f, handles, n);
    } catch (...) {
        w->failed = true;
        throw;
    }
    // streamed checksum: whole 8-byte words, a partial one carried to the next call (zero-padded at the end)
    size_t i = 0;
    while (i < n && w->carry_n > 0 && w->carry_n < 8) w->carry[w->carry_n++] = handles[i++];
    if (w->carry_n == 8) {
        w->c = mix(w->c, w->carry, 8);
        w->carry_n = 0;
    }
    const size_t whole = (n - i) & ~(size_t)7;
    w->c = mix(w->c, handles + i, whole);
    i += whole;
    while (i < n) w->carry[w->carry_n++] = handles[i++];
    w->ranks += n_ranks;
    HGX_API_END
}

int hgx_snapshot_writer_handle_bytes(const hgx_snapshot_writer* w, int32_t* handle_bytes) {
    HGX_API_BEGIN
    if (!w || !handle_bytes) fail(HGX_E_INVALID, "hgx_snapshot_writer_handle_bytes: bad argument");
    *handle_bytes = (int32_t)w->h.handle_bytes;
    HGX_API_END
}

int hgx_snapshot_writer_end(hgx_snapshot_writer* w) {
    HGX_API_BEGIN
    if (!w) fail(HGX_E_INVALID, "hgx_snapshot_writer_end: null writer");
    std::unique_ptr<hgx_snapshot_writer> own(w);
    if (w->failed) fail(HGX_E_DEVICE, "hgx_snapshot_write: an earlier write failed");
    if (w->h.handle_bytes > 0 && w->ranks != w->h.num_atoms)
        fail(HGX_E_INVALID, "hgx_snapshot_writer_end: " + std::to_string(w->ranks) + " of " +
                                std::to_string(w->h.num_atoms) + " handles written");
    if (w->carry_n) w->c = mix(w->c, w->carry, w->carry_n);
    static const char zeros[64] = {0};
    write_all(w->f, zeros, w->s.total - (w->s.off[4] + w->s.len[4]));
    w->h.checksum = w->c;
    if (std::fseek(w->f, 0, SEEK_SET) != 0) fail(HGX_E_DEVICE, "hgx_snapshot_write: seek failed");
    write_all(w->f, &w->h, sizeof(Header));
    // durable before it becomes visible under the final name
    if (std::fflush(w->f) != 0 || fsync(fileno(w->f)) != 0) fail(HGX_E_DEVICE, "hgx_snapshot_write: fsync failed");
    FILE* f = w->f;
    w->f = nullptr;
    if (std::fclose(f) != 0) fail(HGX_E_DEVICE, "hgx_snapshot_write: close failed");
    if (std::rename(w->tmp.c_str(), w->path.c_str()) != 0) fail(HGX_E_DEVICE, "hgx_snapshot_write: rename failed");
    w->tmp.clear();
    HGX_API_END
}

void hgx_snapshot_writer_abort(hgx_snapshot_writer* w) { delete w; }

int hgx_snapshot_write(const char* path, const hgx_graph_desc* d, const uint8_t* handles, int32_t handle_bytes) {
    if (handle_bytes > 0 && !handles) {
        set_last_error("hgx_snapshot_write: bad argument");
        return HGX_E_INVALID;
    }
    hgx_snapshot_writer* w = nullptr;
    int rc = hgx_snapshot_writer_begin(path, d, handle_bytes, &w);
    if (rc) return rc;
    if (handle_bytes > 0) rc = hgx_snapshot_writer_handles(w, handles, d->num_atoms);
    if (rc) {
        hgx_snapshot_writer_abort(w);
        return rc;
    }
    return hgx_snapshot_writer_end(w);
}

int hgx_snapshot_info(const char* path, int64_t* num_atoms, int64_t* num_links, int64_t* num_pins,
                      int32_t* handle_bytes, int32_t* has_types) {
    HGX_API_BEGIN
    if (!path) fail(HGX_E_INVALID, "hgx_snapshot_info: null path");
    auto m = map_file(path, false);
    if (num_atoms) *num_atoms = m->h.num_atoms;
    if (num_links) *num_links = m->h.num_links;
    if (num_pins) *num_pins = m->h.num_pins;
    if (handle_bytes) *handle_bytes = (m->h.flags & 2) ? (int32_t)m->h.handle_bytes : 0;
    if (has_types) *has_types = (m->h.flags & 1) ? 1 : 0;
    HGX_API_END
}

int hgx_snapshot_read(const char* path, int32_t* link_atom, int64_t* tgt_off, int32_t* tgt_idx, int32_t* link_type,
                      uint8_t* handles) {
    HGX_API_BEGIN
    if (!path) fail(HGX_E_INVALID, "hgx_snapshot_read: null path");
    auto m = map_file(path, true);
    void* dst[5] = {link_atom, tgt_off, tgt_idx, link_type, handles};
    for (int k = 0; k < 5; ++k)
        if (dst[k] && m->s.len[k]) std::memcpy(dst[k], m->at(k), m->s.len[k]);
    if (link_type && !(m->h.flags & 1)) std::memset(link_type, 0, 4 * (size_t)m->h.num_links);
    HGX_API_END
}

int hgx_snapshot_read_handles(const char* path, int64_t first_rank, int64_t n, int32_t verify, uint8_t* out) {
    HGX_API_BEGIN
    if (!path || n < 0 || first_rank < 0 || (n > 0 && !out)) fail(HGX_E_INVALID, "hgx_snapshot_read_handles: bad argument");
    auto m = map_file(path, verify != 0);
    if (!(m->h.flags & 2)) fail(HGX_E_NOTFOUND, "hgx_snapshot_read_handles: the file has no handle table");
    if (first_rank > m->h.num_atoms || n > m->h.num_atoms - first_rank)
        fail(HGX_E_INVALID, "hgx_snapshot_read_handles: ranks outside [0, num_atoms)");
    const size_t hb = m->h.handle_bytes;
    if (n) std::memcpy(out, m->at(4) + (size_t)first_rank * hb, (size_t)n * hb);
    HGX_API_END
}

int hgx_graph_open(const char* path, int32_t device, hgx_graph** out) {
    HGX_API_BEGIN
    if (!path || !out) fail(HGX_E_INVALID, "hgx_graph_open: bad argument");
    *out = nullptr;
    auto m = map_file(path, true);
    const Header& h = m->h;
    hgx_graph_desc d{h.num_atoms, h.num_links, (const int32_t*)m->at(0), (const int64_t*)m->at(1),
                     (const int32_t*)m->at(2), (h.flags & 1) ? (const int32_t*)m->at(3) : nullptr};
    *out = graph_create(&d, device, true);
    HGX_API_END
}

int hgx_graph_export(hgx_graph* g, int32_t* link_atom, int64_t* tgt_off, int32_t* tgt_idx, int32_t* link_type) {
    HGX_API_BEGIN
    if (!g) fail(HGX_E_INVALID, "hgx_graph_export: null graph");
    if (g->shard) fail(HGX_E_UNSUPPORTED, "hgx_graph_export: not available on a partition shard");
    std::lock_guard<std::mutex> lk(g->mu);
    HGX_HIP(hipSetDevice(g->device));
    std::vector<int32_t> la, tg, ty;
    std::vector<int64_t> off;
    download(g, la, off, tg, ty);
    if (link_atom) std::memcpy(link_atom, la.data(), 4 * la.size());
    if (tgt_off) std::memcpy(tgt_off, off.data(), 8 * off.size());
    if (tgt_idx) std::memcpy(tgt_idx, tg.data(), 4 * tg.size());
    if (link_type) std::memcpy(link_type, ty.data(), 4 * ty.size());
    HGX_API_END
}

int hgx_graph_update(hgx_graph* g, int64_t num_atoms, int64_t n_add, const int32_t* add_link_atom,
                     const int64_t* add_tgt_off, const int32_t* add_tgt_idx, const int32_t* add_link_type,
                     int64_t n_remove, const int32_t* remove_link_atom) {
    HGX_API_BEGIN
    if (!g || n_add < 0 || n_remove < 0 || (n_add > 0 && (!add_link_atom || !add_tgt_off || !add_tgt_idx)) ||
        (n_remove > 0 && !remove_link_atom))
        fail(HGX_E_INVALID, "hgx_graph_update: bad argument");
    if (g->shard) fail(HGX_E_UNSUPPORTED, "hgx_graph_update: not available on a partition shard");
    if (num_atoms < g->A) fail(HGX_E_INVALID, "hgx_graph_update: atoms cannot disappear from the id space");
    std::lock_guard<std::mutex> lk(g->mu);
    if (g->base) fail(HGX_E_INVALID, "hgx_graph_update: apply store events to the snapshot, not to one of its contexts");
    if (g->refs.load() > 1)
        fail(HGX_E_INVALID, "hgx_graph_update: results or execution contexts of this graph are still alive");
    HGX_HIP(hipSetDevice(g->device));
    std::vector<int32_t> la, tg, ty;
    std::vector<int64_t> off;
    download(g, la, off, tg, ty);
    // merge: drop removed rows, insert added rows, keep link atom order (ascending rank)
    std::vector<int32_t> rm(remove_link_atom, remove_link_atom + n_remove);
    std::sort(rm.begin(), rm.end());
    std::vector<int64_t> add_order((size_t)n_add);
    for (int64_t i = 0; i < n_add; ++i) add_order[i] = i;
    std::sort(add_order.begin(), add_order.end(),
              [&](int64_t a, int64_t b) { return add_link_atom[a] < add_link_atom[b]; });
    std::vector<int32_t> nla, ntg, nty;
    std::vector<int64_t> noff{0};
    nla.reserve(la.size() + n_add);
    auto push_old = [&](int64_t r) {
        nla.push_back(la[r]);
        nty.push_back(ty[r]);
        ntg.insert(ntg.end(), tg.begin() + off[r], tg.begin() + off[r + 1]);
        noff.push_back((int64_t)ntg.size());
    };
    auto push_new = [&](int64_t i) {
        nla.push_back(add_link_atom[i]);
        nty.push_back(add_link_type ? add_link_type[i] : 0);
        ntg.insert(ntg.end(), add_tgt_idx + add_tgt_off[i], add_tgt_idx + add_tgt_off[i + 1]);
        noff.push_back((int64_t)ntg.size());
    };
    for (size_t i = 1; i < add_order.size(); ++i)
        if (add_link_atom[add_order[i]] == add_link_atom[add_order[i - 1]])
            fail(HGX_E_INVALID, "hgx_graph_update: a link is added twice in one batch");
    // Removals apply before additions: removing and adding the same link atom in one batch is a
    // replace (HyperGraph.replace keeps the handle and rewrites type + targets, C/HyperGraph.java:
    // 2100-2141, announced as HGAtomReplacedEvent); the new row takes the old row's rank slot.
    size_t ai = 0;
    for (int64_t r = 0; r < (int64_t)la.size(); ++r) {
        while (ai < add_order.size() && add_link_atom[add_order[ai]] < la[r]) push_new(add_order[ai++]);
        const bool removed = std::binary_search(rm.begin(), rm.end(), la[r]);
        if (ai < add_order.size() && add_link_atom[add_order[ai]] == la[r]) {
            if (!removed) fail(HGX_E_INVALID, "hgx_graph_update: an added link already exists");
            push_new(add_order[ai++]);   // replace
            continue;
        }
        if (!removed) push_old(r);
    }
    while (ai < add_order.size()) push_new(add_order[ai++]);
    hgx_graph_desc d{num_atoms, (int64_t)nla.size(), nla.data(), noff.data(), ntg.data(), nty.data()};
    hgx_graph* fresh = graph_create(&d, g->device, true);   // validates ids and order
    // move the fresh device arrays into g (same object: handles held by callers stay valid)
    std::swap(g->A, fresh->A);
    std::swap(g->M, fresh->M);
    std::swap(g->P, fresh->P);
    std::swap(g->I, fresh->I);
    std::swap(g->link_atom, fresh->link_atom);
    std::swap(g->tgt_off, fresh->tgt_off);
    std::swap(g->tgt_idx, fresh->tgt_idx);
    std::swap(g->link_type, fresh->link_type);
    std::swap(g->inc_off, fresh->inc_off);
    std::swap(g->inc_row, fresh->inc_row);
    std::swap(g->inc_type, fresh->inc_type);
    std::swap(g->inc_ts_row, fresh->inc_ts_row);
    std::swap(g->inc_ts_type, fresh->inc_ts_type);
    std::swap(g->inc_ts_tgt, fresh->inc_ts_tgt);
    std::swap(g->n_heavy, fresh->n_heavy);
    std::swap(g->I_heavy, fresh->I_heavy);
    std::swap(g->n_chunks, fresh->n_chunks);
    std::swap(g->heavy_atom, fresh->heavy_atom);
    std::swap(g->chunks, fresh->chunks);
    if (num_atoms > fresh->A) g->ranks_ordered = false;   // appended ranks (fresh->A = the old count)
    g->max_arity = g->max_deg = -1;
    g->inc_off_host.clear();
    if (g->zacc) (void)hipFree(g->zacc);
    g->zacc = nullptr;
    if (g->hasinc) (void)hipFree(g->hasinc);
    g->hasinc = nullptr;
    if (g->inc_yf) (void)hipFree(g->inc_yf);
    g->inc_yf = nullptr;
    free_yield_lists(g);
    if (g->co_vis) (void)hipFree(g->co_vis);   // per-seed bitmaps sized by the old atom count
    g->co_vis = nullptr;
    g->co_vis_seeds = 0;
    if (g->pchunks) (void)hipFree(g->pchunks);
    g->pchunks = nullptr;
    g->n_pchunks = -1;
    g->zacc_bytes = 0;
    g->zacc_clean = false;
    graph_release(fresh);   // frees the old arrays now held by `fresh`
    HGX_API_END
}

}  // extern "C"
