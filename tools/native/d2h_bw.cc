// Device-to-host copy bandwidth on this box (the order-exact engine's pair copies are its call's floor):
// hipMemcpyAsync from device memory into pinned host memory, by host allocation kind (hipHostMalloc
// mapped / default / coherent, hipHostRegister of an mmap'd region), size, offset alignment and number of
// copy streams.  Build: hipcc --offload-arch=gfx950 -O2 -o tools/native/build/d2h_bw tools/native/d2h_bw.cc
#include <hip/hip_runtime.h>

#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                       \
        }                                                                                       \
    } while (0)

static double run(char* dst, const char* src, size_t bytes, size_t off, int nstreams, hipStream_t* st, int reps) {
    // nstreams copies of bytes / nstreams each, side by side; best of reps
    double best = 1e30;
    for (int r = 0; r < reps; ++r) {
        CK(hipDeviceSynchronize());
        const auto t0 = std::chrono::steady_clock::now();
        const size_t piece = bytes / nstreams;
        for (int k = 0; k < nstreams; ++k)
            CK(hipMemcpyAsync(dst + off + k * piece, src + off + k * piece, piece, hipMemcpyDeviceToHost, st[k]));
        for (int k = 0; k < nstreams; ++k) CK(hipStreamSynchronize(st[k]));
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (s < best) best = s;
    }
    return bytes / best / 1e9;
}

// streams HBM (read + write) until *stop: the engine's ranking kernels beside its copies
__global__ void busy(const float4* a, float4* b, size_t n, int iters) {
    for (int it = 0; it < iters; ++it)
        for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
            float4 v = a[i];
            v.x += 1.0f;
            b[i] = v;
        }
}

// consecutive copies walking a large pinned buffer (the engine's level buffer), optionally beside a kernel
static void walk(size_t total, size_t piece, bool with_kernel) {
    char *d = nullptr, *h = nullptr;
    CK(hipMalloc(&d, total));
    CK(hipMemset(d, 1, total));
    CK(hipHostMalloc(&h, total, hipHostMallocMapped));
    std::memset(h, 0, total);
    float4 *ka = nullptr, *kb = nullptr;
    const size_t kn = ((size_t)1 << 30) / sizeof(float4);
    hipStream_t cs, ks;
    CK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&ks, hipStreamNonBlocking));
    if (with_kernel) {
        CK(hipMalloc(&ka, kn * sizeof(float4)));
        CK(hipMalloc(&kb, kn * sizeof(float4)));
    }
    for (int rep = 0; rep < 2; ++rep) {
        CK(hipDeviceSynchronize());
        if (with_kernel) busy<<<4096, 256, 0, ks>>>(ka, kb, kn, 40);
        const auto t0 = std::chrono::steady_clock::now();
        for (size_t o = 0; o + piece <= total; o += piece) CK(hipMemcpyAsync(h + o, d + o, piece, hipMemcpyDeviceToHost, cs));
        CK(hipStreamSynchronize(cs));
        const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        CK(hipDeviceSynchronize());
        std::printf("walk %zu MB in %zu MB copies%s: %.1f GB/s\n", total >> 20, piece >> 20,
                    with_kernel ? " beside an HBM-streaming kernel" : "", (total / piece * piece) / sec / 1e9);
    }
    CK(hipHostFree(h));
    CK(hipFree(d));
    if (ka) CK(hipFree(ka));
    if (kb) CK(hipFree(kb));
}

int main(int argc, char** argv) {
    if (argc > 1 && argv[1][0] == 'n') {   // NUMA placement of the pinned buffer (mbind before the first touch)
        int dev = 0;
        char bus[64] = {0};
        CK(hipDeviceGetPCIBusId(bus, sizeof(bus), dev));
        for (char* c = bus; *c; ++c) *c = (char)std::tolower(*c);
        char path[256];
        std::snprintf(path, sizeof(path), "/sys/bus/pci/devices/%s/numa_node", bus);
        FILE* f = std::fopen(path, "r");
        int gnode = -2;
        if (f) {
            if (std::fscanf(f, "%d", &gnode) != 1) gnode = -3;
            std::fclose(f);
        }
        std::printf("GPU %s numa_node %d\n", bus, gnode);
        hipStream_t s1;
        CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
        const size_t sz = (size_t)1 << 30;
        char* dd = nullptr;
        CK(hipMalloc(&dd, sz));
        for (int node = -1; node < 8; ++node) {
            void* p = mmap(nullptr, sz, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
            if (node >= 0) {
                unsigned long mask[16] = {0};
                mask[node / 64] = 1ul << (node % 64);
                if (syscall(SYS_mbind, p, sz, 2 /* MPOL_BIND */, mask, 1024, 0) != 0) {
                    munmap(p, sz);
                    continue;   // no such node
                }
            }
            std::memset(p, 0, sz);
            CK(hipHostRegister(p, sz, hipHostRegisterMapped));
            double g = 0;
            for (int r = 0; r < 3; ++r) g = std::max(g, run((char*)p, dd, (size_t)96 << 20, 0, 1, &s1, 3));
            int where = -1;
            void* pp[1] = {p};
            int st_[1] = {-1};
            syscall(SYS_move_pages, 0, 1, pp, nullptr, st_, 0);
            where = st_[0];
            std::printf("pinned buffer bound to node %d (pages on node %d): %.1f GB/s\n", node, where, g);
            CK(hipHostUnregister(p));
            munmap(p, sz);
        }
        char* hh = nullptr;
        for (int k = 0; k < 4; ++k) {
            CK(hipHostMalloc(&hh, sz, hipHostMallocMapped));
            std::memset(hh, 0, sz);
            void* pp[1] = {hh};
            int st_[1] = {-1};
            syscall(SYS_move_pages, 0, 1, pp, nullptr, st_, 0);
            std::printf("hipHostMalloc #%d (pages on node %d): %.1f GB/s\n", k, st_[0], run(hh, dd, (size_t)96 << 20, 0, 1, &s1, 5));
            CK(hipHostFree(hh));
        }
        return 0;
    }
    if (argc > 1 && argv[1][0] == 's') {   // odd sizes / offsets like the engine's packed part copies
        hipStream_t st[1];
        CK(hipStreamCreateWithFlags(&st[0], hipStreamNonBlocking));
        char *dd = nullptr, *hh = nullptr;
        CK(hipMalloc(&dd, (size_t)1 << 30));
        CK(hipHostMalloc(&hh, (size_t)1 << 30, hipHostMallocMapped));
        std::memset(hh, 0, (size_t)1 << 30);
        for (size_t sz : {(size_t)96600000, (size_t)96600003, (size_t)128800000, (size_t)54000000, (size_t)54000004})
            for (size_t off : {(size_t)0, (size_t)192 * 1000, (size_t)4 * 1001, (size_t)3 * 1001})
                std::printf("size %zu offset %zu: %.1f GB/s\n", sz, off, run(hh, dd, sz, off, 1, st, 5));
        return 0;
    }
    if (argc > 1) {   // walk mode only
        walk((size_t)2 << 30, (size_t)96 << 20, false);
        walk((size_t)2 << 30, (size_t)96 << 20, true);
        walk((size_t)2 << 30, (size_t)8 << 20, false);
        return 0;
    }
    const size_t big = (size_t)512 << 20;
    char* d = nullptr;
    CK(hipMalloc(&d, big + 4096));
    CK(hipMemset(d, 1, big + 4096));
    hipStream_t st[4];
    for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    struct Kind {
        const char* name;
        unsigned flags;
        int reg;   // 1: mmap + hipHostRegister
    } kinds[] = {{"hipHostMalloc mapped", hipHostMallocMapped, 0},
                 {"hipHostMalloc default", hipHostMallocDefault, 0},
                 {"hipHostMalloc coherent", hipHostMallocCoherent, 0},
                 {"hipHostMalloc noncoherent", hipHostMallocNonCoherent, 0},
                 {"mmap + hipHostRegister", 0, 1},
                 {"mmap(THP) + hipHostRegister", 0, 2}};
    for (const Kind& k : kinds) {
        char* h = nullptr;
        if (k.reg) {
            void* p = mmap(nullptr, big + 4096, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
            if (p == MAP_FAILED) return 1;
            if (k.reg == 2) madvise(p, big + 4096, MADV_HUGEPAGE);
            std::memset(p, 0, big + 4096);
            CK(hipHostRegister(p, big + 4096, hipHostRegisterDefault));
            h = (char*)p;
        } else {
            CK(hipHostMalloc(&h, big + 4096, k.flags));
        }
        for (size_t sz : {(size_t)32 << 20, (size_t)128 << 20, (size_t)512 << 20})
            for (size_t off : {(size_t)0, (size_t)4, (size_t)3})
                for (int ns : {1, 2, 4}) {
                    if (off != 0 && ns != 1) continue;
                    const double gbs = run(h, d, sz, off, ns, st, 5);
                    std::printf("%-30s size %4zu MB offset %zu streams %d: %6.1f GB/s\n", k.name, sz >> 20, off, ns, gbs);
                }
        std::fflush(stdout);
        if (k.reg) {
            CK(hipHostUnregister(h));
            munmap(h, big + 4096);
        } else {
            CK(hipHostFree(h));
        }
    }
    return 0;
}
