// Micro-benchmark (profiling aid): ways to move a FASTQ file's bytes (page cache) to the GPU.
//   (a) hipMemcpy from a private read-only mmap of the file (pageable)
//   (b) hipHostRegister of mmap'd chunks, then hipMemcpyAsync (pinned)
//   (c) pread by T threads into pinned chunks, then hipMemcpyAsync
//   (d) memcpy from the mmap into pinned chunks by T threads, then hipMemcpyAsync
// Usage: h2d <file> [chunk_MB] [threads]
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

#define CK(x)                                                               \
    do {                                                                    \
        hipError_t e_ = (x);                                                \
        if (e_ != hipSuccess) {                                             \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));         \
            exit(1);                                                        \
        }                                                                   \
    } while (0)

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    const size_t chunk = (argc > 2 ? atol(argv[2]) : 256) << 20;
    const int T = argc > 3 ? atoi(argv[3]) : 8;
    int fd = open(argv[1], O_RDONLY);
    struct stat st;
    fstat(fd, &st);
    const size_t size = st.st_size;
    char* map = (char*)mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
    char* dev = nullptr;
    CK(hipMalloc(&dev, chunk));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipFree(nullptr));
    // warm the page cache
    {
        volatile unsigned long long x = 0;
        for (size_t i = 0; i < size; i += 4096) x += map[i];
    }
    double t0 = now();
    for (size_t o = 0; o < size; o += chunk) CK(hipMemcpyAsync(dev, map + o, std::min(chunk, size - o), hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));
    double t = now() - t0;
    printf("(a) pageable mmap H2D: %.3f s, %.1f GB/s\n", t, size / t / 1e9);

    t0 = now();
    double treg = 0;
    for (size_t o = 0; o < size; o += chunk) {
        const size_t n = std::min(chunk, size - o);
        double r0 = now();
        hipError_t e = hipHostRegister(map + o, n, hipHostRegisterReadOnly);
        treg += now() - r0;
        if (e != hipSuccess) {
            printf("(b) hipHostRegister failed: %s\n", hipGetErrorString(e));
            break;
        }
        CK(hipMemcpyAsync(dev, map + o, n, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
        (void)hipHostUnregister(map + o);
    }
    t = now() - t0;
    printf("(b) register + pinned H2D: %.3f s (register %.3f s), %.1f GB/s\n", t, treg, size / t / 1e9);

    std::vector<char*> pin(2);
    {
        double a0 = now();
        for (auto& p : pin) CK(hipHostMalloc((void**)&p, chunk, hipHostMallocDefault));
        double a = now() - a0;
        printf("hipHostMalloc 2 x %zu MB: %.3f s (%.2f s per GB)\n", chunk >> 20, a, a / (2.0 * chunk / 1e9));
        char* big = nullptr;
        a0 = now();
        CK(hipHostMalloc((void**)&big, (size_t)1 << 30, hipHostMallocPortable));
        double a1 = now();
        memset(big, 1, (size_t)1 << 30);
        double a2 = now();
        CK(hipHostFree(big));
        printf("hipHostMalloc 1 GiB portable: alloc %.3f s, first touch %.3f s, free %.3f s\n", a1 - a0, a2 - a1, now() - a2);
        for (int huge = 0; huge < 2; ++huge) {
            const size_t G = (size_t)1 << 30;
            double b0 = now();
            char* m = (char*)mmap(nullptr, G, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
            if (huge) madvise(m, G, MADV_HUGEPAGE);
            memset(m, 0, G);
            double b1 = now();
            hipError_t e = hipHostRegister(m, G, hipHostRegisterPortable);
            double b2 = now();
            CK(hipMemcpyAsync(dev, m, chunk, hipMemcpyHostToDevice, s));
            CK(hipStreamSynchronize(s));
            double b3 = now();
            CK(hipMemcpyAsync(dev, m, chunk, hipMemcpyHostToDevice, s));
            CK(hipStreamSynchronize(s));
            double b4 = now();
            (void)hipHostUnregister(m);
            double b5 = now();
            munmap(m, G);
            printf("anon 1 GiB%s: mmap+touch %.3f s, register %.3f s (%s), H2D %zu MB %.1f GB/s, unregister %.3f s, munmap %.3f s\n",
                   huge ? " (THP)" : "", b1 - b0, b2 - b1, hipGetErrorString(e), chunk >> 20, chunk / (b4 - b3) / 1e9, b5 - b4, now() - b5);
            (void)b3;
        }
    }
    auto par = [&](char* dst, size_t o, size_t n, bool use_pread) {
        std::vector<std::thread> th;
        const size_t per = (n + T - 1) / T;
        for (int i = 0; i < T; ++i) {
            const size_t a = i * per, b = std::min(n, a + per);
            if (a >= b) break;
            th.emplace_back([&, a, b] {
                if (use_pread) {
                    size_t d = a;
                    while (d < b) {
                        ssize_t r = pread(fd, dst + d, b - d, o + d);
                        if (r <= 0) break;
                        d += r;
                    }
                } else {
                    memcpy(dst + a, map + o + a, b - a);
                }
            });
        }
        for (auto& x : th) x.join();
    };
    for (int mode = 0; mode < 2; ++mode) {
        t0 = now();
        double tcpu = 0;
        int k = 0;
        for (size_t o = 0; o < size; o += chunk, k ^= 1) {
            const size_t n = std::min(chunk, size - o);
            CK(hipStreamSynchronize(s));  // (double buffer: the copy of k's previous use is done)
            double c0 = now();
            par(pin[k], o, n, mode == 0);
            tcpu += now() - c0;
            CK(hipMemcpyAsync(dev, pin[k], n, hipMemcpyHostToDevice, s));
        }
        CK(hipStreamSynchronize(s));
        t = now() - t0;
        printf("(%c) %s x%d threads into pinned + H2D: %.3f s (host copy %.3f s), %.1f GB/s\n", mode ? 'd' : 'c',
               mode ? "memcpy from mmap" : "pread", T, t, tcpu, size / t / 1e9);
    }
    t0 = now();
    par(pin[0], 0, std::min(chunk, size), false);
    t = now() - t0;
    printf("memcpy mmap -> pinned, one chunk: %.1f GB/s\n", std::min(chunk, size) / t / 1e9);
    return 0;
}
