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
    for (auto& p : pin) CK(hipHostMalloc((void**)&p, chunk, hipHostMallocDefault));
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
