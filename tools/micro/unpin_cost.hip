// Profiling aid: does hipHostUnregister wait for work in flight, and what does releasing page-locked
// memory cost when done explicitly (vs at exit, tools/micro/exit_cost)?
//   unpin_cost <pinned_MiB> <chunks> <busy_ms> [threads]   (release on `threads` threads)
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <unistd.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>
__global__ void busy(long long cycles, int* out) {  // bounded: every wave leaves after `cycles` clocks
    const long long t0 = wall_clock64();
    while (wall_clock64() - t0 < cycles) {
    }
    if (threadIdx.x == 0) out[blockIdx.x] = 1;
}
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
int main(int argc, char** argv) {
    const size_t pin = (size_t)atoll(argv[1]) << 20;
    const int chunks = atoi(argv[2]);
    const int busy_ms = atoi(argv[3]);
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n < 1) return 2;
    hipSetDevice(0);
    std::vector<void*> keep;
    const size_t b = pin / chunks;
    for (int c = 0; c < chunks; ++c) {
        void* p = mmap(nullptr, b, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        madvise(p, b, MADV_HUGEPAGE);
        memset(p, 1, b);
        if (hipHostRegister(p, b, hipHostRegisterDefault) != hipSuccess) return 3;
        keep.push_back(p);
    }
    int* d = nullptr;
    hipMalloc(&d, 4096 * sizeof(int));
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    // wall_clock64: 100 MHz on gfx950, busy_ms * 1e5 ticks
    hipLaunchKernelGGL(busy, dim3(256), dim3(64), 0, s, (long long)busy_ms * 100000LL, d);
    const double t0 = now();
    const int nt = argc > 4 ? atoi(argv[4]) : 1;
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t)
        th.emplace_back([&, t] {
            for (size_t i = (size_t)t; i < keep.size(); i += (size_t)nt) {
                hipHostUnregister(keep[i]);
                munmap(keep[i], b);
            }
        });
    for (auto& x : th) x.join();
    const double t1 = now();
    const bool still = hipStreamQuery(s) == hipErrorNotReady;
    hipStreamSynchronize(s);
    const double t2 = now();
    std::printf("release %.3f s (kernel still running after it: %s), kernel done %.3f s after launch\n", t1 - t0,
                still ? "yes" : "no", t2 - t0);
    std::printf("mono %.6f\n", now());
    std::fflush(stdout);
    _exit(0);
}
