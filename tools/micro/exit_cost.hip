// Profiling aid: how long a process's exit takes after HIP work, by what it holds.
//   exit_cost <pinned_MiB> <device_MiB> <chunks> [hostmalloc]   (prints the stamp just before _exit; time the exit
//   from outside; hostmalloc 1: the page-locked memory from hipHostMalloc instead of registered THP)
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <unistd.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
int main(int argc, char** argv) {
    const size_t pin = (size_t)atoll(argv[1]) << 20, dev = (size_t)atoll(argv[2]) << 20;
    const int chunks = argc > 3 ? atoi(argv[3]) : 1;
    const bool hm = argc > 4 && atoi(argv[4]) != 0;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n < 1) return 2;
    hipSetDevice(0);
    hipFree(nullptr);
    const auto t_start = std::chrono::steady_clock::now();
    std::vector<void*> keep;
    for (int c = 0; c < chunks && pin; ++c) {
        const size_t b = pin / chunks;
        if (hm) {
            void* h = nullptr;
            if (hipHostMalloc(&h, b, hipHostMallocDefault) != hipSuccess) return 5;
            memset(h, 1, b);
            keep.push_back(h);
            continue;
        }
        void* p = mmap(nullptr, b, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        madvise(p, b, MADV_HUGEPAGE);
        memset(p, 1, b);
        if (hipHostRegister(p, b, hipHostRegisterDefault) != hipSuccess) return 3;
        keep.push_back(p);
    }
    for (int c = 0; c < chunks && dev; ++c) {
        void* d = nullptr;
        if (hipMalloc(&d, dev / chunks) != hipSuccess) return 4;
        hipMemset(d, 0, dev / chunks);
        keep.push_back(d);
    }
    hipDeviceSynchronize();
    const double t_alloc = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count();
    std::fprintf(stderr, "setup %.3f s\n", t_alloc);
    const double t = std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
    std::printf("mono %.6f\n", t);
    std::fflush(stdout);
    _exit(0);
}
