// Host <-> device transfer costs for the host-buffer frame path (diagnostic; GPU box).
// One 1080p BGR image = 6,220,800 bytes.  Build:
//   hipcc -O2 -std=c++17 pcie_rate.cpp -o pcie_rate -lpthread
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));       \
            std::exit(1);                                                      \
        }                                                                      \
    } while (0)

int main() {
    const size_t n = 1920 * 1080 * 3;
    const int reps = 20;
    void* dev;
    CK(hipMalloc(&dev, n));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    // fresh pageable buffers (as a new frame from a camera would be)
    std::vector<char*> bufs;
    for (int i = 0; i < reps + 2; ++i) {
        char* b = static_cast<char*>(std::malloc(n));
        std::memset(b, i, n);
        bufs.push_back(b);
    }
    double t0 = now_ms();
    for (int i = 0; i < reps; ++i) {
        CK(hipHostRegister(bufs[i], n, hipHostRegisterDefault));
        CK(hipMemcpyAsync(dev, bufs[i], n, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
        CK(hipHostUnregister(bufs[i]));
    }
    double t1 = now_ms();
    std::printf("register + H2D + unregister, 6.2 MB : %.3f ms\n", (t1 - t0) / reps);
    t0 = now_ms();
    for (int i = 0; i < reps; ++i) {
        CK(hipHostRegister(bufs[i], n, hipHostRegisterDefault));
        CK(hipHostUnregister(bufs[i]));
    }
    t1 = now_ms();
    std::printf("register + unregister only           : %.3f ms\n", (t1 - t0) / reps);
    t0 = now_ms();
    for (int i = 0; i < reps; ++i) {
        CK(hipMemcpyAsync(dev, bufs[i], n, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
    }
    t1 = now_ms();
    std::printf("pageable H2D, 6.2 MB                 : %.3f ms\n", (t1 - t0) / reps);
    char* pin;
    CK(hipHostMalloc(reinterpret_cast<void**>(&pin), n, hipHostMallocDefault));
    std::memset(pin, 1, n);
    t0 = now_ms();
    for (int i = 0; i < reps; ++i) {
        CK(hipMemcpyAsync(dev, pin, n, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
    }
    t1 = now_ms();
    std::printf("pinned H2D, 6.2 MB                   : %.3f ms (%.1f GB/s)\n", (t1 - t0) / reps,
                n / ((t1 - t0) / reps) / 1e6);
    t0 = now_ms();
    for (int i = 0; i < reps; ++i) {
        for (int k = 0; k < 6; ++k)
            CK(hipMemcpyAsync(static_cast<char*>(dev) + k * (n / 6), pin + k * (n / 6), n / 6, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
    }
    t1 = now_ms();
    std::printf("pinned H2D in 6 async chunks         : %.3f ms\n", (t1 - t0) / reps);
    for (int nt : {1, 4, 8, 16}) {
        t0 = now_ms();
        for (int i = 0; i < reps; ++i) {
            std::vector<std::thread> th;
            for (int t = 0; t < nt; ++t)
                th.emplace_back([&, t] {
                    const size_t a = n * t / nt, b = n * (t + 1) / nt;
                    std::memcpy(pin + a, bufs[i] + a, b - a);
                });
            for (auto& x : th) x.join();
        }
        t1 = now_ms();
        std::printf("memcpy pageable -> pinned, %2d threads : %.3f ms (incl. thread start)\n", nt, (t1 - t0) / reps);
    }
    char* hout = static_cast<char*>(std::malloc(n));
    std::memset(hout, 0, n);
    t0 = now_ms();
    for (int i = 0; i < reps; ++i) {
        CK(hipMemcpyAsync(pin, dev, n, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
    }
    t1 = now_ms();
    std::printf("pinned D2H, 6.2 MB                   : %.3f ms\n", (t1 - t0) / reps);
    t0 = now_ms();
    for (int i = 0; i < reps; ++i) {
        CK(hipMemcpyAsync(hout, dev, n, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
    }
    t1 = now_ms();
    std::printf("pageable D2H, 6.2 MB                 : %.3f ms\n", (t1 - t0) / reps);
    t0 = now_ms();
    for (int i = 0; i < reps; ++i) {
        CK(hipMemcpyAsync(dev, pin, 64, hipMemcpyHostToDevice, s));
    }
    CK(hipStreamSynchronize(s));
    t1 = now_ms();
    std::printf("hipMemcpyAsync call overhead (64 B)  : %.3f ms\n", (t1 - t0) / reps);
    return 0;
}
