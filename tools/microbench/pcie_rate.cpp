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
    // the host path's median download: 4.1 MB of int16 in 8 pieces, an event after each
    const size_t m = 1920 * 1080 * 2;
    hipEvent_t ev[8];
    for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    auto pieces = [&](char* host, const char* label, int np = 8) {
        double a = now_ms();
        for (int i = 0; i < reps; ++i) {
            for (int q = 0; q < np; ++q) {
                CK(hipMemcpyAsync(host + m * q / np, static_cast<char*>(dev) + m * q / np, m / np,
                                  hipMemcpyDeviceToHost, s));
                CK(hipEventRecord(ev[q], s));
            }
            CK(hipStreamSynchronize(s));
        }
        double b = now_ms();
        std::printf("%-37s: %.3f ms (%.1f GB/s) [%d pieces]\n", label, (b - a) / reps,
                    m / ((b - a) / reps * 1e-3) / 1e9, np);
    };
    pieces(pin, "pinned D2H 4.1 MB, 8 pieces + events");
    char* pin_nc;
    CK(hipHostMalloc(reinterpret_cast<void**>(&pin_nc), n, hipHostMallocNonCoherent));
    pieces(pin_nc, "non-coherent pinned D2H, 8 pieces");
    char* pin_c;
    CK(hipHostMalloc(reinterpret_cast<void**>(&pin_c), n, hipHostMallocCoherent));
    pieces(pin_c, "coherent pinned D2H, 8 pieces");
    char* reg = static_cast<char*>(std::malloc(n));
    std::memset(reg, 0, n);
    CK(hipHostRegister(reg, n, hipHostRegisterPortable));
    pieces(reg, "registered malloc D2H, 8 pieces");
    t0 = now_ms();
    for (int i = 0; i < reps; ++i) {
        CK(hipMemcpyAsync(pin_nc, dev, m, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
    }
    t1 = now_ms();
    std::printf("non-coherent pinned D2H 4.1 MB, 1 piece: %.3f ms\n", (t1 - t0) / reps);
    for (int np : {1, 2, 4, 8}) pieces(pin, "default pinned D2H 4.1 MB (again)", np);
    for (int np : {1, 2, 4, 8}) pieces(pin_nc, "non-coherent pinned D2H 4.1 MB", np);
    // the registered-output path: 22.8 MB (depth f32, disparity f32, colormap BGR) in 8 x 3 pieces
    {
        const size_t nb[3] = {(size_t)1920 * 1080 * 4, (size_t)1920 * 1080 * 4, (size_t)1920 * 1080 * 3};
        void* dv[3];
        char* hv[3];
        for (int k = 0; k < 3; ++k) {
            CK(hipMalloc(&dv[k], nb[k]));
            hv[k] = static_cast<char*>(std::malloc(nb[k]));
            std::memset(hv[k], 0, nb[k]);
            CK(hipHostRegister(hv[k], nb[k], hipHostRegisterPortable));
        }
        for (int np : {1, 8}) {
            double a = now_ms();
            for (int i = 0; i < reps; ++i) {
                for (int q = 0; q < np; ++q)
                    for (int k = 0; k < 3; ++k)
                        CK(hipMemcpyAsync(hv[k] + nb[k] * q / np, static_cast<char*>(dv[k]) + nb[k] * q / np,
                                          nb[k] / np, hipMemcpyDeviceToHost, s));
                CK(hipStreamSynchronize(s));
            }
            double b = now_ms();
            std::printf("registered outputs D2H 22.8 MB, %d x 3 pieces: %.3f ms (%.1f GB/s)\n", np, (b - a) / reps,
                        (nb[0] + nb[1] + nb[2]) / ((b - a) / reps * 1e-3) / 1e9);
        }
    }
    return 0;
}
