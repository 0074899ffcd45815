// lds_unaligned: does gfx950 serve 16-byte LDS loads at any byte offset (ds_read_b128 on an
// unaligned address, the operand fetch of the SSD MFMA kind), and at what cost?
//   1. correctness: every lane reads 16 bytes at byte offset (lane + shift) and the host
//      compares them with the source;
//   2. rate: a loop of dependent-free ds_read_b128 per lane at byte strides 16 (aligned), 1, 4
//      and 8, timed with clock64 (cycles per wave-instruction, one wave per SIMD).
// Build: hipcc --offload-arch=gfx950 -O3 lds_unaligned.hip -o lds_unaligned
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

struct __attribute__((packed, aligned(1))) U16 { uint32_t a, b, c, d; };

__global__ void k_check(const uint8_t* in, uint32_t* out, int sh) {
    __shared__ uint8_t lds[4096];
    for (int i = threadIdx.x; i < 4096; i += blockDim.x) lds[i] = in[i];
    __syncthreads();
    const U16 v = *reinterpret_cast<const U16*>(lds + threadIdx.x + sh);
    out[threadIdx.x * 4 + 0] = v.a;
    out[threadIdx.x * 4 + 1] = v.b;
    out[threadIdx.x * 4 + 2] = v.c;
    out[threadIdx.x * 4 + 3] = v.d;
}

// lane l reads at byte (l * stride + it * 64) & 2047, 64 iterations, xor-folded
__global__ void k_rate(const uint8_t* in, uint32_t* out, long long* cyc, int stride) {
    __shared__ uint8_t lds[4096];
    for (int i = threadIdx.x; i < 4096; i += blockDim.x) lds[i] = in[i];
    __syncthreads();
    uint32_t acc = 0;
    const long long t0 = clock64();
#pragma unroll 16
    for (int it = 0; it < 256; ++it) {
        const int off = (threadIdx.x * stride + it * 64) & 2047;
        const U16 v = *reinterpret_cast<const U16*>(lds + off);
        acc ^= v.a ^ v.b ^ v.c ^ v.d;
    }
    const long long t1 = clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// throughput: 1024 blocks x 256 threads, lane l of the block reads 16 bytes at
// (base + l * stride) & 2047 for 256 iterations (base advances 64 B); kernel time by events
__global__ void k_tput(const uint8_t* in, uint32_t* out, int stride, int shift) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[4096];
    for (int i = threadIdx.x; i < 4096; i += blockDim.x) lds[i] = in[i];
    __syncthreads();
    uint32_t acc = 0;
#pragma unroll 8
    for (int it = 0; it < 256; ++it) {
        const int off = ((threadIdx.x & 63) * stride + it * 64 + shift) & 2047;
        const U16 v = *reinterpret_cast<const U16*>(lds + off);
        acc += v.a ^ v.b ^ v.c ^ v.d;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
    uint8_t h[4096];
    for (int i = 0; i < 4096; ++i) h[i] = (uint8_t)(i * 37 + (i >> 8) * 11 + 5);
    uint8_t* d_in;
    uint32_t* d_out;
    long long* d_cyc;
    hipMalloc(&d_in, 4096);
    hipMalloc(&d_out, 1 << 20);
    hipMalloc(&d_cyc, 1024 * 8);
    hipMemcpy(d_in, h, 4096, hipMemcpyHostToDevice);
    int bad = 0;
    for (int sh = 0; sh < 17; ++sh) {
        hipLaunchKernelGGL(k_check, dim3(1), dim3(256), 0, 0, d_in, d_out, sh);
        uint32_t o[1024];
        hipMemcpy(o, d_out, sizeof(o), hipMemcpyDeviceToHost);
        for (int l = 0; l < 256; ++l)
            if (memcmp(&o[l * 4], h + l + sh, 16) != 0) ++bad;
    }
    printf("correctness: %s (%d lanes wrong over 17 shifts x 256 lanes)\n", bad ? "FAIL" : "ok", bad);
    const int strides[] = {16, 1, 4, 8, 17};
    for (int s : strides) {
        hipLaunchKernelGGL(k_rate, dim3(256), dim3(64), 0, 0, d_in, d_out, d_cyc, s);
        hipLaunchKernelGGL(k_rate, dim3(256), dim3(64), 0, 0, d_in, d_out, d_cyc, s);
        long long c[256];
        hipMemcpy(c, d_cyc, sizeof(c), hipMemcpyDeviceToHost);
        double m = 0;
        for (int i = 0; i < 256; ++i) m += (double)c[i];
        printf("stride %2d B: %.2f cycles per ds_read_b128 (one wave per CU)\n", s, m / 256 / 256);
    }
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    uint32_t* d_big;
    hipMalloc(&d_big, 1024 * 256 * 4);
    const int cases[][2] = {{16, 0}, {16, 4}, {16, 1}, {4, 0}, {1, 0}, {0, 0}, {32, 0}};
    for (auto& cs : cases) {
        float best = 1e9f;
        for (int rep = 0; rep < 5; ++rep) {
            hipEventRecord(e0, 0);
            hipLaunchKernelGGL(k_tput, dim3(1024), dim3(256), 0, 0, d_in, d_big, cs[0], cs[1]);
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            if (ms < best) best = ms;
        }
        // 1024 blocks x 4 waves x 256 ds_read_b128 over 256 CUs at ~2.4 GHz
        const double per_cu = 1024.0 * 4 * 256 / 256;
        printf("throughput stride %2d shift %d: %.3f ms, %.2f cycles per ds_read_b128 per CU\n", cs[0], cs[1], best,
               best * 1e-3 * 2.4e9 / per_cu);
    }
    hipDeviceSynchronize();
    return bad ? 1 : 0;
}
