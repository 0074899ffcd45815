// mfma_i8_layout: pins the operand / result maps of v_mfma_i32_32x32x32_i8 that the SSD MFMA
// kind (sv_ssd_mfma.hip) relies on, with exact integer data and an asymmetric operand:
//   A: lane l holds 16 int8 of row (l & 31), "k slots" (l >> 5, byte j);
//   B: lane l holds 16 int8 of column (l & 31), "k slots" (l >> 5, byte j);
//   D: lane l holds column (l & 31), rows (reg & 3) + 8 (reg >> 2) + 4 (l >> 5), reg 0..15;
//   D[row][col] = sum over (h, j) of A(row, h, j) * B(col, h, j)   (+ C in).
// Only the pairing of A's and B's slots matters to a dot product, not the hardware's k order.
// Also times back-to-back MFMAs on one accumulator chain and on 10 independent ones.
// Build: hipcc --offload-arch=gfx950 -O3 mfma_i8_layout.hip -o mfma_i8_layout
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

__global__ void k_one(const int8_t* A, const int8_t* B, const int* C, int* D) {
    const int l = threadIdx.x;
    v4i a, b;
    int8_t* pa = reinterpret_cast<int8_t*>(&a);
    int8_t* pb = reinterpret_cast<int8_t*>(&b);
    for (int j = 0; j < 16; ++j) {
        pa[j] = A[(l & 31) * 32 + (l >> 5) * 16 + j];   // A[row][slot], slot = 16 h + j
        pb[j] = B[(l & 31) * 32 + (l >> 5) * 16 + j];   // B[col][slot]
    }
    v16i c;
    for (int r = 0; r < 16; ++r) c[r] = C[l * 16 + r];
    c = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c, 0, 0, 0);
    for (int r = 0; r < 16; ++r) D[l * 16 + r] = c[r];
}

template <int N>
__global__ void k_rate(const v4i* in, int* out, long long* cyc, int iters) {
    const int l = threadIdx.x;
    v4i a = in[l], b = in[64 + l];
    v16i c[N];
    for (int n = 0; n < N; ++n)
        for (int r = 0; r < 16; ++r) c[n][r] = r + n;
    const long long t0 = clock64();
    for (int it = 0; it < iters; ++it)
#pragma unroll
        for (int n = 0; n < N; ++n) c[n] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c[n], 0, 0, 0);
    const long long t1 = clock64();
    int s = 0;
    for (int n = 0; n < N; ++n)
        for (int r = 0; r < 16; ++r) s ^= c[n][r];
    out[blockIdx.x * 64 + l] = s;
    if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    int8_t hA[32 * 32], hB[32 * 32];
    int hC[64 * 16], hD[64 * 16];
    srand(7);
    for (int i = 0; i < 1024; ++i) {
        hA[i] = (int8_t)(rand() % 256 - 128);
        hB[i] = (int8_t)(rand() % 256 - 128);
    }
    for (int i = 0; i < 1024; ++i) hC[i] = rand() % 1000 - 500;
    int8_t *dA, *dB;
    int *dC, *dD;
    hipMalloc(&dA, 1024);
    hipMalloc(&dB, 1024);
    hipMalloc(&dC, 4096);
    hipMalloc(&dD, 4096);
    hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice);
    hipMemcpy(dB, hB, 1024, hipMemcpyHostToDevice);
    hipMemcpy(dC, hC, 4096, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_one, dim3(1), dim3(64), 0, 0, dA, dB, dC, dD);
    hipMemcpy(hD, dD, 4096, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; ++l)
        for (int r = 0; r < 16; ++r) {
            const int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), col = l & 31;
            long long s = hC[l * 16 + r];
            for (int k = 0; k < 32; ++k) s += (long long)hA[row * 32 + k] * hB[col * 32 + k];
            if (s != hD[l * 16 + r]) ++bad;
        }
    printf("v_mfma_i32_32x32x32_i8 maps: %s (%d of 1024 results differ)\n", bad ? "FAIL" : "ok", bad);
    v4i* din;
    int* dout;
    long long* dcyc;
    hipMalloc(&din, 128 * 16);
    hipMemset(din, 1, 128 * 16);
    hipMalloc(&dout, 1024 * 64 * 4);
    hipMalloc(&dcyc, 1024 * 8);
    long long hc[1024];
    for (int pass = 0; pass < 2; ++pass) {
        hipLaunchKernelGGL(k_rate<1>, dim3(1024), dim3(64), 0, 0, din, dout, dcyc, 256);
        hipMemcpy(hc, dcyc, sizeof(hc), hipMemcpyDeviceToHost);
        double m = 0;
        for (int i = 0; i < 1024; ++i) m += hc[i];
        if (pass) printf("1 chain: %.1f cycles per MFMA (one wave per SIMD)\n", m / 1024 / 256);
        hipLaunchKernelGGL(k_rate<10>, dim3(1024), dim3(64), 0, 0, din, dout, dcyc, 64);
        hipMemcpy(hc, dcyc, sizeof(hc), hipMemcpyDeviceToHost);
        m = 0;
        for (int i = 0; i < 1024; ++i) m += hc[i];
        if (pass) printf("10 chains: %.1f cycles per MFMA (one wave per SIMD)\n", m / 1024 / 640);
    }
    return bad ? 1 : 0;
}
