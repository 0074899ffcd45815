// VALU issue-rate microbenchmark for the instructions the disparity kernels are built
// from (gfx950).  Each thread runs 8 independent accumulator chains of one instruction
// for ITERS iterations; 16 waves per CU (4 per SIMD).  Reports wave-instructions per
// cycle per SIMD relative to v_add_u32 (full rate = one wave64 instruction / 2 cycles),
// plus absolute ns per wave-instruction per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 valu_rate.hip -o valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define ITERS 2048

#define OP3(name, asmstr)                                                                 \
    __global__ __launch_bounds__(256) void k_##name(uint32_t* out, uint32_t a, uint32_t b) { \
        uint32_t x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4,     \
                 x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;                                   \
        uint32_t p = a ^ threadIdx.x, q = b + threadIdx.x;                                 \
        for (int i = 0; i < ITERS; ++i) {                                                 \
            asm volatile(asmstr : "+v"(x0) : "v"(p), "v"(q));                              \
            asm volatile(asmstr : "+v"(x1) : "v"(p), "v"(q));                              \
            asm volatile(asmstr : "+v"(x2) : "v"(p), "v"(q));                              \
            asm volatile(asmstr : "+v"(x3) : "v"(p), "v"(q));                              \
            asm volatile(asmstr : "+v"(x4) : "v"(p), "v"(q));                              \
            asm volatile(asmstr : "+v"(x5) : "v"(p), "v"(q));                              \
            asm volatile(asmstr : "+v"(x6) : "v"(p), "v"(q));                              \
            asm volatile(asmstr : "+v"(x7) : "v"(p), "v"(q));                              \
        }                                                                                 \
        out[blockIdx.x * 256 + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;      \
    }

OP3(add, "v_add_u32 %0, %1, %0")
OP3(sad_u8, "v_sad_u8 %0, %1, %2, %0")
OP3(sad_u16, "v_sad_u16 %0, %1, %2, %0")
OP3(sad_u32, "v_sad_u32 %0, %1, %2, %0")
OP3(msad_u8, "v_msad_u8 %0, %1, %2, %0")
OP3(dot4_u8, "v_dot4_u32_u8 %0, %1, %2, %0")
OP3(lshl_or, "v_lshl_or_b32 %0, %1, 3, %0")
OP3(min3, "v_min3_u32 %0, %1, %2, %0")
OP3(sub, "v_sub_u32 %0, %0, %1")
OP3(pk_add_u16, "v_pk_add_u16 %0, %1, %0")
OP3(pk_max_u16, "v_pk_max_u16 %0, %1, %0")
OP3(pk_sub_u16, "v_pk_sub_u16 %0, %0, %1")
OP3(perm, "v_perm_b32 %0, %1, %2, %0")
OP3(alignbyte, "v_alignbyte_b32 %0, %1, %2, %0")
OP3(bfe, "v_bfe_u32 %0, %1, %0, 8")
OP3(add3, "v_add3_u32 %0, %1, %2, %0")
OP3(mad_u24, "v_mad_u32_u24 %0, %1, %2, %0")
OP3(max_u32, "v_max_u32 %0, %1, %0")
OP3(cndmask, "v_cndmask_b32 %0, %1, %0, vcc")

OP3(sdwa_add, "v_add_u16_sdwa %0, %1, %0 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_1")
OP3(min_dpp, "v_min_u32_dpp %0, %1, %0 row_ror:1 row_mask:0xf bank_mask:0xf")
OP3(min_dpp_bm, "v_min_u32_dpp %0, %1, %0 row_mirror row_mask:0xf bank_mask:0x3")
OP3(min_e32, "v_min_u32 %0, %1, %0")
OP3(lshl_add, "v_lshl_add_u32 %0, %1, 16, %0")
OP3(pk_min_u16, "v_pk_min_u16 %0, %1, %0")
OP3(sad_hi_u8, "v_sad_hi_u8 %0, %1, %2, %0")
// mixed streams: does a VOP2 op hide behind VOP3 ops?
OP3(mix_sad_sub, "v_sad_u8 %0, %1, %2, %0\n v_sub_u32 %0, %0, %1")
OP3(mix_sad_sdwa, "v_sad_u8 %0, %1, %2, %0\n v_add_u16_sdwa %0, %1, %0 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:WORD_1")
OP3(mix_sad_min, "v_sad_u8 %0, %1, %2, %0\n v_min_u32 %0, %1, %0")
OP3(plswap, "v_mov_b32 %1, %0\n v_permlane16_swap_b32 %0, %1")

// quad SAD: 64-bit source, 32-bit reference, 64-bit (4 x u16) accumulator
__global__ __launch_bounds__(256) void k_qsad(uint32_t* out, uint32_t a, uint32_t b) {
    uint64_t x[8];
    for (int k = 0; k < 8; ++k) x[k] = threadIdx.x + k;
    uint64_t p = ((uint64_t)a << 32) ^ threadIdx.x;
    uint32_t q = b + threadIdx.x;
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) asm volatile("v_qsad_pk_u16_u8 %0, %1, %2, %0" : "+v"(x[k]) : "v"(p), "v"(q));
    }
    uint64_t s = 0;
    for (int k = 0; k < 8; ++k) s += x[k];
    out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)s;
}

__global__ __launch_bounds__(256) void k_mqsad(uint32_t* out, uint32_t a, uint32_t b) {
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    u4 x[4];
    for (int k = 0; k < 4; ++k) x[k] = (u4){threadIdx.x, 1u, 2u, (uint32_t)k};
    uint64_t p = ((uint64_t)a << 32) ^ threadIdx.x;
    uint32_t q = b + threadIdx.x;
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int k = 0; k < 4; ++k) asm volatile("v_mqsad_u32_u8 %0, %1, %2, %0" : "+v"(x[k]) : "v"(p), "v"(q));
#pragma unroll
        for (int k = 0; k < 4; ++k) asm volatile("v_mqsad_u32_u8 %0, %1, %2, %0" : "+v"(x[k]) : "v"(p), "v"(q));
    }
    uint32_t s = 0;
    for (int k = 0; k < 4; ++k) s += x[k].x + x[k].y + x[k].z + x[k].w;
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

typedef void (*kfn)(uint32_t*, uint32_t, uint32_t);

int main() {
    struct { const char* name; kfn f; } ks[] = {
        {"v_add_u32", k_add}, {"v_sad_u8", k_sad_u8}, {"v_sad_u16", k_sad_u16},
        {"v_sad_u32", k_sad_u32}, {"v_msad_u8", k_msad_u8}, {"v_dot4_u32_u8", k_dot4_u8},
        {"v_lshl_or_b32", k_lshl_or}, {"v_min3_u32", k_min3}, {"v_sub_u32", k_sub},
        {"v_pk_add_u16", k_pk_add_u16}, {"v_pk_max_u16", k_pk_max_u16}, {"v_pk_sub_u16", k_pk_sub_u16},
        {"v_perm_b32", k_perm}, {"v_alignbyte_b32", k_alignbyte}, {"v_bfe_u32", k_bfe},
        {"v_add3_u32", k_add3}, {"v_mad_u32_u24", k_mad_u24}, {"v_max_u32", k_max_u32},
        {"v_cndmask_b32", k_cndmask}, {"v_add_u16_sdwa", k_sdwa_add}, {"v_min_u32_dpp", k_min_dpp},
        {"v_min_u32_dpp bankmask", k_min_dpp_bm}, {"v_min_u32_e32", k_min_e32}, {"v_lshl_add_u32", k_lshl_add},
        {"v_pk_min_u16", k_pk_min_u16}, {"v_sad_hi_u8", k_sad_hi_u8}, {"mix sad+sub (x2)", k_mix_sad_sub},
        {"mix sad+sdwa (x2)", k_mix_sad_sdwa}, {"mix sad+min (x2)", k_mix_sad_min}, {"mov+permlane16swap(x2)", k_plswap}, {"v_qsad_pk_u16_u8", k_qsad}, {"v_mqsad_u32_u8", k_mqsad},
    };
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    const char* wps = getenv("WPS");
    const int blocks = ncu * (wps ? atoi(wps) : 4);   // WPS waves per SIMD (default 4)
    uint32_t* out;
    hipMalloc(&out, (size_t)blocks * 256 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    double add_ns = 0;
    printf("CUs %d, blocks %d, 8 chains x %d iters per thread\n", ncu, blocks, ITERS);
    for (auto& k : ks) {
        float best = 1e30f;
        for (int rep = 0; rep < 5; ++rep) {
            hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 0x01020304u, 0x05060708u);
            hipEventRecord(e0);
            hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 0x01020304u, 0x05060708u);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (ms < best) best = ms;
        }
        // wave-instructions per SIMD: blocks*4 waves * 8*ITERS / (ncu*4 SIMDs)
        const double winst = (double)blocks * 4 * 8 * ITERS / (ncu * 4.0);
        const double ns = best * 1e6 / winst;
        if (add_ns == 0) add_ns = ns;
        printf("%-20s %8.3f ms  %6.3f ns/wave-instr/SIMD  rel-cost %.2fx v_add\n", k.name, best, ns, ns / add_ns);
    }
    hipFree(out);
    return 0;
}
