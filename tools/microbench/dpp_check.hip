// Which lane a DPP control reads on this GPU (wave_shr/shl:1, row_shr/shl:1): prints, per
// control, the source lane seen by lanes 0..63 (-1: no source, the old value kept); then
// shl1(v) - shr1(v) of v = lane^2 as the compiler folds it (v_subrev_u32_dpp ... wave_shr:1
// bound_ctrl:1 — reads 0 on every lane on gfx950), expected 4*lane; then the same through a
// plain v_mov_b32_dpp kept unfolded (an asm barrier), which is right.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k(int* out, int salt) {
    const int l = threadIdx.x;
    out[0 * 64 + l] = __builtin_amdgcn_update_dpp(-1, l, 0x138, 0xF, 0xF, false);   // wave_shr:1
    out[1 * 64 + l] = __builtin_amdgcn_update_dpp(-1, l, 0x130, 0xF, 0xF, false);   // wave_shl:1
    out[2 * 64 + l] = __builtin_amdgcn_update_dpp(-1, l, 0x111, 0xF, 0xF, false);   // row_shr:1
    out[3 * 64 + l] = __builtin_amdgcn_update_dpp(-1, l, 0x101, 0xF, 0xF, false);   // row_shl:1
    const int v = l * l + salt;
    out[4 * 64 + l] = __builtin_amdgcn_update_dpp(0, v, 0x130, 0xF, 0xF, false) -
                      __builtin_amdgcn_update_dpp(0, v, 0x138, 0xF, 0xF, false);
    int a = __builtin_amdgcn_update_dpp(v, v, 0x130, 0xF, 0xF, false);
    int b = __builtin_amdgcn_update_dpp(v, v, 0x138, 0xF, 0xF, false);
    asm volatile("" : "+v"(a), "+v"(b));
    out[5 * 64 + l] = a - b;
}

int main() {
    int* d = nullptr;
    int h[6 * 64];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, 0);
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
    const char* names[6] = {"wave_shr:1", "wave_shl:1", "row_shr:1", "row_shl:1", "shl-shr", "unfolded"};
    for (int c = 0; c < 6; ++c) {
        std::printf("%-11s", names[c]);
        for (int l = 0; l < 64; ++l) std::printf(" %d", h[c * 64 + l]);
        std::printf("\n");
    }
    (void)hipFree(d);
    return 0;
}
