// sv_match.hip — the disparity cost-volume + winner-take-all kernel for gfx950.
//
// Replaces the reference's `cv2.StereoSGBM_create(...).compute(gray_left, gray_right)`
// (depth_map.py:894-909, fused_depth_map.py:988-1004) with the build-defined SAD / SSD /
// HOG winner-take-all engine specified in DESIGN.md ("Semantics").  Output: int16 = d*16,
// invalid = (minD-1)*16 outside the matched band [X0, X1).
//
// Work decomposition (one wave = one output row y, 256 output columns):
//   * the wave is split into G = 64/LPG groups of LPG lanes; group g walks the segment
//     [xs, xs+S) of S = 4*LPG columns left to right;
//   * lane l of a group owns the DPL consecutive disparities d = minD + l*DPL + k, so the
//     LPG*DPL candidates of one pixel sit across one group, and the argmin is an in-lane
//     min3 chain over (cost << dbits | d) keys + a DPP row reduction (first-min tie-break);
//   * image data is staged ONCE per wave in LDS as "column packs": the win bytes of one
//     column, rows y-r..y+r, packed 4 per dword (zero padded).  One v_sad_u8 then sums 4
//     vertical taps, so a column's vertical window costs ceil(win/4) VALU ops;
//   * the horizontal window is a running sum along x: per step the group adds the column
//     entering the window and subtracts the column leaving it;
//   * the right-image column a lane needs for disparity k at step t is the column it
//     loaded for k-1 at step t-1, so each lane keeps a DPL-deep register ring and loads
//     ONE new right pack per step (plus one for the leaving column) — LDS traffic is
//     2 R + 2 L reads per step per lane for DPL cost cells;
//   * right packs are stored with a 1-in-8 slot gap (rphys) so the 16 lanes of a group,
//     whose columns are DPL apart, hit distinct LDS banks on ds_read_b128.
// SSD uses the same skeleton with v_dot4_u32_u8: sum (L-R)^2 = sum L^2 + sum R^2 - 2 sum L*R
// (squares precomputed per pack).  HOG reads 9-bin window histograms (u16) as packs and
// compares them with v_sad_u16; it has no running window (r = 0 in the skeleton).
#include "sv_internal.h"

namespace sv {
namespace {

constexpr int WAVE_COLS = 256;
constexpr int ROWS_PER_BLOCK = 4;

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return min(max(v, lo), hi); }
__device__ __forceinline__ int rphys(int i) { return i + (i >> 3); }

template <int COST> struct PackQ { static constexpr int Q = (COST == COST_SAD) ? 1 : 2; };

template <int Q>
__device__ __forceinline__ void load_pack(const uint4* p, uint4 (&v)[Q]) {
#pragma unroll
    for (int q = 0; q < Q; ++q) v[q] = p[q];
}

// Per-cell column cost added to `acc`.
template <int COST, int NDW, int Q>
__device__ __forceinline__ uint32_t vcol(const uint4 (&l)[Q], const uint4 (&r)[Q], uint32_t acc) {
    if constexpr (COST == COST_SAD) {
        acc = __builtin_amdgcn_sad_u8(l[0].x, r[0].x, acc);
        if constexpr (NDW > 1) acc = __builtin_amdgcn_sad_u8(l[0].y, r[0].y, acc);
        if constexpr (NDW > 2) acc = __builtin_amdgcn_sad_u8(l[0].z, r[0].z, acc);
        if constexpr (NDW > 3) acc = __builtin_amdgcn_sad_u8(l[0].w, r[0].w, acc);
        return acc;
    } else if constexpr (COST == COST_SSD) {
        uint32_t dot = __builtin_amdgcn_udot4(l[0].x, r[0].x, 0u, false);
        if constexpr (NDW > 1) dot = __builtin_amdgcn_udot4(l[0].y, r[0].y, dot, false);
        if constexpr (NDW > 2) dot = __builtin_amdgcn_udot4(l[0].z, r[0].z, dot, false);
        if constexpr (NDW > 3) dot = __builtin_amdgcn_udot4(l[0].w, r[0].w, dot, false);
        return acc + (l[1].x + r[1].x) - (dot << 1);
    } else {  // HOG: 9 u16 bins in 5 dwords
        acc = __builtin_amdgcn_sad_u16(l[0].x, r[0].x, acc);
        acc = __builtin_amdgcn_sad_u16(l[0].y, r[0].y, acc);
        acc = __builtin_amdgcn_sad_u16(l[0].z, r[0].z, acc);
        acc = __builtin_amdgcn_sad_u16(l[0].w, r[0].w, acc);
        acc = __builtin_amdgcn_sad_u16(l[1].x, r[1].x, acc);
        return acc;
    }
}

// Build one column pack for logical column c around row y (replicate-clamped).
template <int COST, int Q>
__device__ __forceinline__ void build_pack(const MatchParams& a, const uint8_t* img,
                                           const uint16_t* hist, int c, int y, uint4* dst) {
    const int cc = clampi(c, 0, a.W - 1);
    if constexpr (COST == COST_HOG) {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(hist + ((size_t)y * a.W + cc) * 10);
        dst[0] = make_uint4(src[0], src[1], src[2], src[3]);
        dst[1] = make_uint4(src[4], 0u, 0u, 0u);
    } else {
        uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0, sq = 0;
        for (int j = 0; j < a.win; ++j) {
            const int yy = clampi(y - a.r + j, 0, a.H - 1);
            const uint32_t v = img[(size_t)yy * a.pitch + cc];
            sq += v * v;
            const uint32_t sh = v << (8 * (j & 3));
            const int q = j >> 2;
            w0 |= q == 0 ? sh : 0u;
            w1 |= q == 1 ? sh : 0u;
            w2 |= q == 2 ? sh : 0u;
            w3 |= q == 3 ? sh : 0u;
        }
        dst[0] = make_uint4(w0, w1, w2, w3);
        if constexpr (Q > 1) dst[1] = make_uint4(sq, 0u, 0u, 0u);
    }
}

// min over the LPG lanes of a group; the result is exact in the group's LAST lane
// (in every lane for LPG = 16).
__device__ __forceinline__ uint32_t group_min(uint32_t v, int lpg) {
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, (int)v, 0x121, 0xF, 0xF, false));  // row_ror:1
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, (int)v, 0x122, 0xF, 0xF, false));  // row_ror:2
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, (int)v, 0x124, 0xF, 0xF, false));  // row_ror:4
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0u, (int)v, 0x128, 0xF, 0xF, false));  // row_ror:8
    if (lpg >= 32)  // row_bcast:15 into rows 1 and 3
        v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x142, 0xA, 0xF, false));
    if (lpg == 64)  // row_bcast:31 into rows 2 and 3
        v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v, 0x143, 0xC, 0xF, false));
    return v;
}

template <int COST, int NDW, int DPL>
__global__ __launch_bounds__(256) void k_match(MatchParams a) {
    constexpr int Q = PackQ<COST>::Q;
    extern __shared__ __attribute__((aligned(16))) uint4 smem[];
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const int LPG = a.lpg;
    const int S = 4 * LPG;                 // segment width per group
    const int r = a.r;
    const int W2 = 2 * r + 1;
    const int NL = WAVE_COLS + 4 * r + DPL;
    const int NRlog = WAVE_COLS + 4 * r + LPG * DPL + DPL;
    const int NRphys = NRlog + (NRlog >> 3) + 1;
    uint4* Lp = smem + (size_t)wid * (NL + NRphys) * Q;
    uint4* Rp = Lp + (size_t)NL * Q;

    const int y = a.row0 + (int)blockIdx.y * ROWS_PER_BLOCK + wid;
    const int yc = min(y, a.row1 - 1);
    const int xw = a.X0 + (int)blockIdx.x * WAVE_COLS;
    const int cL0 = xw - 3 * r - 1;
    const int cR0 = cL0 - a.minD - (LPG * DPL - 1);

    for (int i = lane; i < NL; i += 64) build_pack<COST, Q>(a, a.L, a.HL, cL0 + i, yc, Lp + (size_t)i * Q);
    for (int i = lane; i < NRlog; i += 64)
        build_pack<COST, Q>(a, a.R, a.HR, cR0 + i, yc, Rp + (size_t)rphys(i) * Q);

    if (blockIdx.x == 0 && y < a.row1) {  // columns outside the matched band are invalid
        const int16_t inv = (int16_t)((a.minD - 1) * 16);
        int16_t* orow = a.out + (size_t)y * a.opitch;
        for (int x = lane; x < a.X0; x += 64) orow[x] = inv;
        for (int x = a.X1 + lane; x < a.W; x += 64) orow[x] = inv;
    }
    __syncthreads();
    if (y >= a.row1) return;

    const int g = lane >> a.lpg_log2;
    const int l = lane & (LPG - 1);
    const int xs = xw + g * S;
    const int iL0 = g * S + 2 * r + 1;
    const int iR0 = g * S + 2 * r + (LPG - l) * DPL;
    const int T = (S + 2 * r + DPL - 1) / DPL * DPL;
    const uint32_t dmask = (1u << a.dbits) - 1u;
    const int dbits = a.dbits;
    const bool emitter = (l == LPG - 1);
    int16_t* orow = a.out + (size_t)y * a.opitch;

    uint32_t mk[DPL];
#pragma unroll
    for (int k = 0; k < DPL; ++k) {
        const int idx = l * DPL + k;
        mk[k] = idx < a.D ? (uint32_t)idx : 0xFFFFFFFFu;
    }
    uint4 rn[DPL][Q];
    uint4 ro[DPL][Q];
#pragma unroll
    for (int j = 1; j < DPL; ++j) {
        load_pack<Q>(Rp + (size_t)rphys(iR0 - j) * Q, rn[DPL - j]);
        if constexpr (COST != COST_HOG) load_pack<Q>(Rp + (size_t)rphys(iR0 - j - W2) * Q, ro[DPL - j]);
    }
    uint32_t h[DPL];
#pragma unroll
    for (int k = 0; k < DPL; ++k) h[k] = 0u;

    for (int t0 = 0; t0 < T; t0 += DPL) {
#pragma unroll
        for (int u = 0; u < DPL; ++u) {
            const int t = t0 + u;
            load_pack<Q>(Rp + (size_t)rphys(iR0 + t) * Q, rn[u]);
            uint4 ln[Q];
            load_pack<Q>(Lp + (size_t)(iL0 + t) * Q, ln);
            if constexpr (COST == COST_HOG) {
#pragma unroll
                for (int k = 0; k < DPL; ++k) h[k] = vcol<COST, NDW, Q>(ln, rn[(u - k + DPL) % DPL], 0u);
            } else {
                load_pack<Q>(Rp + (size_t)rphys(iR0 + t - W2) * Q, ro[u]);
#pragma unroll
                for (int k = 0; k < DPL; ++k) h[k] = vcol<COST, NDW, Q>(ln, rn[(u - k + DPL) % DPL], h[k]);
                if (t >= W2) {
                    uint4 lo[Q];
                    load_pack<Q>(Lp + (size_t)(iL0 + t - W2) * Q, lo);
#pragma unroll
                    for (int k = 0; k < DPL; ++k) h[k] -= vcol<COST, NDW, Q>(lo, ro[(u - k + DPL) % DPL], 0u);
                }
            }
            if (t >= 2 * r) {
                uint32_t best = 0xFFFFFFFFu;
#pragma unroll
                for (int k = 0; k < DPL; ++k) best = min(best, (h[k] << dbits) | mk[k]);
                best = group_min(best, LPG);
                const int e = t - 2 * r;
                const int x = xs + e;
                if (emitter && e < S && x < a.X1)
                    orow[x] = (int16_t)(((int)(best & dmask) + a.minD) * 16);
            }
        }
    }
}

__global__ void k_fill_i16(int16_t* out, int opitch, int H, int W, int16_t v) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    if (x < W && y < H) out[(size_t)y * opitch + x] = v;
}

template <int COST, int NDW, int DPL>
int launch_one(const MatchParams& a, size_t lds, hipStream_t s) {
    auto fn = k_match<COST, NDW, DPL>;
    if (lds > 65536) {  // opt in to > 64 KiB of dynamic LDS (per device, cheap host call)
        hipError_t e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return (int)e;
    }
    dim3 grid((a.X1 - a.X0 + WAVE_COLS - 1) / WAVE_COLS, (a.row1 - a.row0 + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK);
    hipLaunchKernelGGL(fn, grid, dim3(256), lds, s, a);
    return (int)hipGetLastError();
}

template <int COST, int NDW>
int launch_dpl(const MatchParams& a, const MatchPlan& p, size_t lds, hipStream_t s) {
    switch (p.dpl) {
        case 4: return launch_one<COST, NDW, 4>(a, lds, s);
        case 6: return launch_one<COST, NDW, 6>(a, lds, s);
        case 8: return launch_one<COST, NDW, 8>(a, lds, s);
    }
    return (int)hipErrorInvalidValue;
}

template <int COST>
int launch_ndw(const MatchParams& a, const MatchPlan& p, size_t lds, hipStream_t s) {
    if constexpr (COST == COST_HOG) {
        return launch_dpl<COST, 5>(a, p, lds, s);
    } else {
        switch (p.ndw) {
            case 1: return launch_dpl<COST, 1>(a, p, lds, s);
            case 2: return launch_dpl<COST, 2>(a, p, lds, s);
            case 3: return launch_dpl<COST, 3>(a, p, lds, s);
            case 4: return launch_dpl<COST, 4>(a, p, lds, s);
        }
        return (int)hipErrorInvalidValue;
    }
}

}  // namespace

int plan_match(int num_disp, int win, int cost, MatchPlan* plan) {
    static const int menu[][2] = {{4, 16}, {6, 16}, {8, 16}, {6, 32}, {8, 32}, {6, 64}, {8, 64}};
    if (num_disp <= 0 || win < 1 || (win & 1) == 0 || win > 15) return -22;
    if (cost != COST_SAD && cost != COST_SSD && cost != COST_HOG) return -22;
    int i = 0;
    for (; i < 7; ++i)
        if (menu[i][0] * menu[i][1] >= num_disp) break;
    if (i == 7) return -22;
    plan->dpl = menu[i][0];
    plan->lpg = menu[i][1];
    plan->ndw = cost == COST_HOG ? 5 : (win + 3) / 4;
    int n = plan->dpl * plan->lpg - 1, bits = 0;
    while (n > 0) { ++bits; n >>= 1; }
    plan->dbits = bits < 1 ? 1 : bits;
    uint64_t cmax = cost == COST_SAD ? (uint64_t)win * win * 255
                  : cost == COST_SSD ? (uint64_t)win * win * 255 * 255
                                     : (uint64_t)9 * win * win * 255;
    if ((cmax << plan->dbits) >= (1ull << 32)) return -34;  // ERANGE: key would overflow
    return 0;
}

size_t match_lds_bytes(const MatchPlan& p, int r, int cost) {
    const int Q = cost == COST_SAD ? 1 : 2;
    const int NL = WAVE_COLS + 4 * r + p.dpl;
    const int NRlog = WAVE_COLS + 4 * r + p.lpg * p.dpl + p.dpl;
    const int NRphys = NRlog + (NRlog >> 3) + 1;
    return (size_t)ROWS_PER_BLOCK * (NL + NRphys) * Q * 16;
}

int launch_fill_i16(int16_t* out, int opitch, int H, int W, int16_t v, hipStream_t s) {
    if (H <= 0 || W <= 0) return 0;
    hipLaunchKernelGGL(k_fill_i16, dim3((W + 255) / 256, H), dim3(256), 0, s, out, opitch, H, W, v);
    return (int)hipGetLastError();
}

int launch_match(const MatchParams& a, const MatchPlan& p, int cost, hipStream_t s) {
    if (a.row1 <= a.row0) return 0;
    if (a.X1 <= a.X0)
        return launch_fill_i16(a.out + (size_t)a.row0 * a.opitch, a.opitch, a.row1 - a.row0, a.W,
                               (int16_t)((a.minD - 1) * 16), s);
    const size_t lds = match_lds_bytes(p, a.r, cost);
    if (lds > 160 * 1024) return (int)hipErrorInvalidValue;
    switch (cost) {
        case COST_SAD: return launch_ndw<COST_SAD>(a, p, lds, s);
        case COST_SSD: return launch_ndw<COST_SSD>(a, p, lds, s);
        case COST_HOG: return launch_ndw<COST_HOG>(a, p, lds, s);
    }
    return (int)hipErrorInvalidValue;
}

}  // namespace sv
