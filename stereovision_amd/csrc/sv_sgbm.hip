// sv_sgbm.hip — SGBM-3WAY disparity mode on gfx950.
//
// The reference's disparity call is cv2.StereoSGBM(..., MODE_SGBM_3WAY).compute
// (depth_map.py:894-909, fused_depth_map.py:988-1004).  Semantics: oracle/sv_sgbm_oracle.py
// (OpenCV's published algorithm, one stripe, int32 aggregated costs; parity with OpenCV
// itself unpinned).  Pipeline, one frame:
//
//  k_sgbm_hsum_tiled  per (row, 256-column slab): x-Sobel prefilter (clip to +-cap) and raw
//                 channel with their Birchfield-Tomasi half-pixel intervals as 16-byte LDS
//                 records; pixel cost BT(sobel) + BT(raw) >> 2 in packed u16 ops for every
//                 (x, d) of the band, summed over the window columns (running sum with a
//                 register ring, band-clamped) -> hsum u16 [H][Wb][Dp]
//  k_sgbm_vsum    window rows (running sum down the column, row-clamped) -> C u16 [H][Wb][Dp]
//  k_sgbm_hpath   left->right and right->left paths: 16 lanes per row, 4 rows per wave; lane
//                 j owns DPL consecutive disparities; per step d+-1 come from row_shr/shl DPP
//                 and the path minimum from a row_ror butterfly; the next PF steps' costs
//                 are in flight in a register ring -> L_lr, L_rl (int16 when every value
//                 fits, else int32)
//  k_sgbm_vpath   top->bottom path, 32 lanes per band column (two DPP rows joined by
//                 v_permlane16_swap) walking down the rows with the same prefetch ring ->
//                 L_tb; on a second stream, concurrent with k_sgbm_hpath
//  k_sgbm_wta     S = L_lr + L_rl + L_tb per pixel, argmin over ((S + 2^20) << 9 | d) keys,
//                 uniqueness from the smallest non-neighbour S, S[b-1] / S[b+1] through LDS
//                 for the sub-pixel parabola, one 8-byte record per pixel (full occupancy)
//  k_sgbm_lrcheck per row: the right-view disparity by 64-bit LDS atomicMin over
//                 (minS, rightmost x) keys, the +-disp12MaxDiff consistency test, band
//                 borders -> int16 x16 output
//  k_cc_*         filterSpeckles as union-find over 4-connected |d1 - d2| <= maxDiff edges:
//                 32x32 tiles in LDS first (with local component sizes), then the
//                 tile-border edges in the global forest (atomicMin linking; edges between
//                 two trees that already hold a component > maxSpeckleSize are skipped), sizes
//                 summed per local root
//
// The DP kernels are latency-bound chains (W or H dependent steps); the sums are HBM-bound.
#include "sv_internal.h"

#include <algorithm>

#include <cstdlib>

namespace sv {
namespace {

constexpr int kInf = 0x3FFFFFFF;

__device__ __forceinline__ int dpp_shr1(int v, int old) {   // lane j <- lane j-1 (row of 16)
    return __builtin_amdgcn_update_dpp(old, v, 0x111, 0xF, 0xF, false);
}
__device__ __forceinline__ int dpp_shl1(int v, int old) {   // lane j <- lane j+1
    return __builtin_amdgcn_update_dpp(old, v, 0x101, 0xF, 0xF, false);
}
template <int ROR>
__device__ __forceinline__ int dpp_ror(int v) {
    return __builtin_amdgcn_update_dpp(v, v, 0x120 + ROR, 0xF, 0xF, false);
}
__device__ __forceinline__ int row_min(int v) {             // min over the 16-lane row, all lanes
    v = min(v, dpp_ror<8>(v));
    v = min(v, dpp_ror<4>(v));
    v = min(v, dpp_ror<2>(v));
    v = min(v, dpp_ror<1>(v));
    return v;
}
__device__ __forceinline__ uint32_t row_min_u(uint32_t v) {
    v = min(v, (uint32_t)dpp_ror<8>((int)v));
    v = min(v, (uint32_t)dpp_ror<4>((int)v));
    v = min(v, (uint32_t)dpp_ror<2>((int)v));
    v = min(v, (uint32_t)dpp_ror<1>((int)v));
    return v;
}
__device__ __forceinline__ int row_max(int v) {
    v = max(v, dpp_ror<8>(v));
    v = max(v, dpp_ror<4>(v));
    v = max(v, dpp_ror<2>(v));
    v = max(v, dpp_ror<1>(v));
    return v;
}

// -------------------------------------------------------------------------------------
// pixel cost + horizontal window sums
// -------------------------------------------------------------------------------------
// Pixel cost + window columns: one workgroup per (row, 256-column slab of the band).  Per image column a 16-byte record {value, BT lo, BT hi} with the two channels
// (x-Sobel, raw) as the u16 halves of each dword, so the pixel cost of a cell is 7 packed
// u16 ops (saturating subtracts give the max(0, .) of Birchfield-Tomasi for free) + 2; the
// window's leaving column comes from a register ring (one pixel cost per cell, not two).
constexpr int kHX = 256;          // band columns per workgroup
constexpr int kMaxR = 7;          // blockSize <= 15 (check_match)
typedef unsigned short us2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ us2 as_us2(uint32_t v) { return __builtin_bit_cast(us2, v); }
__device__ __forceinline__ uint32_t as_u32(us2 v) { return __builtin_bit_cast(uint32_t, v); }

// {value, lo, hi} of image column x of row y, both channels: x-Sobel clipped to +-cap (+cap)
// and the raw value, columns 0 and W-1 holding cap in both (OpenCV's tab[0]), with the
// Birchfield-Tomasi half-pixel interval [min, max] of (c, (c+left)/2, (c+right)/2)
__device__ __forceinline__ uint4 bt_record(const SgbmArgs& a, const uint8_t* img, int y, int x) {
    const int W = a.W;
    const int ym = y > 0 ? y - 1 : y, yp = y < a.H - 1 ? y + 1 : y;
    const uint8_t* r0 = img + (size_t)y * a.pitch;
    const uint8_t* rm = img + (size_t)ym * a.pitch;
    const uint8_t* rp = img + (size_t)yp * a.pitch;
    int pf[3], raw[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {   // columns x-1, x, x+1
        const int xx = x - 1 + k;
        int p = a.cap, w = a.cap;
        if (xx > 0 && xx < W - 1) {
            const int s = (r0[xx + 1] - r0[xx - 1]) * 2 + rm[xx + 1] - rm[xx - 1] + rp[xx + 1] - rp[xx - 1];
            p = min(max(s, -a.cap), a.cap) + a.cap;
            w = r0[xx];
        }
        pf[k] = p;
        raw[k] = w;
    }
    auto bt = [&](const int (&v)[3], int& lo, int& hi) {
        const int c = v[1];
        const int l = x > 0 ? (c + v[0]) >> 1 : c;
        const int r = x < W - 1 ? (c + v[2]) >> 1 : c;
        lo = min(min(l, r), c);
        hi = max(max(l, r), c);
    };
    int plo, phi, rlo, rhi;
    bt(pf, plo, phi);
    bt(raw, rlo, rhi);
    return make_uint4((uint32_t)pf[1] | ((uint32_t)raw[1] << 16), (uint32_t)plo | ((uint32_t)rlo << 16),
                      (uint32_t)phi | ((uint32_t)rhi << 16), 0u);
}

__device__ __forceinline__ int bt_cost(const uint4 l, const uint4 r) {
    const us2 U = as_us2(l.x), U0 = as_us2(l.y), U1 = as_us2(l.z);
    const us2 V = as_us2(r.x), V0 = as_us2(r.y), V1 = as_us2(r.z);
    const us2 c0 = __builtin_elementwise_max(__builtin_elementwise_sub_sat(U, V1), __builtin_elementwise_sub_sat(V0, U));
    const us2 c1 = __builtin_elementwise_max(__builtin_elementwise_sub_sat(V, U1), __builtin_elementwise_sub_sat(U0, V));
    const uint32_t m = as_u32(__builtin_elementwise_min(c0, c1));
    return (int)(m & 0xFFFFu) + (int)(m >> 18);
}

template <int R>
__global__ __launch_bounds__(256) void k_sgbm_hsum_tiled(SgbmArgs a) {
    if (blockIdx.z) a.select_frame(blockIdx.z);   // frame batch
    extern __shared__ uint4 rec[];
    constexpr int W2 = 2 * R + 1;
    const int y = blockIdx.y, t = threadIdx.x;
    const int D = a.D, Wb = a.Wb;
    const int xb0 = blockIdx.x * kHX, xb1 = min(xb0 + kHX, Wb);   // output band columns
    // left records: band columns xb0-R .. xb1+R-1 (clamped to the band); right records:
    // image columns xr0 .. xr1 that those columns reach at d = D-1 .. 0
    const int nL = xb1 - xb0 + 2 * R;
    const int xr0 = a.X0 + max(xb0 - R, 0) - a.minD - (D - 1);
    const int xr1 = a.X0 + min(xb1 + R - 1, Wb - 1) - a.minD;
    const int nR = xr1 - xr0 + 1;
    uint4* recL = rec;
    uint4* recR = rec + nL;
    for (int i = t; i < nL + nR; i += 256) {
        if (i < nL) recL[i] = bt_record(a, a.L, y, a.X0 + min(max(xb0 - R + i, 0), Wb - 1));
        else recR[i - nL] = bt_record(a, a.R, y, xr0 + (i - nL));
    }
    __syncthreads();
    const int nc = max(1, kHX / D);                  // column chunks per disparity
    const int clen = (kHX + nc - 1) / nc;
    for (int item = t; item < D * nc; item += 256) {
        const int d = item % D, c = item / D;
        const int xs = xb0 + c * clen, xe = min(xb1, xs + clen);
        if (xs >= xe) continue;
        // cell (xb, d): left record xb - (xb0 - R), right record x(xb) - minD - d - xr0
        const int roff = a.X0 - a.minD - d - xr0;
        auto pc = [&](int xb) {
            const int xc = min(max(xb, 0), Wb - 1);
            return bt_cost(recL[xb - xb0 + R], recR[xc + roff]);
        };
        uint16_t* out = a.hsum + ((size_t)y * Wb + xs) * a.Dp + d;
        int ring[W2];
        int hs = 0;
#pragma unroll
        for (int k = 0; k < W2; ++k) {
            ring[k] = pc(xs - R + k);
            hs += ring[k];
        }
        out[0] = (uint16_t)hs;
        // step j (output column xs + 1 + j) drops entry j (ring slot j mod W2)
        for (int j0 = 0; xs + 1 + j0 < xe; j0 += W2) {
#pragma unroll
            for (int k = 0; k < W2; ++k) {
                const int x = xs + 1 + j0 + k;
                if (x < xe) {
                    const int pn = pc(x + R);
                    hs += pn - ring[k];
                    ring[k] = pn;
                    out[(size_t)(1 + j0 + k) * a.Dp] = (uint16_t)hs;
                }
            }
        }
    }
}

// window rows: C(y) = sum_{j=-r..r} hsum(clamp(y + j))
__global__ __launch_bounds__(256) void k_sgbm_vsum(SgbmArgs a) {
    if (blockIdx.z) a.select_frame(blockIdx.z);   // frame batch
    const size_t plane = (size_t)a.Wb * a.Dp;
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= plane) return;
    const uint16_t* h = a.hsum + i;
    uint16_t* c = a.C + i;
    const int H = a.H, r = a.r;
    int s = 0;
    for (int j = -r; j <= r; ++j) s += h[(size_t)min(max(j, 0), H - 1) * plane];
    c[0] = (uint16_t)s;
    for (int y0 = 1; y0 < H; y0 += 8) {   // 16 independent loads in flight per step of 8 rows
        int ad[8], sb[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int y = min(y0 + u, H - 1);
            ad[u] = h[(size_t)min(y + r, H - 1) * plane];
            sb[u] = h[(size_t)max(y - r - 1, 0) * plane];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            if (y0 + u >= H) break;
            s += ad[u] - sb[u];
            c[(size_t)(y0 + u) * plane] = (uint16_t)s;
        }
    }
}

// The same window-row sums, 8 elements (16 B) per lane over the contiguous (x, d) plane
// and the rows split into bands of `vb` rows (each band re-sums its first window), so a
// 1080p D=128 volume runs ~3.6k waves with 16-byte loads instead of 448 waves of 2-byte
// loads.  Sums wrap mod 2^16 in packed u16 lanes: bit-identical to the u16 store of the
// int sum in k_sgbm_vsum.
typedef unsigned short us2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint4 add4(uint4 s, uint4 a, uint4 b) {
    uint4 o;
    o.x = __builtin_bit_cast(uint32_t, __builtin_bit_cast(us2v, s.x) + __builtin_bit_cast(us2v, a.x) - __builtin_bit_cast(us2v, b.x));
    o.y = __builtin_bit_cast(uint32_t, __builtin_bit_cast(us2v, s.y) + __builtin_bit_cast(us2v, a.y) - __builtin_bit_cast(us2v, b.y));
    o.z = __builtin_bit_cast(uint32_t, __builtin_bit_cast(us2v, s.z) + __builtin_bit_cast(us2v, a.z) - __builtin_bit_cast(us2v, b.z));
    o.w = __builtin_bit_cast(uint32_t, __builtin_bit_cast(us2v, s.w) + __builtin_bit_cast(us2v, a.w) - __builtin_bit_cast(us2v, b.w));
    return o;
}

template <int R>   // window radius: the 2R+1 rows of the window stay in a register ring
__global__ __launch_bounds__(256) void k_sgbm_vsum8(SgbmArgs a, int vb) {
    if (blockIdx.z) a.select_frame(blockIdx.z);   // frame batch
    constexpr int W2 = 2 * R + 1;
    const size_t p8 = (size_t)a.Wb * a.Dp / 8;        // uint4 per row plane
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= p8) return;
    const uint4* h = reinterpret_cast<const uint4*>(a.hsum) + i;
    uint4* c = reinterpret_cast<uint4*>(a.C) + i;
    const int H = a.H;
    const int y0 = blockIdx.y * vb, n = min(H, y0 + vb) - y0;
    const uint4 z = make_uint4(0u, 0u, 0u, 0u);
    // ring[k] = row clamp(y0 - R + k): the window of output row y0
    uint4 ring[W2];
    uint4 s = z;
#pragma unroll
    for (int k = 0; k < W2; ++k) {
        ring[k] = h[(size_t)min(max(y0 - R + k, 0), H - 1) * p8];
        s = add4(s, ring[k], z);
    }
    c[(size_t)y0 * p8] = s;
    // output row y0 + t adds row clamp(y0 + t + R) and drops ring slot (t - 1) mod W2, which
    // holds row clamp(y0 + t - R - 1); loads past the band stay in the image (clamped)
    for (int t0 = 1; t0 < n; t0 += W2) {
        uint4 in[W2];
#pragma unroll
        for (int u = 0; u < W2; ++u) in[u] = h[(size_t)min(y0 + t0 + u + R, H - 1) * p8];
#pragma unroll
        for (int u = 0; u < W2; ++u) {
            s = add4(s, in[u], ring[u]);
            ring[u] = in[u];
            if (t0 + u < n) c[(size_t)(y0 + t0 + u) * p8] = s;
        }
    }
}

// Pixel cost + both window sums in one pass (r <= 4): the hsum volume never leaves the
// chip.  Every wave is independent (no workgroup barriers): it owns 64 consecutive
// disparities (lane = d, so its stores coalesce), a chunk of CL band columns and a band of
// output rows, and walks the rows top to bottom.  Per input row it copies that row's
// {value, BT lo, BT hi} records (from k_sgbm_records' planes, prefetched into registers one
// row ahead) into its own LDS slice, forms the CL window-column sums of the chunk with a
// horizontal running sum (CL + 2R pixel costs per lane) and keeps the last 2R+1 rows of them
// in a register ring of packed u16 pairs: C(y) = C(y-1) + hsum(y+R) - hsum(y-R-1), by
// v_pk_add/sub_u16 (exact: every window sum fits 16 bits, enqueue_sgbm checks).  Rows are
// clamped like k_sgbm_vsum's, columns like k_sgbm_hsum_tiled's.
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_add16(uint32_t a, uint32_t b) {   // v_pk_add_u16 (mod 2^16)
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, a) + __builtin_bit_cast(u16x2, b));
}
__device__ __forceinline__ uint32_t pk_sub16(uint32_t a, uint32_t b) {   // v_pk_sub_u16 (mod 2^16)
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, a) - __builtin_bit_cast(u16x2, b));
}

// Per-pixel {value, BT lo, BT hi} records of both images (k_sgbm_cost stages rows of them)
__global__ __launch_bounds__(256) void k_sgbm_records(SgbmArgs a) {
    if (blockIdx.z) a.select_frame(blockIdx.z);   // frame batch
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y >> 1, img = blockIdx.y & 1;
    if (x >= a.W) return;
    a.recs[((size_t)img * a.H + y) * a.W + x] = bt_record(a, img ? a.R : a.L, y, x);
}

// columns per lane (ring: (2R+1)*CL/2 VGPRs).  A chunk re-costs its 2R halo columns; wider
// chunks for r 3 (24: 256 VGPRs, no spills) measured slower (D=320 w7: 362 -> 355 frames/s per
// call, 460-470 -> 447-456 at batch 8, round 4), r 4 with 24+ spills or lands in scratch
__host__ __device__ constexpr int cost_cl(int r) { return r <= 2 ? 32 : 16; }
template <int R> struct CostCfg {
    static constexpr int CL = cost_cl(R);
    static constexpr int NREC = 2 * (CL + 2 * R) + 63;    // records per row of a wave
    static constexpr int NRT = (NREC + 63) / 64;          // per lane
};

// wave-scope ordering of the LDS slice (LDS instructions of one wave execute in order; this
// keeps the compiler from moving accesses across)
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// waves per SIMD the register budget allows (r 3: 160 VGPRs since the window sums update by
// v_sad_u32; 3 waves measured even with 2, 390 vs 389 frames/s at D=320 w7)
#ifndef SV_COST_WPE
#define SV_COST_WPE(R) ((R) == 3 ? 3 : 2)
#endif
template <int R>
__global__ __launch_bounds__(64, SV_COST_WPE(R)) void k_sgbm_cost(SgbmArgs a, int vb, int ndg) {
    if (blockIdx.z) a.select_frame(blockIdx.z);   // frame batch
    constexpr int W2 = 2 * R + 1, CL = CostCfg<R>::CL, CP = CL / 2, NRT = CostCfg<R>::NRT;
    __shared__ uint4 rec[2 * CostCfg<R>::NREC];
    const int lane = threadIdx.x, D = a.D, Wb = a.Wb, H = a.H;
    const int dg = (int)blockIdx.y % ndg, band = (int)blockIdx.y / ndg;
    const int d = 64 * dg + lane, dmax = min(64 * dg + 63, D - 1);
    const int xs = (int)blockIdx.x * CL;                 // first band column of the chunk
    const int y0 = band * vb, n = min(H, y0 + vb) - y0;
    const bool active = d < D;
    // records: left band columns xs-R .. xs+CL+R-1 (band-clamped), right image columns
    // xr0 .. xr1 that those columns reach at d = dmax .. 64*dg
    const int xr0 = a.X0 + max(xs - R, 0) - a.minD - dmax;
    const int xr1 = a.X0 + min(xs + CL + R - 1, Wb - 1) - a.minD - 64 * dg;
    const int nL = CL + 2 * R;
    const int nrec = nL + (xr1 - xr0 + 1);
    const int roff = a.X0 - a.minD - min(d, dmax) - xr0;
    const uint4* recLg = a.recs;                          // [H][W] left records, then right
    const uint4* recRg = a.recs + (size_t)H * a.W;
    uint32_t nx[NRT][4];   // scalar words (a uint4 array stayed in scratch)
    auto load = [&](int iy) {
        const uint4* lrow = recLg + (size_t)iy * a.W;
        const uint4* rrow = recRg + (size_t)iy * a.W;
#pragma unroll
        for (int q = 0; q < NRT; ++q) {   // unconditional (clamped) loads keep nx in VGPRs
            const int i = min(lane + 64 * q, nrec - 1);
            const uint4 v = i < nL ? lrow[a.X0 + min(max(xs - R + i, 0), Wb - 1)] : rrow[xr0 + (i - nL)];
            nx[q][0] = v.x;
            nx[q][1] = v.y;
            nx[q][2] = v.z;
            nx[q][3] = v.w;
        }
    };
    auto put = [&](uint4* buf) {
#pragma unroll
        for (int q = 0; q < NRT; ++q) {
            const int i = lane + 64 * q;
            if (i < nrec) buf[i] = make_uint4(nx[q][0], nx[q][1], nx[q][2], nx[q][3]);
        }
        wave_lds_sync();
    };
    // window-column sums of this lane's CL cells from the row in `buf`, packed in pairs;
    // interior chunks (no band clamp among their columns) read with immediate offsets
    const bool interior = xs - R >= 0 && xs + CL + R - 1 <= Wb - 1;
    // (left records as uniform scalar loads instead of LDS broadcasts: 275 -> 700 us per 1080p
    // frame, the loads' latency exposed)
    auto hrow = [&](const uint4* buf, uint32_t (&hp)[CP]) {
        int pcs[CL + 2 * R];
        if (interior) {
            const uint4* rb = buf + nL + (xs - R + roff);
#pragma unroll
            for (int k = 0; k < CL + 2 * R; ++k) pcs[k] = bt_cost(buf[k], rb[k]);
        } else {
#pragma unroll
            for (int k = 0; k < CL + 2 * R; ++k)
                pcs[k] = bt_cost(buf[k], buf[nL + min(max(xs - R + k, 0), Wb - 1) + roff]);
        }
        uint32_t hs = 0;
#pragma unroll
        for (int k = 0; k < W2; ++k) hs += (uint32_t)pcs[k];
        uint32_t lo = hs;
#pragma unroll
        for (int j = 1; j < CL; ++j) {
            sad_u32_acc(hs, (uint32_t)pcs[j - 1], (uint32_t)pcs[j + 2 * R]);   // hs - leaving + entering
            if (j & 1) hp[j >> 1] = (lo & 0xFFFFu) | (hs << 16);
            else lo = hs;
        }
    };
    // stores through a per-row buffer descriptor: 32-bit lane offsets, the column step as the
    // uniform soffset (no per-column 64-bit addresses to keep live)
    const int voff = 2 * (xs * a.Dp + d);
    auto store = [&](int y, const uint32_t (&cp)[CP]) {
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(a.C + (size_t)y * Wb * a.Dp, 0, 0x7FFFFFFF, 0x00020000);
#pragma unroll
        for (int j = 0; j < CL; ++j)
            if (xs + j < Wb)
                __builtin_amdgcn_raw_buffer_store_b16((uint16_t)(cp[j >> 1] >> (16 * (j & 1))), rs, voff,
                                                      2 * j * a.Dp, 0);
    };
    constexpr int NB = CostCfg<R>::NREC;
    int cur = 0;   // LDS buffer of the row being summed: rec + cur * NB
    // warm-up: rows clamp(y0-R .. y0+R) into the ring, C(y0) = their sum
    uint32_t ring[W2][CP], acc[CP];
#pragma unroll
    for (int j = 0; j < CP; ++j) acc[j] = 0u;
    load(min(max(y0 - R, 0), H - 1));
    put(rec);
#pragma unroll
    for (int k = 0; k < W2; ++k) {
        const int ny = k < W2 - 1 ? y0 - R + k + 1 : y0 + 1 + R;
        load(min(max(ny, 0), H - 1));
        hrow(rec + cur * NB, ring[k]);
#pragma unroll
        for (int j = 0; j < CP; ++j) acc[j] = pk_add16(acc[j], ring[k][j]);
        put(rec + (cur ^ 1) * NB);
        cur ^= 1;
    }
    if (active) store(y0, acc);
    // output row y0 + t adds row clamp(y0 + t + R) and drops ring slot (t - 1) mod W2
    for (int t0 = 1; t0 < n; t0 += W2) {
#pragma unroll
        for (int u = 0; u < W2; ++u) {
            if (t0 + u < n) {   // uniform across the wave
                load(min(y0 + t0 + u + 1 + R, H - 1));
                uint32_t hp[CP];
                hrow(rec + cur * NB, hp);
#pragma unroll
                for (int j = 0; j < CP; ++j) {   // both u16 halves: acc - leaving + entering
                    sad_u32_acc(acc[j], ring[u][j], hp[j]);
                    ring[u][j] = hp[j];
                }
                if (active) store(y0 + t0 + u, acc);
                put(rec + (cur ^ 1) * NB);
                cur ^= 1;
            }
        }
    }
}

// The path kernels run one line's DP (a chain of W or H dependent steps: the path minimum
// of step s feeds step s+1) in a 16-lane row of a wave, so a wave advances 4 lines at once
// and the loop-carried chain per step is ~11 VALU ops: the d+-1 neighbours by row_shr/shl
// DPP, 4 ops per disparity, an in-lane min3 tree and a 4-step row_ror min butterfly (no
// readlane, no SALU).  Lane j of a row owns d = j*DPL .. j*DPL+DPL-1.  The inputs of the
// next PF steps are loaded ahead into a register ring; the loads are unconditional (a
// branch between a prefetch and its use makes the compiler wait for it at once).

// DPL contiguous elements of type T as one vector load/store.
constexpr int pack_align(int bytes) {
    return bytes % 16 == 0 ? 16 : bytes % 8 == 0 ? 8 : bytes % 4 == 0 ? 4 : bytes % 2 == 0 ? 2 : 1;
}
template <typename T, int DPL>
struct alignas(pack_align(sizeof(T) * DPL)) Pack {
    T v[DPL];
};

// Lines of LPC lanes (16: one DPP row; 32: two rows, joined by v_permlane16_swap, which
// hands each row of a pair the other's values in one VALU op).
struct RowPair {
    int even, odd;   // per lane: the value of the pair's even row / odd row
};
__device__ __forceinline__ RowPair row_pair(int v) {
    const auto r = __builtin_amdgcn_permlane16_swap((unsigned)v, (unsigned)v, false, false);
    return {(int)r[0], (int)r[1]};
}
template <int LPC> __device__ __forceinline__ int line_min(int v) {
    v = row_min(v);
    if constexpr (LPC == 32) {
        const RowPair p = row_pair(v);
        v = min(p.even, p.odd);
    }
    return v;
}
template <int LPC> __device__ __forceinline__ uint32_t line_min_u(uint32_t v) {
    v = row_min_u(v);
    if constexpr (LPC == 32) {
        const RowPair p = row_pair((int)v);
        v = min((uint32_t)p.even, (uint32_t)p.odd);
    }
    return v;
}
template <int LPC> __device__ __forceinline__ int line_max(int v) {
    v = row_max(v);
    if constexpr (LPC == 32) {
        const RowPair p = row_pair(v);
        v = max(p.even, p.odd);
    }
    return v;
}
// value of lane j-1 / j+1 of the line (`edge` at the line's ends)
template <int LPC> __device__ __forceinline__ int from_left(int v, int edge, int j) {
    if constexpr (LPC == 16) return dpp_shr1(v, edge);
    const int t = __builtin_amdgcn_update_dpp(edge, v, 0x138, 0xF, 0xF, false);   // wave_shr:1
    return j == 0 ? edge : t;
}
template <int LPC> __device__ __forceinline__ int from_right(int v, int edge, int j) {
    if constexpr (LPC == 16) return dpp_shl1(v, edge);
    const int t = __builtin_amdgcn_update_dpp(edge, v, 0x130, 0xF, 0xF, false);   // wave_shl:1
    return j == LPC - 1 ? edge : t;
}

// One SGBM step for the DPL disparities of a lane: OpenCV's
// L = C + min(prev[d], prev[d-1] + P1, prev[d+1] + P1, minprev + P2) - (minprev + P2).
// pad[k] = INT_MIN for d < D, kInf for the padding disparities (which stay at kInf: a max
// instead of a per-disparity branch).
template <int DPL, int LPC>
__device__ __forceinline__ void path_step(int (&prev)[DPL], const int (&c)[DPL], int mn, int P1, int P2,
                                          const int (&pad)[DPL], int j) {
    const int lo_in = from_left<LPC>(prev[DPL - 1], kInf, j);
    const int hi_in = from_right<LPC>(prev[0], kInf, j);
    int nxt[DPL];
    const int mp = mn + P2, nmp = -mp;
#pragma unroll
    for (int k = 0; k < DPL; ++k) {
        const int lo = k > 0 ? prev[k - 1] : lo_in;
        const int hi = k < DPL - 1 ? prev[k + 1] : hi_in;
        const int m = min(min(prev[k], min(lo, hi) + P1), mp);
        nxt[k] = max(c[k] + m + nmp, pad[k]);
    }
#pragma unroll
    for (int k = 0; k < DPL; ++k) prev[k] = nxt[k];
}

template <int DPL>
__device__ __forceinline__ void pad_init(int (&pad)[DPL], int dbase, int D) {
#pragma unroll
    for (int k = 0; k < DPL; ++k) pad[k] = dbase + k < D ? (int)0x80000000 : kInf;
}

template <int DPL>
__device__ __forceinline__ int lane_min(const int (&v)[DPL]) {
    int m = v[0];
#pragma unroll
    for (int k = 1; k < DPL; ++k) m = min(m, v[k]);
    return m;
}

// Horizontal paths: 64/LPC rows per wave; blockIdx.y = 0: left->right into Llr, 1:
// right->left into Lrl.
// WPE: waves per SIMD the register budget allows (2 for frame batches, where ~2 lines' waves
// share a SIMD; 1 with deeper prefetch for single frames, whose ~540 waves leave SIMDs idle)
template <int DPL, int LPC, typename LT, int PF, int WPE>
__global__ __launch_bounds__(64, WPE) void k_sgbm_hpath(SgbmArgs a) {
    if (blockIdx.z) a.select_frame(blockIdx.z);   // frame batch
    constexpr int NL = 64 / LPC;
    const int lane = threadIdx.x, g = lane / LPC, j = lane & (LPC - 1);
    const int y = blockIdx.x * NL + g, dir = blockIdx.y;
    const int D = a.D, Wb = a.Wb, Dp = a.Dp, dbase = j * DPL;
    // rows past H and lanes past D re-read valid cells and store into a private dummy
    // slot: no load or store sits under a branch
    const bool live = y < a.H && dbase < D;
    const int yc = min(y, a.H - 1);
    // x walks 0 .. Wb-1 (dir 0) or Wb-1 .. 0 (dir 1): pointers step by +-Dp per x
    const ptrdiff_t xstep = dir == 0 ? Dp : -(ptrdiff_t)Dp;
    const size_t x0 = dir == 0 ? 0 : (size_t)(Wb - 1) * Dp;
    LT* Lp = live ? static_cast<LT*>(dir == 0 ? a.Llr : a.Lrl) + (size_t)yc * Wb * Dp + dbase + x0
                  : reinterpret_cast<LT*>(a.dummy) + lane * (128 / sizeof(LT));
    const ptrdiff_t lstep = live ? xstep : 0;
    const uint16_t* Crow = a.C + (size_t)yc * Wb * Dp + (dbase < D ? dbase : 0) + x0;
    using CP = Pack<uint16_t, DPL>;
    using LP = Pack<LT, DPL>;
    CP ring[PF];
#pragma unroll
    for (int p = 0; p < PF; ++p) ring[p] = *reinterpret_cast<const CP*>(Crow + (ptrdiff_t)min(p, Wb - 1) * xstep);
    // next load: x index PF, clamped to Wb-1 (the pointer stops there)
    const uint16_t* Cn = Crow + (ptrdiff_t)min(PF, Wb - 1) * xstep;
    int prev[DPL], pad[DPL];
    pad_init<DPL>(pad, dbase, D);
#pragma unroll
    for (int k = 0; k < DPL; ++k) prev[k] = dbase + k < D ? 0 : kInf;
    int mn = 0;
    auto step = [&](const CP& cp) {
        int c[DPL];
#pragma unroll
        for (int k = 0; k < DPL; ++k) c[k] = (int)cp.v[k];
        path_step<DPL, LPC>(prev, c, mn, a.P1, a.P2, pad, j);
        mn = line_min<LPC>(lane_min<DPL>(prev));
        LP o;
#pragma unroll
        for (int k = 0; k < DPL; ++k) o.v[k] = (LT)prev[k];
        *reinterpret_cast<LP*>(Lp) = o;
        Lp += lstep;
    };
    int s0 = 0;
    for (; s0 + PF <= Wb; s0 += PF) {
#pragma unroll
        for (int u = 0; u < PF; ++u) {
            const CP cur = ring[u];
            ring[u] = *reinterpret_cast<const CP*>(Cn);
            Cn += s0 + u + PF < Wb - 1 ? xstep : 0;
            step(cur);
        }
    }
#pragma unroll
    for (int u = 0; u < PF; ++u)
        if (s0 + u < Wb) step(ring[u]);
}

struct BandOut {      // one 8-byte record per band pixel
    int16_t disp, best;
    int32_t minS;
};

// Winner-take-all of one pixel on a line of LPC lanes (lane j holds S[dbase .. dbase+DPL)):
// argmin over keys (S << 9) + (d + 2^29) = ((S + 2^20) << 9) | d (first minimum), the
// uniqueness test from the smallest S with |d - b| > 1 (24-bit products: |S| < 2^23), S[b-1]
// and S[b+1] through the line's LDS slice (LDS ops of one wave are ordered), the sub-pixel
// parabola with a float-reciprocal quotient plus one correction (C's truncating division;
// |num| <= 17 * den / 2 because S[b+-1] >= minS).
template <int DPL, int LPC>
__device__ __forceinline__ BandOut wta_line(const SgbmArgs& a, const int (&s)[DPL], int dbase, int* my_s,
                                            const int* line_s) {
    const int D = a.D;
    uint32_t key = 0xFFFFFFFFu;
#pragma unroll
    for (int k = 0; k < DPL; ++k) {
        my_s[k] = s[k];
        if (dbase + k < D) key = min(key, ((uint32_t)s[k] << 9) + ((uint32_t)(dbase + k) + (1u << 29)));
    }
    key = line_min_u<LPC>(key);
    const int b = (int)(key & 511u);
    const int minS = (int)(key >> 9) - (1 << 20);
    const int e = dbase - b + 1;
    int m2 = 0x7FFFFFFF;
#pragma unroll
    for (int k = 0; k < DPL; ++k)
        if (dbase + k < D && (unsigned)(e + k) > 2u) m2 = min(m2, s[k]);
    m2 = line_min<LPC>(m2);
    const bool viol = m2 != 0x7FFFFFFF && __mul24(m2, 100 - a.uniq) < __mul24(minS, 100);
    int d16 = b * 16;
    if (b > 0 && b < D - 1) {
        const int sm = line_s[b - 1], sp = line_s[b + 1];
        const int denom2 = max(sm + sp - 2 * minS, 1);
        const int num = (sm - sp) * 16 + denom2, den = denom2 * 2;
        const int an = abs(num);
        int q = (int)((float)an * __builtin_amdgcn_rcpf((float)den));
        const int r = an - (int)__umul24((unsigned)q, (unsigned)den);
        q += (r >= den) - (r < 0);
        d16 += num < 0 ? -q : q;
    }
    BandOut o;
    o.disp = (int16_t)(viol ? (a.minD - 1) * 16 : d16 + a.minD * 16);
    o.best = (int16_t)b;
    o.minS = viol ? 0x7FFFFFFF : minS;
    return o;
}

// Top->bottom path: one band column per line of LPC lanes walking down the rows -> L_tb.  It
// depends on C only, so it runs on a second stream beside the horizontal paths (both are
// chains of dependent steps that leave most of a SIMD idle).
template <int DPL, int LPC, typename LT, int PF>
__global__ __launch_bounds__(64) void k_sgbm_vpath(SgbmArgs a) {
    if (blockIdx.z) a.select_frame(blockIdx.z);   // frame batch
    constexpr int NL = 64 / LPC;
    const int lane = threadIdx.x, g = lane / LPC, j = lane & (LPC - 1);
    const int xb = blockIdx.x * NL + g;
    const int D = a.D, Wb = a.Wb, dbase = j * DPL;
    const bool live = xb < Wb && dbase < D;
    const size_t plane = (size_t)Wb * a.Dp;
    const size_t col = (size_t)min(xb, Wb - 1) * a.Dp + (dbase < D ? dbase : 0);
    const uint16_t* Cc = a.C + col;
    LT* Lt = live ? static_cast<LT*>(a.Ltb) + col : reinterpret_cast<LT*>(a.dummy) + lane * (128 / sizeof(LT));
    const size_t ystride = live ? plane : 0;
    using CP = Pack<uint16_t, DPL>;
    using LP = Pack<LT, DPL>;
    CP rc[PF];
#pragma unroll
    for (int p = 0; p < PF; ++p) rc[p] = *reinterpret_cast<const CP*>(Cc + (size_t)min(p, a.H - 1) * plane);
    int prev[DPL], pad[DPL];
    pad_init<DPL>(pad, dbase, D);
#pragma unroll
    for (int k = 0; k < DPL; ++k) prev[k] = dbase + k < D ? 0 : kInf;
    int mn = 0;
    auto row = [&](int y, const CP& cp) {
        int c[DPL];
#pragma unroll
        for (int k = 0; k < DPL; ++k) c[k] = (int)cp.v[k];
        path_step<DPL, LPC>(prev, c, mn, a.P1, a.P2, pad, j);
        mn = line_min<LPC>(lane_min<DPL>(prev));
        LP o;
#pragma unroll
        for (int k = 0; k < DPL; ++k) o.v[k] = (LT)prev[k];
        *reinterpret_cast<LP*>(Lt + (size_t)y * ystride) = o;
    };
    int y0 = 0;
    for (; y0 + PF <= a.H; y0 += PF) {
#pragma unroll
        for (int u = 0; u < PF; ++u) {
            const CP c = rc[u];
            rc[u] = *reinterpret_cast<const CP*>(Cc + (size_t)min(y0 + u + PF, a.H - 1) * plane);
            row(y0 + u, c);
        }
    }
#pragma unroll
    for (int u = 0; u < PF; ++u)
        if (y0 + u < a.H) row(y0 + u, rc[u]);
}

// Top->bottom path fused with the winner-take-all (unfused launches, VWTA): the horizontal
// paths run first (both directions stored), then each line walks its band column down the
// rows like k_sgbm_vpath and at every row sums its fresh L_tb with L_lr and L_rl (prefetched
// in register rings beside C) and runs wta_line on the sum: L_tb is never stored, so its
// write and the WTA's read of it leave the pipeline, and the WTA launch goes.
template <int DPL, int LPC, typename LT, int PF, int WPE>
__global__ __launch_bounds__(64, WPE) void k_sgbm_vpath_wta(SgbmArgs a) {
    if (blockIdx.z) a.select_frame(blockIdx.z);   // frame batch
    constexpr int NL = 64 / LPC;
    const int lane = threadIdx.x, g = lane / LPC, j = lane & (LPC - 1);
    const int xb = blockIdx.x * NL + g;
    const int D = a.D, Wb = a.Wb, dbase = j * DPL;
    const size_t plane = (size_t)Wb * a.Dp;
    const size_t col = (size_t)min(xb, Wb - 1) * a.Dp + (dbase < D ? dbase : 0);
    const uint16_t* Cc = a.C + col;
    const LT* Ac = static_cast<const LT*>(a.Llr) + col;
    const LT* Bc = static_cast<const LT*>(a.Lrl) + col;
    BandOut* bout = reinterpret_cast<BandOut*>(a.band) + min(xb, Wb - 1);
    const bool emit = xb < Wb && j == 0;
    __shared__ int lds_s[64 * DPL];
    using CP = Pack<uint16_t, DPL>;
    using LP = Pack<LT, DPL>;
    CP rc[PF];
    LP ra[PF], rb[PF];
#pragma unroll
    for (int p = 0; p < PF; ++p) {
        const size_t o = (size_t)min(p, a.H - 1) * plane;
        rc[p] = *reinterpret_cast<const CP*>(Cc + o);
        ra[p] = *reinterpret_cast<const LP*>(Ac + o);
        rb[p] = *reinterpret_cast<const LP*>(Bc + o);
    }
    int prev[DPL], pad[DPL];
    pad_init<DPL>(pad, dbase, D);
#pragma unroll
    for (int k = 0; k < DPL; ++k) prev[k] = dbase + k < D ? 0 : kInf;
    int mn = 0;
    auto row = [&](int y, const CP& cp, const LP& lp, const LP& rp) {
        int c[DPL];
#pragma unroll
        for (int k = 0; k < DPL; ++k) c[k] = (int)cp.v[k];
        path_step<DPL, LPC>(prev, c, mn, a.P1, a.P2, pad, j);
        mn = line_min<LPC>(lane_min<DPL>(prev));
        int sm[DPL];
#pragma unroll
        for (int k = 0; k < DPL; ++k) sm[k] = prev[k] + (int)lp.v[k] + (int)rp.v[k];
        const BandOut o = wta_line<DPL, LPC>(a, sm, dbase, lds_s + lane * DPL, lds_s + g * LPC * DPL);
        if (emit) bout[(size_t)y * Wb] = o;
    };
    int y0 = 0;
    for (; y0 + PF <= a.H; y0 += PF) {
#pragma unroll
        for (int u = 0; u < PF; ++u) {
            const CP c = rc[u];
            const LP la = ra[u], lb = rb[u];
            const size_t o = (size_t)min(y0 + u + PF, a.H - 1) * plane;
            rc[u] = *reinterpret_cast<const CP*>(Cc + o);
            ra[u] = *reinterpret_cast<const LP*>(Ac + o);
            rb[u] = *reinterpret_cast<const LP*>(Bc + o);
            row(y0 + u, c, la, lb);
        }
    }
#pragma unroll
    for (int u = 0; u < PF; ++u)
        if (y0 + u < a.H) row(y0 + u, rc[u], ra[u], rb[u]);
}

// S = L_lr + L_rl + L_tb and the winner-take-all, one pixel per line of LPC lanes: every
// pixel is independent, so this runs with full occupancy (it was the issue-bound half of a
// fused vertical-path kernel on ~900 waves).
template <int DPL, int LPC, typename LT>
__global__ __launch_bounds__(64) void k_sgbm_wta(SgbmArgs a) {
    if (blockIdx.z) a.select_frame(blockIdx.z);   // frame batch
    constexpr int NL = 64 / LPC;
    const int lane = threadIdx.x, g = lane / LPC, j = lane & (LPC - 1);
    const size_t npx = (size_t)a.H * a.Wb;
    const size_t p = (size_t)blockIdx.x * NL + g;
    const int dbase = j * DPL;
    const size_t pc = p < npx ? p : npx - 1;
    const size_t off = pc * a.Dp + (dbase < a.D ? dbase : 0);
    using LP = Pack<LT, DPL>;
    const LP l = *reinterpret_cast<const LP*>(static_cast<const LT*>(a.Llr) + off);
    const LP r = *reinterpret_cast<const LP*>(static_cast<const LT*>(a.Lrl) + off);
    const LP t = *reinterpret_cast<const LP*>(static_cast<const LT*>(a.Ltb) + off);
    __shared__ int lds_s[64 * DPL];
    int s[DPL];
#pragma unroll
    for (int k = 0; k < DPL; ++k) s[k] = (int)l.v[k] + (int)r.v[k] + (int)t.v[k];
    const BandOut o = wta_line<DPL, LPC>(a, s, dbase, lds_s + lane * DPL, lds_s + g * LPC * DPL);
    if (p < npx && j == 0) reinterpret_cast<BandOut*>(a.band)[p] = o;
}

// Right->left path fused with the winner-take-all: the line walks x = Wb-1 .. 0 like
// k_sgbm_hpath's second direction, and at every step sums its fresh L_rl[x] with L_lr[x]
// and L_tb[x] (prefetched in register rings beside C) and runs wta_line on the sum.  L_rl
// is never stored, so the R->L volume's write and the WTA's read of it (2 of the pipeline's
// volume passes) disappear, and so does the WTA launch.  The WTA work hangs off the DP
// chain (only `prev` and the path minimum are loop-carried), so it fills the chain's gaps.
// 2 waves per SIMD (256 VGPRs) where that does not spill: batches put ~2 lines' waves on a SIMD
template <int DPL, typename LT, int PF>
__global__ __launch_bounds__(64, DPL <= 16 ? 2 : 1) void k_sgbm_rl_wta(SgbmArgs a) {
    if (blockIdx.z) a.select_frame(blockIdx.z);   // frame batch
    constexpr int LPC = 16, NL = 64 / LPC;
    const int lane = threadIdx.x, g = lane / LPC, j = lane & (LPC - 1);
    const int y = blockIdx.x * NL + g;
    const int D = a.D, Wb = a.Wb, Dp = a.Dp, dbase = j * DPL;
    const int yc = min(y, a.H - 1);
    const size_t x0 = (size_t)(Wb - 1) * Dp;
    const size_t row = (size_t)yc * Wb * Dp + (dbase < D ? dbase : 0) + x0;
    const uint16_t* Cp = a.C + row;
    const LT* Ap = static_cast<const LT*>(a.Llr) + row;
    const LT* Bp = static_cast<const LT*>(a.Ltb) + row;
    BandOut* bout = reinterpret_cast<BandOut*>(a.band) + (size_t)yc * Wb + (Wb - 1);
    const bool emit = y < a.H && j == 0;
    __shared__ int lds_s[64 * DPL];
    using CP = Pack<uint16_t, DPL>;
    using LP = Pack<LT, DPL>;
    CP rc[PF];
    LP ra[PF], rb[PF];
#pragma unroll
    for (int p = 0; p < PF; ++p) {
        const ptrdiff_t o = -(ptrdiff_t)min(p, Wb - 1) * Dp;
        rc[p] = *reinterpret_cast<const CP*>(Cp + o);
        ra[p] = *reinterpret_cast<const LP*>(Ap + o);
        rb[p] = *reinterpret_cast<const LP*>(Bp + o);
    }
    ptrdiff_t on = -(ptrdiff_t)min(PF, Wb - 1) * Dp;   // next load: step PF, clamped to x = 0
    int prev[DPL], pad[DPL];
    pad_init<DPL>(pad, dbase, D);
#pragma unroll
    for (int k = 0; k < DPL; ++k) prev[k] = dbase + k < D ? 0 : kInf;
    int mn = 0;
    auto step = [&](int t, const CP& cp, const LP& lp, const LP& tp) {
        int c[DPL];
#pragma unroll
        for (int k = 0; k < DPL; ++k) c[k] = (int)cp.v[k];
        path_step<DPL, LPC>(prev, c, mn, a.P1, a.P2, pad, j);
        mn = line_min<LPC>(lane_min<DPL>(prev));
        int s[DPL];
#pragma unroll
        for (int k = 0; k < DPL; ++k) s[k] = prev[k] + (int)lp.v[k] + (int)tp.v[k];
        const BandOut o = wta_line<DPL, LPC>(a, s, dbase, lds_s + lane * DPL, lds_s + g * LPC * DPL);
        if (emit) bout[-t] = o;
    };
    int s0 = 0;
    for (; s0 + PF <= Wb; s0 += PF) {
#pragma unroll
        for (int u = 0; u < PF; ++u) {
            const CP cc = rc[u];
            const LP la = ra[u], lb = rb[u];
            rc[u] = *reinterpret_cast<const CP*>(Cp + on);
            ra[u] = *reinterpret_cast<const LP*>(Ap + on);
            rb[u] = *reinterpret_cast<const LP*>(Bp + on);
            on -= s0 + u + PF < Wb - 1 ? Dp : 0;
            step(s0 + u, cc, la, lb);
        }
    }
#pragma unroll
    for (int u = 0; u < PF; ++u)
        if (s0 + u < Wb) step(s0 + u, rc[u], ra[u], rb[u]);
}

// Left-right consistency (disp12MaxDiff) and band borders: one workgroup per row.
__global__ __launch_bounds__(256) void k_sgbm_lrcheck(SgbmArgs a) {
    if (blockIdx.z) a.select_frame(blockIdx.z);   // frame batch
    extern __shared__ unsigned long long keys[];
    const int y = blockIdx.x, t = threadIdx.x, W = a.W, Wb = a.Wb;
    for (int x = t; x < W; x += 256) keys[x] = ~0ull;
    __syncthreads();
    const BandOut* band = reinterpret_cast<const BandOut*>(a.band) + (size_t)y * Wb;
    for (int xb = t; xb < Wb; xb += 256) {
        const int ms = band[xb].minS;
        if (ms < 32767) {                                   // disp2cost starts at SHRT_MAX
            const int x = a.X0 + xb;
            const int x2 = x - (band[xb].best + a.minD);
            const unsigned long long k = ((unsigned long long)(uint32_t)(ms + 0x40000000) << 32) |
                                         (uint32_t)(0xFFFFFFFFu - (uint32_t)x);
            atomicMin(&keys[x2], k);
        }
    }
    __syncthreads();
    const int inv = (a.minD - 1) * 16;
    int16_t* orow = a.out + (size_t)y * a.opitch;
    for (int x = t; x < W; x += 256) {
        int v = inv;
        const int xb = x - a.X0;
        if (xb >= 0 && xb < Wb) {
            v = band[xb].disp;
            if (v != inv && a.disp12 >= 0) {
                const int dd = (v >> 4), du = (v + 15) >> 4;
                const int x1 = x - dd, x2 = x - du;
                auto d2 = [&](int xx) -> int {
                    const unsigned long long k = keys[xx];
                    if (k == ~0ull) return a.minD - 1;
                    const int xs = (int)(0xFFFFFFFFu - (uint32_t)(k & 0xFFFFFFFFull));
                    return xs - xx;
                };
                if (x1 >= 0 && x1 < W && x2 >= 0 && x2 < W) {
                    const int a1 = d2(x1), a2 = d2(x2);
                    if (a1 >= a.minD && abs(a1 - dd) > a.disp12 && a2 >= a.minD && abs(a2 - du) > a.disp12)
                        v = inv;
                }
            }
        }
        orow[x] = (int16_t)v;
    }
}

// ---- filterSpeckles: union-find connected components -----------------------------------
// Find with path halving: a non-root's parent is only ever replaced by one of its
// ancestors (roots are the only entries unite() hooks), so the plain stores keep every
// node inside its tree while shortening the chains.
__device__ __forceinline__ int uf_find(int* p, int x) {
    int q = __atomic_load_n(&p[x], __ATOMIC_RELAXED);
    while (q != x) {
        const int r = __atomic_load_n(&p[q], __ATOMIC_RELAXED);
        if (r != q) __atomic_store_n(&p[x], r, __ATOMIC_RELAXED);
        x = q;
        q = r;
    }
    return x;
}

__device__ __forceinline__ void uf_unite(int* p, int a, int b) {
    while (true) {
        a = uf_find(p, a);
        b = uf_find(p, b);
        if (a == b) return;
        if (a < b) {
            const int t = a;
            a = b;
            b = t;
        }
        const int old = atomicMin(&p[a], b);
        if (old == a) return;
        a = old;
    }
}

// Phase 1: union-find inside a 32x32 tile in LDS (no global atomics).  A component's
// local root is its smallest row-major tile index, whose global index is therefore also the
// smallest of its members: parent[i] <= i holds globally, as uf_unite() requires.  The
// local component sizes are counted in LDS and stored at the local roots (size[] is 0
// everywhere else).
constexpr int kCT = 32;
__global__ __launch_bounds__(256) void k_cc_local(const int16_t* img, int H, int W, int pitch, int newv,
                                                  int maxdiff, int* parent, int* size, long long fimg) {
    img += blockIdx.z * fimg;   // map z of a batch; its forest at z*H*W
    parent += (size_t)blockIdx.z * H * W;
    size += (size_t)blockIdx.z * H * W;
    __shared__ int lp[kCT * kCT];
    __shared__ int lc[kCT * kCT];
    __shared__ int16_t lv[kCT * kCT];
    const int x0 = blockIdx.x * kCT, y0 = blockIdx.y * kCT, t = threadIdx.x;
    for (int l = t; l < kCT * kCT; l += 256) {
        const int x = x0 + (l % kCT), y = y0 + l / kCT;
        const bool in = x < W && y < H;
        const int v = in ? img[(size_t)y * pitch + x] : newv;
        lv[l] = (int16_t)v;
        lp[l] = v != newv ? l : -1;
        lc[l] = 0;
    }
    __syncthreads();
    for (int l = t; l < kCT * kCT; l += 256) {
        const int v = lv[l];
        if (v == newv) continue;
        const int lx = l % kCT;
        if (lx + 1 < kCT) {
            const int w = lv[l + 1];
            if (w != newv && abs(w - v) <= maxdiff) uf_unite(lp, l, l + 1);
        }
        if (l + kCT < kCT * kCT) {
            const int w = lv[l + kCT];
            if (w != newv && abs(w - v) <= maxdiff) uf_unite(lp, l, l + kCT);
        }
    }
    __syncthreads();
    int root[kCT * kCT / 256];
#pragma unroll
    for (int u = 0; u < kCT * kCT / 256; ++u) {
        const int l = t + 256 * u;
        root[u] = lp[l] < 0 ? -1 : uf_find(lp, l);
        if (root[u] >= 0) atomicAdd(&lc[root[u]], 1);
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kCT * kCT / 256; ++u) {
        const int l = t + 256 * u;
        const int x = x0 + (l % kCT), y = y0 + l / kCT;
        if (x >= W || y >= H) continue;
        const size_t gi = (size_t)y * W + x;
        const int r = root[u];
        parent[gi] = r < 0 ? -1 : (y0 + r / kCT) * W + x0 + (r % kCT);
        size[gi] = r == l ? lc[l] : 0;
    }
}

// Phase 2: the edges that cross tile borders, united in the global forest.  An edge whose
// two ends both already sit in a tree holding a local component larger than maxsize is
// skipped: both ends end up in components that are not speckles whether or not they are
// joined (parent[p] is always a local root of p's tree, whose size[] is a local size).
// This drops the background's border edges, which otherwise all contend for one root.
__global__ __launch_bounds__(256) void k_cc_border(const int16_t* img, int H, int W, int pitch, int newv,
                                                   int maxdiff, int maxsize, int* parent, const int* size,
                                                   long long fimg) {
    img += blockIdx.z * fimg;
    parent += (size_t)blockIdx.z * H * W;
    size += (size_t)blockIdx.z * H * W;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= H * W) return;
    const int y = i / W, x = i % W;
    const bool right = (x % kCT) == kCT - 1 && x + 1 < W;
    const bool down = (y % kCT) == kCT - 1 && y + 1 < H;
    if (!right && !down) return;
    const int v = img[(size_t)y * pitch + x];
    if (v == newv) return;
    auto big = [&](int p) { return size[__atomic_load_n(&parent[p], __ATOMIC_RELAXED)] > maxsize; };
    const bool bi = big(i);
    if (right) {
        const int w = img[(size_t)y * pitch + x + 1];
        if (w != newv && abs(w - v) <= maxdiff && !(bi && big(i + 1))) uf_unite(parent, i, i + 1);
    }
    if (down) {
        const int w = img[(size_t)(y + 1) * pitch + x];
        if (w != newv && abs(w - v) <= maxdiff && !(bi && big(i + W))) uf_unite(parent, i, i + W);
    }
}

// Component sizes: every local root adds its local size to its tree's root, unless that
// count already exceeds maxsize (the decision size <= maxsize stays exact).  Non-roots
// keep size 0 and the roots' own entries start at their local size.
__global__ __launch_bounds__(256) void k_cc_count(int H, int W, int maxsize, int* parent, int* size) {
    parent += (size_t)blockIdx.z * H * W;
    size += (size_t)blockIdx.z * H * W;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= H * W) return;
    const int s = size[i];
    if (s <= 0) return;
    const int r = uf_find(parent, i);
    if (r != i && __atomic_load_n(&size[r], __ATOMIC_RELAXED) <= maxsize) atomicAdd(&size[r], s);
}

__global__ __launch_bounds__(256) void k_cc_apply(int16_t* img, int H, int W, int pitch, int newv, int maxsize,
                                                  int* parent, const int* size, long long fimg) {
    img += blockIdx.z * fimg;
    parent += (size_t)blockIdx.z * H * W;
    size += (size_t)blockIdx.z * H * W;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= H * W || parent[i] < 0) return;
    if (size[uf_find(parent, i)] <= maxsize) img[(size_t)(i / W) * pitch + i % W] = (int16_t)newv;
}

// Line plans: (lanes per line, disparities per lane).
//  * horizontal paths: 16-lane lines.  One wave per SIMD issues the W-step chain; 32-lane
//    lines (1080 waves at 1080p, some SIMDs holding two) measured 490 vs 471 us.
//  * vertical path and WTA: 32-lane lines for D > 32 (two DPP rows joined by
//    v_permlane16_swap).  The vertical path runs beside the horizontal ones on a second
//    stream; 16-lane lines there measured the same (536 vs 528 us, concurrent).
struct PathPlan {
    int lpc, dpl;
};
PathPlan hpath16_plan(int D) {
    const int need = (D + 15) / 16;
    const int opts[] = {1, 2, 4, 8, 12, 16, 20, 24, 32};
    for (int o : opts)
        if (o >= need) return {16, o};
    return {0, -1};
}
PathPlan vpath_plan(int D) {
    if (D <= 32) return hpath16_plan(D);
    const int need = (D + 31) / 32;
    const int opts[] = {2, 4, 6, 8, 10, 12, 16};
    for (int o : opts)
        if (o >= need) return {32, o};
    return {0, -1};
}

PathPlan hpath_plan(int D) { return hpath16_plan(D); }

template <typename LT>
int launch_paths_t(const SgbmArgs& a, int nf, hipStream_t s, hipStream_t aux, hipEvent_t fork, hipEvent_t join) {
    const bool fused = a.fused != 0;
    // single frames / small batches (unfused): the horizontal lines take the vertical path's
    // 32-lane plan (half the disparities per lane: a shorter dependent chain per step, and
    // twice the waves of the 16-lane plan on a machine the ~540 16-lane waves leave half
    // idle); batches keep 16-lane lines (the fused R->L/WTA kernel is 16-lane).
    // SV_SGBM_H32=0: 16-lane lines for every launch (A/B).
    static const bool h32 = [] {
        const char* e = std::getenv("SV_SGBM_H32");
        return !(e && e[0] == '0');
    }();
    const PathPlan ph = (fused || !h32) ? hpath_plan(a.D) : vpath_plan(a.D), pv = vpath_plan(a.D), pw = pv;
    const dim3 gh((a.H + 64 / ph.lpc - 1) / (64 / ph.lpc), fused ? 1 : 2, nf), gv((a.Wb + 64 / pv.lpc - 1) / (64 / pv.lpc), 1, nf);
    const size_t npx = (size_t)a.H * a.Wb;
    const dim3 gw((unsigned)((npx + 64 / pw.lpc - 1) / (64 / pw.lpc)), 1, nf);
    // unfused launches (SV_SGBM_VWTA=0: A/B): the horizontal paths first, then the vertical
    // path fused with the WTA (L_tb never stored); otherwise the vertical path on the second
    // stream beside the horizontal paths and a separate WTA
    static const bool vwta_on = [] {
        const char* e = std::getenv("SV_SGBM_VWTA");
        return !(e && e[0] == '0');
    }();
    // (D <= 128 measured even: 703 vs 707 frames/s per call at D=128, so the concurrent form
    // stays there; D=320: 337 -> 359 per call, 373 -> 416 at batch 4.  Round 4, with the deep
    // one-wave variant also for D <= 128: 1080p D=128 712 -> 719, VGA D=64 7,160 -> 5,640)
    const bool vwta = !fused && vwta_on && pv.lpc == 32 && a.D > 128;
    // deep: the vertical path + WTA of a launch this small (at most ~1 wave per SIMD: one
    // 1080p frame is ~800 waves) takes the variant with one wave per SIMD and a 3x deeper
    // prefetch ring of its three volumes (Little's law: the bytes in flight set the bandwidth):
    // D=320 w7 952 -> 855-863 us, 362 -> 374 frames/s per call.  Batches keep the 2-wave form
    // (every launch deep: batch 8 459-468 -> 453, batch 4 438 -> 416 frames/s).
    // SV_SGBM_DEEP=0 / 2: the 2-wave / the deep variant everywhere (A/B)
    const char* de = std::getenv("SV_SGBM_DEEP");   // read per call (tests switch it)
    const int deep_mode = de && (de[0] == '0' || de[0] == '2') ? de[0] - '0' : 1;
    const long long vwaves = (long long)gv.x * gv.y * gv.z;
    const bool deep = !fused && (deep_mode == 2 || (deep_mode == 1 && vwaves <= 1280));
    if (vwta) aux = nullptr;
    hipStream_t sv = aux ? aux : s;
    if (aux) {
        if (hipEventRecord(fork, s) != hipSuccess || hipStreamWaitEvent(aux, fork, 0) != hipSuccess)
            return (int)hipErrorLaunchFailure;
    }
    bool v = false, h = false, w = false;
#define SV_VPATH(L, N, PF)                                                           \
    if (!v && pv.lpc == L && pv.dpl == N) {                                          \
        hipLaunchKernelGGL((k_sgbm_vpath<N, L, LT, PF>), gv, dim3(64), 0, sv, a);   \
        v = true;                                                                    \
    }
    if (!vwta) {
        SV_VPATH(16, 1, 16) SV_VPATH(16, 2, 16)
        SV_VPATH(32, 2, 16) SV_VPATH(32, 4, 12) SV_VPATH(32, 6, 10) SV_VPATH(32, 8, 8) SV_VPATH(32, 10, 6)
        SV_VPATH(32, 12, 4) SV_VPATH(32, 16, 3)
    } else {
        v = true;   // launched after the horizontal paths (below)
    }
#undef SV_VPATH
    if (aux && hipEventRecord(join, aux) != hipSuccess) return (int)hipErrorLaunchFailure;
#define SV_HPATH(L, N, PF, WPE)                                                      \
    if (!h && ph.lpc == L && ph.dpl == N) {                                          \
        hipLaunchKernelGGL((k_sgbm_hpath<N, L, LT, PF, WPE>), gh, dim3(64), 0, s, a); \
        h = true;                                                                    \
    }
    if (fused) {   // batches: 2 waves per SIMD
        SV_HPATH(16, 1, 24, 2) SV_HPATH(16, 2, 24, 2) SV_HPATH(16, 4, 16, 2) SV_HPATH(16, 8, 12, 2)
        SV_HPATH(16, 12, 8, 2) SV_HPATH(16, 16, 6, 2) SV_HPATH(16, 20, 4, 2) SV_HPATH(16, 24, 4, 2)
        SV_HPATH(16, 32, 4, 1)
    }
    // (Deeper prefetch did not pay for the horizontal lines of a single D=320 frame: one wave
    // per SIMD with 16 steps ahead 1,105 -> 1,355 us, two waves with 9 steps ahead 1,119 us;
    // round 6, an LDS-DMA ring 11 steps deep (global_load_lds_dwordx4, counted vmcnt, no
    // register ring for the compiler to drain at the loop back-edge): 1,116 -> 1,175 us.  The
    // horizontal paths are bound by their volume traffic, 4.43 GB per D=320 frame at ~3.8-4.0
    // TB/s — DESIGN.md §10.8.)
    SV_HPATH(32, 2, 16, 2) SV_HPATH(32, 4, 12, 2) SV_HPATH(32, 6, 10, 2) SV_HPATH(32, 8, 8, 2)
    SV_HPATH(32, 10, 6, 2) SV_HPATH(32, 12, 4, 2) SV_HPATH(32, 16, 3, 2)
    SV_HPATH(16, 1, 24, 1) SV_HPATH(16, 2, 24, 1) SV_HPATH(16, 4, 16, 1) SV_HPATH(16, 8, 16, 1)
    SV_HPATH(16, 12, 10, 1) SV_HPATH(16, 16, 8, 1) SV_HPATH(16, 20, 6, 1) SV_HPATH(16, 24, 6, 1)
    SV_HPATH(16, 32, 4, 1)
#undef SV_HPATH
    if (aux && hipStreamWaitEvent(s, join, 0) != hipSuccess) return (int)hipErrorLaunchFailure;
    if (vwta) {
#define SV_VWTA(N, PF, WPE)                                                                      \
        if (!w && pv.dpl == N) {                                                                 \
            hipLaunchKernelGGL((k_sgbm_vpath_wta<N, 32, LT, PF, WPE>), gv, dim3(64), 0, s, a);   \
            w = true;                                                                            \
        }
        if (deep) {   // <= ~1 wave per SIMD: the whole register file for a deeper prefetch
            SV_VWTA(6, 8, 1) SV_VWTA(8, 6, 1) SV_VWTA(10, 6, 1) SV_VWTA(12, 4, 1) SV_VWTA(16, 3, 1)
        }
        SV_VWTA(2, 8, 2) SV_VWTA(4, 6, 2) SV_VWTA(6, 4, 2) SV_VWTA(8, 3, 2) SV_VWTA(10, 2, 2) SV_VWTA(12, 2, 2)
        SV_VWTA(16, 1, 2)
#undef SV_VWTA
    }
    if (fused) {
        const dim3 gf((a.H + 3) / 4, 1, nf);
#define SV_RLWTA(N, PF)                                                              \
        if (!w && ph.dpl == N) {                                                     \
            hipLaunchKernelGGL((k_sgbm_rl_wta<N, LT, PF>), gf, dim3(64), 0, s, a);   \
            w = true;                                                                \
        }
        SV_RLWTA(1, 16) SV_RLWTA(2, 16) SV_RLWTA(4, 8) SV_RLWTA(8, 4) SV_RLWTA(12, 3) SV_RLWTA(16, 2)
        SV_RLWTA(20, 3) SV_RLWTA(24, 3) SV_RLWTA(32, 2)
#undef SV_RLWTA
    }
#define SV_WTA(L, N)                                                                 \
    if (!w && pw.lpc == L && pw.dpl == N) {                                          \
        hipLaunchKernelGGL((k_sgbm_wta<N, L, LT>), gw, dim3(64), 0, s, a);           \
        w = true;                                                                    \
    }
    SV_WTA(16, 1) SV_WTA(16, 2) SV_WTA(32, 2) SV_WTA(32, 4) SV_WTA(32, 6) SV_WTA(32, 8) SV_WTA(32, 10)
    SV_WTA(32, 12) SV_WTA(32, 16)
#undef SV_WTA
    if (!v || !h || !w) return (int)hipErrorInvalidValue;
    return (int)hipGetLastError();
}

}  // namespace

bool sgbm_cost_fused(int D, int r) {
    static const bool off = [] {
        const char* e = std::getenv("SV_SGBM_COST");
        return e && e[0] == '0';
    }();
    // r >= 5: the ring no longer fits the registers of 2 waves per SIMD (spills), and the 13/15-
    // row bodies of r 6..7 are too large to unroll
    return !off && D >= 1 && D <= 512 && r <= 4;
}

bool sgbm_fused(int nf, int D) {
    const char* e = std::getenv("SV_SGBM_FUSED");   // read per call (tests switch it)
    const int force = e && (e[0] == '0' || e[0] == '1') ? e[0] - '0' : -1;
    return force >= 0 ? force == 1 : (nf >= 8 && D <= 128);
}

int sgbm_dp(int D) {
    if (D < 1 || D > 512) return -1;
    int x = hpath_plan(D).dpl, y = vpath_plan(D).dpl;   // Dp: a multiple of both lane widths
    int g = x, r = y;
    while (r) {
        const int t = g % r;
        g = r;
        r = t;
    }
    const int l = x / g * y;
    return (D + l - 1) / l * l;
}

int launch_sgbm(const SgbmArgs& a, int nf, hipStream_t s, hipStream_t aux, hipEvent_t fork, hipEvent_t join) {
    if (a.H <= 0 || a.W <= 0 || nf <= 0) return 0;
    if (a.Wb > 0 && sgbm_cost_fused(a.D, a.r)) {
        if (a.r > kMaxR) return (int)hipErrorInvalidValue;
        // pixel cost + window sums in one pass (k_sgbm_cost): one wave per (CL-column chunk,
        // 64 disparities, row band, frame); bands of >= 32 rows (the ring warm-up is 2r+1 rows)
        const int cl = cost_cl(a.r);                        // CostCfg<R>::CL
        const int chunks = (a.Wb + cl - 1) / cl, ndg = (a.D + 63) / 64;
        const long long per_band = (long long)chunks * ndg * nf;
        // ~16k waves (D=320 w7 1080p: 33-row bands; 8k / 4k waves measured 598 / slower us,
        // round 4: the bands' 2r-row warm-up is not what bounds the kernel)
        const int nb = (int)std::max<long long>(1, std::min<long long>(a.H / 32, (16384 + per_band - 1) / per_band));
        const int vb = (a.H + nb - 1) / nb;
        const dim3 grid((unsigned)chunks, (unsigned)(ndg * ((a.H + vb - 1) / vb)), (unsigned)nf);
        hipLaunchKernelGGL(k_sgbm_records, dim3((a.W + 255) / 256, 2 * a.H, nf), dim3(256), 0, s, a);
        switch (a.r) {
#define SV_COST_R(R) case R: hipLaunchKernelGGL(k_sgbm_cost<R>, grid, dim3(64), 0, s, a, vb, ndg); break;
            SV_COST_R(0) SV_COST_R(1) SV_COST_R(2) SV_COST_R(3) SV_COST_R(4)
#undef SV_COST_R
        }
        const int e = a.l32 ? launch_paths_t<int32_t>(a, nf, s, aux, fork, join)
                            : launch_paths_t<int16_t>(a, nf, s, aux, fork, join);
        if (e) return e;
    } else if (a.Wb > 0) {
        if (a.r > kMaxR) return (int)hipErrorInvalidValue;
        const dim3 grid((unsigned)((a.Wb + kHX - 1) / kHX), (unsigned)a.H, (unsigned)nf);
        const size_t lds = (size_t)(2 * kHX + 4 * a.r + a.D - 1) * sizeof(uint4);
        switch (a.r) {
#define SV_HSUM_R(R) case R: hipLaunchKernelGGL(k_sgbm_hsum_tiled<R>, grid, dim3(256), lds, s, a); break;
            SV_HSUM_R(0) SV_HSUM_R(1) SV_HSUM_R(2) SV_HSUM_R(3) SV_HSUM_R(4) SV_HSUM_R(5) SV_HSUM_R(6)
            SV_HSUM_R(7)
#undef SV_HSUM_R
        }
        const size_t plane = (size_t)a.Wb * a.Dp;
        if (plane % 8 == 0 && ((uintptr_t)a.hsum & 15) == 0 && ((uintptr_t)a.C & 15) == 0) {
            // enough bands for ~4 waves per SIMD (4 waves per block), each >= 64 rows so the
            // per-band warm-up of 2r+1 rows stays small
            const size_t blocks = (plane / 8 + 255) / 256;
            const int nb = (int)std::max<size_t>(1, std::min<size_t>((size_t)a.H / 64, (1024 + blocks * nf - 1) / (blocks * nf)));
            const int vb = (a.H + nb - 1) / nb;
            const dim3 grid8((unsigned)blocks, (unsigned)((a.H + vb - 1) / vb), (unsigned)nf);
            switch (a.r) {
#define SV_VSUM_R(R) case R: hipLaunchKernelGGL(k_sgbm_vsum8<R>, grid8, dim3(256), 0, s, a, vb); break;
                SV_VSUM_R(0) SV_VSUM_R(1) SV_VSUM_R(2) SV_VSUM_R(3) SV_VSUM_R(4) SV_VSUM_R(5) SV_VSUM_R(6)
                SV_VSUM_R(7)
#undef SV_VSUM_R
            }
        } else {
            hipLaunchKernelGGL(k_sgbm_vsum, dim3((unsigned)((plane + 255) / 256), 1, (unsigned)nf), dim3(256), 0, s, a);
        }
        const int e = a.l32 ? launch_paths_t<int32_t>(a, nf, s, aux, fork, join)
                            : launch_paths_t<int16_t>(a, nf, s, aux, fork, join);
        if (e) return e;
    }
    hipLaunchKernelGGL(k_sgbm_lrcheck, dim3(a.H, 1, nf), dim3(256), (size_t)a.W * 8, s, a);
    return (int)hipGetLastError();
}

int launch_speckles(int16_t* img, int H, int W, int pitch, int newv, int maxsize, int maxdiff, int* parent,
                    int* size, hipStream_t s, int nf, long long fimg) {
    if (H <= 0 || W <= 0 || maxsize <= 0 || nf <= 0) return 0;
    const dim3 n((unsigned)(((size_t)H * W + 255) / 256), 1, (unsigned)nf);
    dim3 tiles((W + kCT - 1) / kCT, (H + kCT - 1) / kCT, (unsigned)nf);
    hipLaunchKernelGGL(k_cc_local, tiles, dim3(256), 0, s, img, H, W, pitch, newv, maxdiff, parent, size, fimg);
    hipLaunchKernelGGL(k_cc_border, n, dim3(256), 0, s, img, H, W, pitch, newv, maxdiff, maxsize, parent,
                       size, fimg);
    hipLaunchKernelGGL(k_cc_count, n, dim3(256), 0, s, H, W, maxsize, parent, size);
    hipLaunchKernelGGL(k_cc_apply, n, dim3(256), 0, s, img, H, W, pitch, newv, maxsize, parent, size, fimg);
    return (int)hipGetLastError();
}

}  // namespace sv
