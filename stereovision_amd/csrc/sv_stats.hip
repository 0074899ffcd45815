// sv_stats.hip — reductions on either side of the disparity path.
//
//  * k_frame_stats   the image statistics behind detect_camera_occlusion
//                    (fused_depth_map.py:131-301, run every OCCLUSION_CHECK_INTERVAL frames on
//                    the rectified pair, :2515-2522): per 48x48 block the exact integer
//                    moments (sum, sum of squares) that np.std(block) is built from, and the
//                    256-bin histogram (cv2.calcHist) whose moments also give the global
//                    np.mean / np.std.  BGR input is converted to gray on the fly (cvtColor).
//  * k_select_hist   one pass of a radix select over float32 keys: the order statistics
//                    np.percentile interpolates between (calibrate_midas_to_stereo
//                    fused_depth_map.py:1169-1257, normalize_to_stereo_range :1503-1554),
//                    with the reference's boolean masks (x > 0, confidence > 0.7) applied
//                    as predicates, so the masked array is never materialised.
//  * k_affine_f32    the elementwise epilogues of those functions, in NumPy's precision
//                    (float32 ops in order, or float64 scale/offset then astype(float32)).
// All HBM-bound: one read of the image / map per pass.
#include "sv_internal.h"

namespace sv {
namespace {

constexpr int kTile = 48;   // compute_block_homogeneity block_size (fused_depth_map.py:185)

// Wave64 sum of a 32-bit value (xor butterfly through DPP/permute).
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// LDS histogram increment with wave aggregation: when every active lane of the wave adds
// to the same bin (flat image regions, or the constant high digits of a radix pass: the
// common case) one atomic adds the population; otherwise each lane adds 1.
__device__ __forceinline__ void hist_add(uint32_t* h, uint32_t bin) {
    const uint32_t b0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)bin);
    const unsigned long long act = __ballot(1);
    const unsigned long long same = __ballot(bin == b0);
    if (same == act) {
        if (__lane_id() == (unsigned)__builtin_ctzll(act)) atomicAdd(&h[b0], (uint32_t)__builtin_popcountll(act));
    } else {
        atomicAdd(&h[bin], 1u);
    }
}

// One workgroup (256 threads) per 48x48 tile of one image (grid.z = image).  A thread owns
// one (row, 4-pixel group) of the tile per iteration (48 rows x 12 groups), gray rows read
// as dwords (48 is a multiple of 4: a group never straddles two tiles); one LDS histogram
// copy per wave.
__global__ __launch_bounds__(256) void k_frame_stats(FrameStatsArgs a) {
    __shared__ uint32_t hist[4][256];
    __shared__ uint32_t part[2][4];
    const int z = blockIdx.z;
    const uint8_t* img = z == 0 ? a.img0 : a.img1;
    const int tx = blockIdx.x, ty = blockIdx.y, t = threadIdx.x, wv = t >> 6;
    for (int i = t; i < 4 * 256; i += 256) (&hist[0][0])[i] = 0;
    __syncthreads();
    const int x0 = tx * kTile, y0 = ty * kTile;
    const int w = min(kTile, a.W - x0), h = min(kTile, a.H - y0);
    const int groups = (w + 3) >> 2;
    uint32_t s = 0, q = 0;
    for (int i = t; i < h * groups; i += 256) {
        const int r = i / groups, g = i - r * groups;
        const int x = x0 + 4 * g, n = min(4, w - 4 * g);
        const uint8_t* p = img + (size_t)(y0 + r) * a.pitch + (size_t)x * a.cn;
        uint32_t v4[4];
        if (a.cn == 1 && n == 4 && (((uintptr_t)p & 3) == 0)) {
            const uint32_t d = *reinterpret_cast<const uint32_t*>(p);
            v4[0] = d & 0xff;
            v4[1] = (d >> 8) & 0xff;
            v4[2] = (d >> 16) & 0xff;
            v4[3] = d >> 24;
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint8_t* pk = p + k * a.cn;
                v4[k] = k >= n ? 0u
                        : a.cn == 3 ? (uint32_t)((pk[0] * 1868 + pk[1] * 9617 + pk[2] * 4899 + (1 << 13)) >> 14)
                                    : (uint32_t)pk[0];
            }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (k < n) {
                s += v4[k];
                q += v4[k] * v4[k];
            }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (k < n) hist_add(hist[wv], v4[k]);
    }
    s = wave_sum(s);
    q = wave_sum(q);
    if ((t & 63) == 0) {
        part[0][t >> 6] = s;
        part[1][t >> 6] = q;
    }
    __syncthreads();
    if (t == 0 && tx < a.bw && ty < a.bh) {   // a block of compute_block_homogeneity
        const int b = z * a.bh * a.bw + ty * a.bw + tx;
        a.block_sum[b] = part[0][0] + part[0][1] + part[0][2] + part[0][3];
        a.block_sq[b] = part[1][0] + part[1][1] + part[1][2] + part[1][3];
    }
    const uint32_t c = hist[0][t] + hist[1][t] + hist[2][t] + hist[3][t];
    if (c) atomicAdd(&a.hist[z * 256 + t], c);
}

// Order-preserving map of float32 bits to uint32 (-0.0 folded onto +0.0, NaN excluded by
// the caller's predicate and counted separately).
__device__ __forceinline__ uint32_t f32_key(float f) {
    uint32_t u = __float_as_uint(f);
    if (u == 0x80000000u) u = 0;
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// Pass `shift` of the select: histogram of digit (key >> shift) & (nbins-1) over the
// selected elements whose key agrees with prefix[r] above the digit, for each rank r.
// Pass 0 (shift = 21, all prefixes empty) also counts selected elements and NaNs.
__global__ __launch_bounds__(256) void k_select_hist(SelectArgs a) {
    __shared__ uint32_t h[kMaxRanks][2048];
    const int nb = 1 << a.bits;
    for (int r = 0; r < a.nranks; ++r)
        for (int i = threadIdx.x; i < nb; i += 256) h[r][i] = 0;
    __syncthreads();
    uint32_t cnt = 0, nan = 0;
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < a.n; i += stride) {
        if (a.mask_mode == SEL_MASK_GT && !(a.mask[i] > a.thr)) continue;   // confidence > 0.7
        const float v = a.x[i];
        if (v != v) {                        // NaN in the selection: np.percentile -> nan
            nan += a.mask_mode != SEL_POSITIVE;
            continue;
        }
        if (a.mask_mode == SEL_POSITIVE && !(v > 0.f)) continue;            // disparity > 0
        ++cnt;
        const uint32_t k = f32_key(v);
        const uint32_t d = (k >> a.shift) & (uint32_t)(nb - 1);
        const uint32_t hi = a.shift + a.bits >= 32 ? 0u : (k >> (a.shift + a.bits));
        for (int r = 0; r < a.nranks; ++r)
            if (hi == a.prefix[r]) hist_add(h[r], d);
    }
    __syncthreads();
    for (int r = 0; r < a.nranks; ++r)
        for (int i = threadIdx.x; i < nb; i += 256)
            if (h[r][i]) atomicAdd(&a.ghist[r * 2048 + i], h[r][i]);
    if (a.counts) {
        cnt = wave_sum(cnt);
        nan = wave_sum(nan);
        if ((threadIdx.x & 63) == 0) {
            atomicAdd(&a.counts[0], (unsigned long long)cnt);
            atomicAdd(&a.counts[1], (unsigned long long)nan);
        }
    }
}

__global__ __launch_bounds__(256) void k_affine_f32(AffineArgs a) {
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < a.n; i += stride) {
        const float x = a.x[i];
        float y;
        if (a.mode == AFF_F32) {          // c + ((x - a) / b) * d, float32, in this order
            const float nrm = (x - a.fa) / a.fb;
            y = a.fc + nrm * a.fd;
        } else if (a.mode == AFF_F64) {   // astype(float32) of (float64(x) * s + o)
            y = (float)((double)x * a.ds + a.doff);
        } else {                          // np.full_like(x, c)
            y = a.fc;
        }
        a.out[i] = y;
    }
}

}  // namespace

int launch_frame_stats(const FrameStatsArgs& a, int nimg, hipStream_t s) {
    if (a.H <= 0 || a.W <= 0 || nimg <= 0) return 0;
    dim3 grid((a.W + kTile - 1) / kTile, (a.H + kTile - 1) / kTile, nimg);
    hipLaunchKernelGGL(k_frame_stats, grid, dim3(256), 0, s, a);
    return (int)hipGetLastError();
}

int launch_select_hist(const SelectArgs& a, hipStream_t s) {
    if (a.n == 0) return 0;
    // ~16 elements per thread: each block zeroes and merges a 2048-bin histogram per rank
    int blocks = (int)((a.n + 4095) / 4096);
    if (blocks > 1024) blocks = 1024;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(k_select_hist, dim3(blocks), dim3(256), 0, s, a);
    return (int)hipGetLastError();
}

int launch_affine_f32(const AffineArgs& a, hipStream_t s) {
    if (a.n == 0) return 0;
    int blocks = (int)((a.n + 255) / 256);
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(k_affine_f32, dim3(blocks), dim3(256), 0, s, a);
    return (int)hipGetLastError();
}

}  // namespace sv
