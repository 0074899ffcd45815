// sv_ssd_mfma.hip — the SSD cost volume on the matrix cores (gfx950 v_mfma_i32_32x32x32_i8).
//
// Replaces stereo.compute (depth_map.py:909, fused_depth_map.py:1004) for the SSD cost of the
// north_star engine: d* = first argmin over d of C(x,y,d) = sum over the win x win window of
// (Lp(x+i, y+j) - Rp(x+i-d, y+j))^2 (replicate-clamped images, oracle/sv_oracle.py
// disparity16).  With L' = L - 128, R' = R - 128 (exact, the differences do not change):
//
//     C = SL2(x) + SR2(x') - 2 X(x, x'),   x' = x - d,
//     SL2 = sum L'^2, SR2 = sum R'^2 over the window, X = sum L'(x+i,y+j) R'(x'+i,y+j).
//
// For a fixed x, SL2(x) is a constant, so the argmin (and its first-min tie break) is that of
// SR2(x') - 2 X(x, x').  X is an int8 correlation: for one image row it is the product of a
// [x' rows] x [16 horizontal taps] R' matrix and a [16 taps] x [x columns] L' matrix (taps
// i >= win zero on the L side) — a banded GEMM, on the MFMA.
//
// Kernel shape (one 256-thread block = 4 waves, a band of output rows, 128 XT columns):
//   * MFMA A = R' rows (M = 32 x' values), B = L' columns (N = 32 x values), K = 32 =
//     [16 taps of the row entering the vertical window | 16 taps of the row leaving it].  The
//     32x32 accumulator of every (x-tile, x'-tile) pair PERSISTS across the band's rows: each
//     row adds the entering row's products and removes the leaving row's, so the window's
//     vertical sum costs one MFMA per tile pair and row whatever the window height.
//     The accumulator holds -X: the entering row's A bytes are ~R' = -R' - 1 (the MFMA adds
//     -X_enter - sum_i L'(x - r + i, y_enter)) and the leaving row's are R' (it adds X_leave),
//     so no negated int8 operand is needed (-(-128) does not exist); the extra term depends on
//     the COLUMN x only (one lane), i.e. it shifts every key of that x by the same multiple of
//     2M — neither the argmin nor its index bits change (ranges checked by the launcher).
//   * epilogue per cell (lane = x column, 16 registers = x' rows):
//       key = U(x') + 2M * acc = U(x') - 2M * X - 2M * Cor(x)   (one v_lshl_add_u32)
//       U(x') = M * (SR2(x') - bias) - ix'   (per row, built once per x' by the block, in LDS)
//     so key = M * (val - bias) + d + c_x: for one x, the order of the keys is the order of
//     (cost, d) — the oracle's first minimum — and d - minD = (key + ix + D - 1) & (M - 1).
//     best = v_min3(best, key, key) over the x'-tiles; the first and the last x'-tile of an
//     x-tile hold complementary triangles of valid d (D % 32 == 0), so their keys are merged
//     with one v_cndmask per cell by a lane-constant mask (row >= column) before the min.
//   * SR2: per staged row the block computes hsq(x') = sum_{i<win} R'(x'-r+i)^2 (4 v_dot4 on the
//     masked 16 bytes) once; the per-column running vertical sum adds the entering row's and
//     subtracts the leaving row's.
//   * staging: every step one LDS-DMA per thread (global_load_lds_dword) lands the raw dwords of
//     the row entering PRE = 5 steps later in a ring of win + 5 raw rows, retired by a counted
//     s_waitcnt vmcnt(3) two steps before use — no global load result ever sits in a VGPR, the
//     row loop has one barrier per step (lgkmcnt + s_barrier only) and no global latency.
//     From the raw ring each step builds 4 byte-shifted copies of its entering (L', ~R') and
//     leaving (L', R') rows, so every 16-byte operand at any byte offset is 4 aligned
//     ds_read_b32 (an unaligned ds_read_b128 costs ~7x: tools/microbench/lds_unaligned).
//   * the hsq ring (win + 2 rows) and U (double-buffered) live in LDS beside them.
//   * D <= 160 (<= 6 x'-tiles: the accumulators fit in the 256 VGPRs beside the operands); the
//     4-byte alignment of the images is checked by the launcher (ssd_mfma_fits).
#include "sv_internal.h"

namespace sv {
namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr int kWaves = 4;
constexpr int kThreads = 64 * kWaves;


// v_min3_u32 as written (the compiler re-associates min(min(a, b), c) chains into v_min pairs)
__device__ __forceinline__ uint32_t min3u(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t d;
    asm("v_min3_u32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}

// Reduce-scatter of 8 keys over the 16 lanes of a row: on return lanes 2j and 2j+1 hold the
// min over the row of key j = (l >> 1) & 7 in v[0] (bank-masked DPP for lane bits 3 and 2, a
// select for bit 1, then one step with lane l ^ 1: 16 ops for 8 keys; sv_match.hip's form).
__device__ __forceinline__ void reduce_scatter8(uint32_t (&v)[8], int l) {
#define SV_BM_PAIR(A, B, CTRL, M0, M1)                                                          \
    "v_min_u32_dpp %" #A ", %" #A ", %" #A " " CTRL " row_mask:0xf bank_mask:" M0 "\n\t"      \
    "v_min_u32_dpp %" #A ", %" #B ", %" #B " " CTRL " row_mask:0xf bank_mask:" M1 "\n\t"
    asm volatile("s_nop 1\n\t"
                 SV_BM_PAIR(0, 4, "row_mirror", "0x3", "0xc") SV_BM_PAIR(1, 5, "row_mirror", "0x3", "0xc")
                 SV_BM_PAIR(2, 6, "row_mirror", "0x3", "0xc") SV_BM_PAIR(3, 7, "row_mirror", "0x3", "0xc")
                 : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3])
                 : "v"(v[4]), "v"(v[5]), "v"(v[6]), "v"(v[7]));
    asm volatile("s_nop 1\n\t"
                 SV_BM_PAIR(0, 2, "row_half_mirror", "0x5", "0xa") SV_BM_PAIR(1, 3, "row_half_mirror", "0x5", "0xa")
                 : "+v"(v[0]), "+v"(v[1])
                 : "v"(v[2]), "v"(v[3]));
#undef SV_BM_PAIR
    const bool hi = (l & 2) != 0;
    const uint32_t send = hi ? v[0] : v[1];
    const uint32_t keep = hi ? v[1] : v[0];
    v[0] = min(keep, (uint32_t)__builtin_amdgcn_update_dpp(0u, (int)send, 0x1B, 0xF, 0xF, false));  // l ^ 3
    v[0] = min(v[0], (uint32_t)__builtin_amdgcn_update_dpp(0u, (int)v[0], 0xB1, 0xF, 0xF, false));  // l ^ 1
}

// A staged image row lives in LDS as 4 copies shifted by 0..3 bytes (copy s, dword w = bytes
// 4w + s .. 4w + s + 3 of the row), so the 16 bytes at ANY byte offset p are 4 dword-aligned
// ds_read_b32 of copy p & 3: a 16-byte LDS load that is not 16-byte aligned costs ~68 LDS cycles
// per wave-instruction against ~9.5 aligned (tools/microbench/lds_unaligned).  Copies are
// 8 dwords (mod 32 banks) apart, so the 32 lanes of a group (8 dwords x 4 copies) never
// conflict.
template <int BYTES>
struct Copies {
    static constexpr int DW = ((BYTES + 4) / 4 + 31 - 8) / 32 * 32 + 8;   // dwords per copy, = 8 (mod 32)
    static constexpr int SIZE = 4 * 4 * DW;                               // bytes, 4 copies
    static_assert(DW * 4 >= BYTES + 4 && DW % 32 == 8, "copy stride");
};

// Block barrier for LDS hand-offs only: __syncthreads() is a workgroup release fence, which
// also waits for every outstanding GLOBAL load and store (s_waitcnt vmcnt(0)) — the next rows'
// prefetch and the previous row's output stores would then be waited on at every row step.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ v4i ld16c(const uint32_t* copies, int dw, int p) {
    const uint32_t* q = copies + (p & 3) * dw + (p >> 2);
    return v4i{(int)q[0], (int)q[1], (int)q[2], (int)q[3]};
}

template <int XT, int NT, int MB>
struct SsdCfg {
    static constexpr int M = 1 << MB;
    static constexpr int XW = 32 * XT * kWaves;        // output columns per block
    static constexpr int GT = kWaves * XT + NT - 1;    // x'-tiles per block
    static constexpr int XPW = 32 * GT;                // x' columns per block (ix' in [0, XPW))
    static constexpr int LB = XW + 16;                 // L' bytes a row's operands read
    static constexpr int RB = XPW + 16;                // R' bytes
    using CL = Copies<LB>;
    using CR = Copies<RB>;
    static constexpr int SLOT = CL::SIZE + CR::SIZE;   // one staged row: L' copies | R' (or ~R') copies
    // physical dwords of a row the operands read: starts up to XW - 1 (XPW - 1) plus the 4-byte
    // alignment offset, 4 dwords each
    static constexpr int NLD = LB / 4 + 1;
    static constexpr int NRD = RB / 4 + 1;
    static_assert(NLD <= CL::DW && NRD <= CR::DW, "copies hold every dword the operands read");
    // 3 entering + 3 leaving slots (a fast wave stages step s + 2 while a slow one reads step s),
    // the hsq ring (win + 2 rows of XPW ints) and U[2][XPW]
    // raw ring (LDS-DMA landing rows): one dword per thread, NLD L dwords then NRD R dwords
    static constexpr int NIT = NLD + NRD;
    static_assert(NIT <= kThreads, "one raw dword per thread");
    static constexpr int RAWB = 4 * kThreads;
    static constexpr int PRE = 5;                      // DMA issue distance (steps)
    static constexpr int lds(int win) { return 6 * SLOT + (win + 2) * 4 * XPW + 2 * 4 * XPW + (win + PRE) * RAWB; }
    static_assert(XT * NT * 16 <= 160, "accumulators must stay in arch VGPRs");
    static_assert(XPW <= 3 * kThreads, "three x' columns per thread at most");
    static_assert(6 * SLOT + 19 * 4 * XPW + (15 + PRE) * RAWB <= 160 * 1024, "LDS per block (win 15)");
};

// The raw rows arrive by LDS-DMA (global_load_lds_dword: wave-uniform LDS base + 4 x lane), one
// dword per thread: the 4-byte aligned dword of columns c0 .. c0 + 3 (c0 % 4 == 0) clamped into
// the row, ca = clamp(c0, 0, (W - 1) & ~3).  Columns outside [0, W) replicate the edge pixel
// (the oracle's replicate border): for blocks whose streams cross an image edge the copy builder
// re-selects the bytes with one v_perm (selector below); interior blocks skip it.
__device__ __forceinline__ int clamp_dword(int c0, int W) { return min(max(c0, 0), (W - 1) & ~3); }
__device__ __forceinline__ uint32_t edge_fix(uint32_t v, int c0, int W) {
    const int ca = clamp_dword(c0, W);
    uint32_t sel = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) sel |= (uint32_t)(min(max(c0 + b, 0), W - 1) - ca) << (8 * b);
    return __builtin_amdgcn_perm(v, v, sel);
}

// SSD matrix-core kernel, MFMA A = L' (rows: 32 x of an x-tile), B = R' (columns: 32 x' of an
// x'-tile), so a lane holds ONE x' column (its key term U(x') is one register) and 16 x rows.
// waves per SIMD the register allocation targets: 3 up to 4 accumulator tiles (64 VGPRs), else 2
template <int XT, int NT> struct SsdOcc {
    static constexpr int W = XT * NT <= 4 ? 3 : 2;
};

template <int XT, int NT, int MB>
__global__ __launch_bounds__(kThreads, (SsdOcc<XT, NT>::W)) void k_ssd_mfma(MatchParams a, int hb, int bias, int dbg) {
    using C = SsdCfg<XT, NT, MB>;
    constexpr int M = C::M;
    constexpr int DWL = C::CL::DW, DWR = C::CR::DW;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int z = blockIdx.z;
    const uint8_t* Limg = a.L + z * a.fs_in;
    const uint8_t* Rimg = a.R + z * a.fs_in;
    int16_t* out = a.out + z * a.fs_out;
    const int W = a.W, H = a.H, r = a.r, win = a.win, D = a.D;
    const int xw = a.X0 + blockIdx.x * C::XW;               // first output column of the block
    const int xpb = xw - (a.minD + D - 1);                  // x' of ix' = 0
    const int y0 = a.row0 + blockIdx.y * hb;
    const int y1 = min(a.row1, y0 + hb);
    if (y0 >= y1) return;
    const int hr = win + 2;                                 // hsq ring rows
    // physical row streams start 4-byte aligned: logical byte b of the L' stream (column
    // xw - r + b) is physical byte b + oL
    const int aL = (xw - r) & ~3, oL = (xw - r) - aL;
    const int aR = (xpb - r) & ~3, oR = (xpb - r) - aR;
    auto slot = [&](int side, int k) { return smem + (side * 3 + k) * C::SLOT; };   // side 0 enter, 1 leave
    int32_t* hsq = reinterpret_cast<int32_t*>(smem + 6 * C::SLOT);          // [hr][XPW]
    uint32_t* Ub = reinterpret_cast<uint32_t*>(smem + 6 * C::SLOT + hr * 4 * C::XPW);   // [2][XPW]

    // ---- staging.  Raw rows: the entering row of step k (L' stream dwords, then R') lands in raw
    // ring row k % rawr by LDS-DMA issued PRE steps ahead (always one per step and thread, so
    // the counted wait below is exact: rows past the band reload the clamped last row into a
    // ring row no build reads again).  Copies: phase A of step s builds step s + 1's entering
    // slot (raw row s + 1: L' and ~R') and leaving slot (raw row s + 1 - win: L' and R').
    constexpr int PRE = C::PRE;
    const int rawr = win + PRE;
    uint32_t* raw = reinterpret_cast<uint32_t*>(Ub + 2 * C::XPW);   // [rawr][kThreads]
    const bool isLq = tid < C::NLD;
    const int c0q = isLq ? aL + 4 * tid : aR + 4 * (tid - C::NLD);   // this thread's raw dword
    const uint8_t* gq = (isLq ? Limg : Rimg) + clamp_dword(c0q, W);
    const bool edge = aL < 0 || aR < 0 || aL + 4 * C::NLD > W || aR + 4 * C::NRD > W;
    auto issue_raw = [&](int k, int rk) {   // rk = k % rawr
        const int y = min(max(y0 - r + k, 0), H - 1);
        typedef __attribute__((address_space(1))) void gvoid;
        typedef __attribute__((address_space(3))) void lvoid;
        __builtin_amdgcn_global_load_lds((gvoid*)(gq + (size_t)y * a.pitch), (lvoid*)(raw + rk * kThreads + wave * 64),
                                         4, 0, 0);
    };
    // copies of step k into slot ks (= k % 3): side 0 = raw row k (ring row r0 = k % rawr: L',
    // ~R'), side 1 = raw row k - win (ring row r1: L', R').  All ring indices are block-uniform
    // and advance incrementally (a runtime modulo is a VALU reciprocal chain plus readfirstlane)
    auto build = [&](int k, int ks, int r0, int r1) {
        const int sides = k >= win ? 2 : 1;
        const uint32_t* p0 = raw + r0 * kThreads;
        const uint32_t* p1 = raw + r1 * kThreads;
#pragma unroll
        for (int u = 0; u < (2 * C::NIT + kThreads - 1) / kThreads; ++u) {
            const int q = tid + u * kThreads;
            if (q >= sides * C::NIT) break;
            const int side = q < C::NIT ? 0 : 1;
            const int rq = side ? q - C::NIT : q;
            const uint32_t* p = side ? p1 : p0;
            const bool isL = rq < C::NLD;
            const int w = isL ? rq : rq - C::NLD;
            const bool more = isL ? (w + 1 < C::NLD) : (w + 1 < C::NRD);
            uint32_t lo = p[rq];
            uint32_t hi = more ? p[rq + 1] : lo;
            if (edge) {   // block-uniform
                const int c0 = (isL ? aL : aR) + 4 * w;
                lo = edge_fix(lo, c0, W);
                hi = edge_fix(hi, c0 + 4, W);
            }
            // L' = L ^ 0x80 both sides; R side: ~R' = R ^ 0x7f entering, R' = R ^ 0x80 leaving
            const uint32_t x = (isL || side) ? 0x80808080u : 0x7F7F7F7Fu;
            lo ^= x;
            hi ^= x;
            uint32_t* base = reinterpret_cast<uint32_t*>(slot(side, ks) + (isL ? 0 : C::CL::SIZE));
            const int dw = isL ? DWL : DWR;
#pragma unroll
            for (int sh = 0; sh < 4; ++sh) base[sh * dw + w] = __builtin_amdgcn_alignbyte(hi, lo, sh);
        }
    };
    // the taps i >= win are zero on the L side (A operand) and in the hsq sums
    v4i wmask;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int nb = min(max(win - 4 * q, 0), 4);
        wmask[q] = nb >= 4 ? -1 : (int)((1u << (8 * nb)) - 1u);
    }

    int sr2[3] = {0, 0, 0};
    v16i acc[XT][NT];
#pragma unroll
    for (int k = 0; k < XT; ++k)
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int q = 0; q < 16; ++q) acc[k][t][q] = 0;
    const int h = lane >> 5, j = lane & 31;
    // lane-constant selection of the edge tiles: cell (x row i, x' column j) of x'-tile 0 is a
    // valid disparity iff j >= i, of x'-tile NT-1 iff j < i (D % 32 == 0)
    bool sel0[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) sel0[q] = j >= ((q & 3) + 8 * (q >> 2) + 4 * h);

    const int nsteps = (y1 - y0) + win - 1;
    // the DMA of raw row k is issued at step k - PRE (the prologue issues rows 0 .. PRE - 1) and
    // retired by the counted wait of step k - 2, whose barrier precedes build(k) in step k - 1:
    // PRE - 2 younger DMAs per thread may stay in flight (the epilogue's stores, also counted,
    // only make the wait stricter)
    static_assert(PRE == 5, "vmcnt immediate below");
#pragma unroll
    for (int k = 0; k < PRE; ++k) issue_raw(k, k);
    asm volatile("s_waitcnt vmcnt(3)" ::: "memory");   // rows 0 and 1
    lds_barrier();
    build(0, 0, 0, 0);
    lds_barrier();
    auto inc = [](int v, int n) { return v + 1 == n ? 0 : v + 1; };
    // s % 3, s % hr, (s + 2) % hr (= the leaving hsq row, hr = win + 2), (s + PRE) % rawr,
    // (s + 1) % rawr, (s + 1 + PRE) % rawr (= raw row s + 1 - win)
    int si = 0, he = 0, hl = 2 % hr, rp = PRE, rb = 1 % rawr, rbl = (1 + PRE) % rawr;
    for (int s = 0; s < nsteps;
         ++s, si = inc(si, 3), he = inc(he, hr), hl = inc(hl, hr), rp = inc(rp, rawr), rb = inc(rb, rawr),
         rbl = inc(rbl, rawr)) {
        const bool leave = s >= win;
        issue_raw(s + PRE, rp);
        // ---- phase A: hsq of the entering row, SR2, U; stage the next step's rows ------------
        {
            const uint32_t* er = reinterpret_cast<const uint32_t*>(slot(0, si) + C::CL::SIZE);   // ~R'
            int32_t* hs_e = hsq + he * C::XPW;
            const int32_t* hs_l = hsq + hl * C::XPW;
            uint32_t* U = Ub + (s & 1) * C::XPW;
#pragma unroll
            for (int jj = 0; jj < 3; ++jj) {
                const int ix = tid + jj * kThreads;
                if (ix < C::XPW) {
                    const v4i v = ld16c(er, DWR, ix + oR);
                    int hs = 0;
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int m = ~v[q] & wmask[q];   // R' = ~(~R')
                        hs = __builtin_amdgcn_sdot4(m, m, hs, false);
                    }
                    hs_e[ix] = hs;
                    sr2[jj] += hs - (leave ? hs_l[ix] : 0);
                    // unsigned keys: + 2^31 makes the signed order the unsigned one
                    U[ix] = (uint32_t)((sr2[jj] - bias) * M - ix) + 0x80000000u;
                }
            }
            if (s + 1 < nsteps) build(s + 1, inc(si, 3), rb, rbl);
        }
        asm volatile("s_waitcnt vmcnt(3)" ::: "memory");   // raw row s + 2 (issued at step s - 3)
        lds_barrier();
        // ---- phase B: one MFMA per (x-tile, x'-tile) pair --------------------------------------
        const uint8_t* se = slot(0, si);
        const uint8_t* sl = slot(1, si);
        v4i aop[XT];
#pragma unroll
        for (int k = 0; k < XT; ++k) {
            const int c = 32 * (wave * XT + k) + j;   // A row = x column xw + c
            if (h == 0) aop[k] = ld16c(reinterpret_cast<const uint32_t*>(se), DWL, c + oL) & wmask;
            else if (leave) aop[k] = ld16c(reinterpret_cast<const uint32_t*>(sl), DWL, c + oL) & wmask;
            else aop[k] = v4i{0, 0, 0, 0};   // warm-up: the leaving half contributes nothing
        }
#pragma unroll
        for (int gi = 0; gi < XT + NT - 1; ++gi) {
            const int ix = 32 * (wave * XT + gi) + j;   // B column = x' of ix
            // entering half ~R' (= -R' - 1), leaving half R': the accumulator holds -X - Cor(x)
            const v4i bop = ld16c(reinterpret_cast<const uint32_t*>((h == 0 ? se : sl) + C::CL::SIZE), DWR, ix + oR);
#pragma unroll
            for (int k = 0; k < XT; ++k) {
                const int t = gi - k;
                if (t >= 0 && t < NT && !(dbg & 1)) acc[k][t] = __builtin_amdgcn_mfma_i32_32x32x32_i8(aop[k], bop, acc[k][t], 0, 0, 0);
                if (t >= 0 && t < NT && (dbg & 1)) acc[k][t][0] ^= aop[k][0] ^ bop[1];
            }
        }
        if (s < win - 1) continue;   // the window of the first output row is not complete yet
        if (dbg & 2) {               // A/B timing: no epilogue
            if (h == 0 && (acc[0][0][0] == 0x7fffffff)) out[0] = 1;
            continue;
        }
        const int y = y0 + s - (win - 1);
        const uint32_t* U = Ub + (s & 1) * C::XPW;
        uint32_t T[XT + NT - 1];
#pragma unroll
        for (int gi = 0; gi < XT + NT - 1; ++gi) T[gi] = U[32 * (wave * XT + gi) + j];
        // ---- keys: key = U(x') + 2M * acc, the running minimum over the x'-tiles per x row ----
#pragma unroll
        for (int k = 0; k < XT; ++k) {
            uint32_t best[16], ka[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) {   // the edge pair: complementary triangles
                const uint32_t e0 = ((uint32_t)acc[k][0][q] << (MB + 1)) + T[k];
                const uint32_t e1 = ((uint32_t)acc[k][NT - 1][q] << (MB + 1)) + T[k + NT - 1];
                best[q] = sel0[q] ? e0 : e1;
            }
#pragma unroll
            for (int t = 1; t < NT - 1; t += 2) {
                if (t + 1 < NT - 1) {
#pragma unroll
                    for (int q = 0; q < 16; ++q)
                        best[q] = min3u(best[q], ((uint32_t)acc[k][t][q] << (MB + 1)) + T[k + t],
                                        ((uint32_t)acc[k][t + 1][q] << (MB + 1)) + T[k + t + 1]);
                } else {
#pragma unroll
                    for (int q = 0; q < 16; ++q) best[q] = min(best[q], ((uint32_t)acc[k][t][q] << (MB + 1)) + T[k + t]);
                }
            }
            // min over the 32 x' columns (lanes) of each half, per x row (register): the
            // 16-lane rows first (permlane16_swap pairs registers), then a reduce-scatter
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const auto p = __builtin_amdgcn_permlane16_swap(best[2 * q], best[2 * q + 1], false, false);
                ka[q] = min((uint32_t)p[0], (uint32_t)p[1]);
            }
            uint32_t v8[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) v8[q] = ka[q];
            reduce_scatter8(v8, lane & 15);
            // lanes 2m, 2m+1 of 16-lane row rho hold x row reg = 2m + rho
            const int reg = 2 * ((lane >> 1) & 7) + ((lane >> 4) & 1);
            const int i = (reg & 3) + 8 * (reg >> 2) + 4 * h;
            const int c = 32 * (wave * XT + k) + i;
            const int x = xw + c;
            if ((lane & 1) == 0 && x < a.X1) {
                const int drel = (int)((v8[0] + (uint32_t)(c + D - 1)) & (uint32_t)(M - 1));
                out[(size_t)y * a.opitch + x] = (int16_t)((a.minD + drel) * 16);
            }
        }
    }
}

// invalid columns [0, X0) and [X1, W) of rows [row0, row1) (the matched band of valid_columns)
__global__ void k_fill_sides(int16_t* out, int opitch, long long fs_out, int row0, int W, int X0, int X1,
                             int16_t v) {
    const int y = row0 + blockIdx.x;
    int16_t* o = out + blockIdx.y * fs_out + (size_t)y * opitch;
    const int nl = X0, nr = W - X1;
    for (int i = threadIdx.x; i < nl + nr; i += blockDim.x) o[i < nl ? i : X1 + (i - nl)] = v;
}

struct SsdShape {
    int xt, nt, mb, hb, bias;
};

// Whether the MFMA kind runs (win, D) and its tile / band shape.  Key range: val - bias in
// [-hw, hw] (val = SR2 - 2X, bias = its centre), the leaving-row term bounded by the band height
// hb: |2M * Cor| <= 2M * (hb + win) * win * 128 (one term per entering row); M * hw + that + the
// x' index must stay below 2^31 (the keys are compared exactly; the shift wraps nothing).
bool ssd_shape(int win, int D, int rows, SsdShape* sh) {
    // D > 160 (7+ x'-tiles): the accumulators no longer fit beside the operands (spills; the
    // 4K D=256 w9 frame ran 3.2x slower than the ring kernel) — the ring / one-row kinds keep it
    if (win < 1 || win > 15 || (win & 1) == 0 || D < 32 || D > 160 || D % 32 != 0) return false;
    static const bool on = [] {
        const char* e = std::getenv("SV_SSD_MFMA");
        return !(e && e[0] == '0');
    }();
    if (!on) return false;
    const int nt = D / 32 + 1;
    const int xt = nt <= 5 ? 2 : 1;
    const int mb = D <= 128 ? 7 : 8;
    const long long M = 1LL << mb;
    const long long n = (long long)win * win;
    const long long cmax = n * 255 * 255, sl2 = n * 128 * 128;
    const long long bias = (cmax - sl2) / 2, hw = (cmax + sl2 + 1) / 2;
    int hb = rows < 96 ? rows : 64;
    if (rows >= 256 && win <= 9) hb = 96;
    if (hb < 1) hb = 1;
    const long long cor = (long long)(hb + win) * win * 128;
    const long long xpw = 32LL * (4 * xt + nt - 1);
    if (M * hw + 2 * M * cor + xpw + 64 >= (1LL << 31)) return false;
    if (2 * M * (sl2 + cor) >= (1LL << 31)) return false;   // 2M * acc itself
    *sh = SsdShape{xt, nt, mb, hb, (int)bias};
    return true;
}

template <int XT, int NT, int MB>
int launch_t(const MatchParams& a, const SsdShape& sh, hipStream_t s) {
    using C = SsdCfg<XT, NT, MB>;
    const int nf = a.nf > 1 ? a.nf : 1;
    const int rows = a.row1 - a.row0;
    dim3 grid((a.X1 - a.X0 + C::XW - 1) / C::XW, (rows + sh.hb - 1) / sh.hb, nf);
    static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ssd_mfma<XT, NT, MB>),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, C::lds(15));
    if (attr != hipSuccess) return (int)attr;
    static const int dbg = [] {
        const char* e = std::getenv("SV_SSD_DBG");   // A/B timing only: 1 no MFMA, 2 no epilogue
        return e ? std::atoi(e) : 0;
    }();
    hipLaunchKernelGGL((k_ssd_mfma<XT, NT, MB>), grid, dim3(kThreads), C::lds(a.win), s, a, sh.hb, sh.bias, dbg);
    return (int)hipGetLastError();
}

}  // namespace

bool ssd_mfma(int cost, int win, int num_disp) {
    SsdShape sh;
    return cost == COST_SSD && ssd_shape(win, num_disp, 1 << 20, &sh) && ssd_shape(win, num_disp, 1, &sh);
}

bool ssd_mfma_fits(const MatchParams& a, int cost) {
    // the raw rows arrive as 4-byte aligned dwords (LDS-DMA): image bases, row pitch and frame
    // stride must be multiples of 4 (torch / hipMalloc buffers of even widths are)
    const uintptr_t al = reinterpret_cast<uintptr_t>(a.L) | reinterpret_cast<uintptr_t>(a.R) | (uintptr_t)a.pitch |
                         (uintptr_t)(a.nf > 1 ? a.fs_in : 0);
    return ssd_mfma(cost, a.win, a.D) && a.r == a.win / 2 && (al & 3) == 0;
}

int launch_ssd_mfma(const MatchParams& a, hipStream_t s) {
    SsdShape sh;
    const int rows = a.row1 - a.row0;
    if (!ssd_shape(a.win, a.D, rows, &sh)) return (int)hipErrorInvalidValue;
    const int nf = a.nf > 1 ? a.nf : 1;
    const int16_t inv = (int16_t)((a.minD - 1) * 16);
    if (a.X0 > 0 || a.X1 < a.W) {
        hipLaunchKernelGGL(k_fill_sides, dim3(rows, nf), dim3(256), 0, s, a.out, a.opitch, nf > 1 ? a.fs_out : 0LL,
                           a.row0, a.W, a.X0, a.X1, inv);
        const int e = (int)hipGetLastError();
        if (e) return e;
    }
    MatchParams b = a;
    b.fs_out = nf > 1 ? a.fs_out : 0;
    b.fs_in = nf > 1 ? a.fs_in : 0;
    static const int xt_env = [] {   // A/B only: SV_SSD_XT=1|2 overrides the x-tiles per wave
        const char* e = std::getenv("SV_SSD_XT");
        return e ? std::atoi(e) : 0;
    }();
    SsdShape s2 = sh;
    if (xt_env == 1 || xt_env == 2) s2.xt = sh.nt <= 5 ? xt_env : 1;
    switch (sh.nt * 4 + s2.xt) {
        case 2 * 4 + 1: return launch_t<1, 2, 7>(b, s2, s);
        case 2 * 4 + 2: return launch_t<2, 2, 7>(b, s2, s);
        case 3 * 4 + 1: return launch_t<1, 3, 7>(b, s2, s);
        case 3 * 4 + 2: return launch_t<2, 3, 7>(b, s2, s);
        case 4 * 4 + 1: return launch_t<1, 4, 7>(b, s2, s);
        case 4 * 4 + 2: return launch_t<2, 4, 7>(b, s2, s);
        case 5 * 4 + 1: return launch_t<1, 5, 7>(b, s2, s);
        case 5 * 4 + 2: return launch_t<2, 5, 7>(b, s2, s);
        case 6 * 4 + 1: return launch_t<1, 6, 8>(b, s2, s);
    }
    return (int)hipErrorInvalidValue;
}

}  // namespace sv
