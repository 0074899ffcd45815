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
//       U(x') = M * (SR2(x') - bias) - ix' + off   (per row, built once per x' by the block)
//     so for one x the order of the keys is the order of (cost, d) — the oracle's first
//     minimum — and d - minD = (key + c + D - 1) mod M (c: the x column's block index).  The
//     lane's minimum over its registers and x'-tiles is a v_min3 chain; one v_permlane32_swap
//     joins the two lane halves (the two x' row halves of one x).  The first and the last
//     x'-tile of an x-tile hold complementary triangles of valid d (D % 32 == 0): masked by an
//     offset planted in the accumulators where the key range allows (BM), else by one
//     v_cndmask per edge cell.
//   * SR2: per staged row the block computes hsq(x') = sum_{i<win} R'(x'-r+i)^2 (4 v_dot4 on the
//     masked 16 bytes) once; the per-column running vertical sum adds the entering row's and
//     subtracts the leaving row's.
//   * staging: every step one LDS-DMA per thread (global_load_lds_dword) lands the raw dwords of
//     the row entering PRE = 5 steps later in a ring of win + 5 raw rows, retired by a counted
//     s_waitcnt vmcnt before the barrier that precedes its use — no global load result ever
//     sits in a VGPR, the row loop has one barrier per step (lgkmcnt + s_barrier only) and no
//     exposed global latency.  From the raw ring each step builds 4 byte-shifted copies of its
//     entering (L', ~R') and leaving (L', R') rows, so every 16-byte operand at any byte offset
//     is 4 aligned ds_read_b32 (an unaligned ds_read_b128 costs ~7x:
//     tools/microbench/lds_unaligned).
//   * the hsq ring (win + 2 rows) and U (double-buffered) live in LDS beside them.
//   * D <= 256 (<= 9 x'-tiles of accumulators) where the key range fits 32 bits (D > 128: win
//     <= 13); the 4-byte alignment of the images is checked by the launcher (ssd_mfma_fits).
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

template <int XT, int NT, int MB>
struct SsdCfg {
    static constexpr int M = 1 << MB;
    static constexpr int XW = 32 * XT * kWaves;        // output columns per block
    static constexpr int GT = kWaves * XT + NT - 1;    // x'-tiles per block
    static constexpr int XPW = 32 * GT;                // x' columns per block (ix' in [0, XPW))
    static constexpr int XPP = XPW + 32;               // hsq / U row length (+ a pad column block)
    static constexpr int LB = XW + 16;                 // L' bytes a row's operands read
    static constexpr int RB = XPW + 16;                // R' bytes
    // physical dwords of a row the operands read: starts up to XW - 1 (XPW - 1) plus the 4-byte
    // alignment offset, 4 dwords each
    static constexpr int NLD = LB / 4 + 1;
    static constexpr int NRD = RB / 4 + 1;
    // both streams' copies use one stride (immediate LDS offsets in the copy builder); the
    // dwords past NLD / NRD are never read (the builder's idle threads write one of them)
    using CP = Copies<(LB > RB ? LB : RB) + 4>;
    static constexpr int DWC = CP::DW;
    static_assert(NRD + 1 <= DWC && NLD + 1 <= DWC, "copies hold every dword the operands read + a pad");
    static constexpr int SIDE = CP::SIZE;              // one stream's 4 copies
    static constexpr int SLOT = 2 * SIDE;              // one staged row: L' copies | R' (or ~R') copies
    // raw ring (LDS-DMA landing rows): one dword per thread, NLD L dwords then NRD R dwords
    static constexpr int NIT = NLD + NRD;
    static_assert(NIT <= kThreads, "one raw dword per thread");
    static constexpr int NB = (2 * NIT + kThreads - 1) / kThreads;   // copy-builder items per thread
    static constexpr int NJ = (XPW + kThreads - 1) / kThreads;       // hsq columns per thread
    static constexpr int RAWD = (NIT + 63) / 64 * 64;   // raw ring row (dwords): the DMA waves' lanes
    static constexpr int RAWB = 4 * RAWD;
    static constexpr int PRE = 5;                      // DMA issue distance (steps)
    // 3 entering + 3 leaving slots, the hsq ring (win + 2 rows), U[2], the raw ring (win + PRE)
    static constexpr int lds(int win) { return 6 * SLOT + (win + 2) * 4 * XPP + 2 * 4 * XPP + (win + PRE) * RAWB; }
    static_assert(XT * NT * 16 <= 160, "accumulators must stay in arch VGPRs");
    static_assert(lds(15) <= 160 * 1024, "LDS per block (win 15)");
};

// The raw rows arrive by LDS-DMA (global_load_lds_dword: wave-uniform LDS base + 4 x lane), one
// dword per thread: the 4-byte aligned dword of columns c0 .. c0 + 3 (c0 % 4 == 0) clamped into
// the row, ca = clamp(c0, 0, (W - 1) & ~3).  Columns outside [0, W) replicate the edge pixel
// (the oracle's replicate border): the copy builder re-selects the bytes with one v_perm per
// dword (the selector below, fixed per thread: the identity inside the image).
__device__ __forceinline__ int clamp_dword(int c0, int W) { return min(max(c0, 0), (W - 1) & ~3); }
// v_perm selector taking the dword loaded at clamp_dword(c0) to the replicate-clamped bytes of
// columns c0 .. c0 + 3 (0x03020100, the identity, inside the image)
__device__ __forceinline__ uint32_t edge_sel(int c0, int W) {
    const int ca = clamp_dword(c0, W);
    uint32_t sel = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) sel |= (uint32_t)(min(max(c0 + b, 0), W - 1) - ca) << (8 * b);
    return sel;
}

template <int XT, int NT> struct SsdOcc {
    static constexpr int W = XT * NT <= 4 ? 3 : 2;
};

// SSD matrix-core kernel.  One block = 4 waves = a band of hb output rows x 128 XT columns; row
// step s of the band (s = 0 .. rows + win - 2) enters image row y0 - r + s and leaves row
// y0 - r + s - win.  Software-pipelined: iteration s runs, between two barriers,
//   B(s)   the MFMAs of step s (operand slot s % 3),
//   A(s+1) hsq / SR2 / U of step s + 1 (slot (s + 1) % 3's ~R') and the copies of step s + 2
//          (slot (s + 2) % 3, from the raw ring),
//   E(s)   the keys and the output row of step s (U buffer s & 1),
// all independent, and branch-free so the compiler can interleave them (LDS latency under
// MFMA and VALU work).  BM: edge masking by the accumulator offset (see SsdShape).
template <int XT, int NT, int MB, bool BM>
__global__ __launch_bounds__(kThreads, (SsdOcc<XT, NT>::W)) void k_ssd_mfma(MatchParams a, int hb, int bias,
                                                                          uint32_t off) {
    using C = SsdCfg<XT, NT, MB>;
    constexpr int M = C::M, DWC = C::DWC, XPP = C::XPP, PRE = C::PRE;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int h = lane >> 5, j = lane & 31;
    const int z = blockIdx.z;
    const uint8_t* Limg = a.L + z * a.fs_in;
    const uint8_t* Rimg = a.R + z * a.fs_in;
    const int W = a.W, H = a.H, r = a.r, win = a.win, D = a.D;
    const int xw = a.X0 + blockIdx.x * C::XW;               // first output column of the block
    const int xpb = xw - (a.minD + D - 1);                  // x' of ix' = 0
    const int y0 = a.row0 + blockIdx.y * hb;
    const int y1 = min(a.row1, y0 + hb);
    if (y0 >= y1) return;
    const int hr = win + 2;                                 // hsq ring rows
    const int rawr = win + PRE;                             // raw ring rows
    // physical row streams start 4-byte aligned: logical byte b of the L' stream (column
    // xw - r + b) is physical byte b + oL
    const int aL = (xw - r) & ~3, oL = (xw - r) - aL;
    const int aR = (xpb - r) & ~3, oR = (xpb - r) - aR;
    uint32_t* const sm32 = reinterpret_cast<uint32_t*>(smem);
    int32_t* const hsq = reinterpret_cast<int32_t*>(smem + 6 * C::SLOT);                  // [hr][XPP]
    uint32_t* const Ub = reinterpret_cast<uint32_t*>(smem + 6 * C::SLOT + hr * 4 * XPP);  // [2][XPP]
    uint32_t* const raw = Ub + 2 * XPP;                                                    // [rawr][RAWD]

    // ---- raw rows: one LDS-DMA per step from every wave that holds one of the NIT stream dwords
    // (the thread's dword of the L' | R' streams, clamped into the image row; rows past the band
    // reload the clamped last row into a ring row no copy reads again), so each wave's counted
    // waits below are exact; a wave without stream dwords issues none (its waits then only
    // cover its own stores)
    const bool isLq = tid < C::NLD;
    const int c0q = isLq ? aL + 4 * tid : aR + 4 * (tid - C::NLD);
    const uint8_t* gq = (isLq ? Limg : Rimg) + clamp_dword(c0q, W);
    const bool dma_wave = 64 * wave < C::NIT;
    auto issue_raw = [&](int k, int rk) {   // the entering row of step k into ring row rk
        if (!dma_wave) return;               // wave-uniform
        const int y = min(max(y0 - r + k, 0), H - 1);
        typedef __attribute__((address_space(1))) void gvoid;
        typedef __attribute__((address_space(3))) void lvoid;
        __builtin_amdgcn_global_load_lds((gvoid*)(gq + (size_t)y * a.pitch), (lvoid*)(raw + rk * C::RAWD + wave * 64),
                                         4, 0, 0);
    };

    // ---- the copy builder: item q < NIT of a step builds dword w of the entering slot's L' or
    // ~R' copies from raw row k, item NIT + q the leaving slot's L' or R' from raw row k - win;
    // each thread's items are fixed, so their addresses, xor masks and edge selectors are
    // computed once (the edge byte select is the identity inside the image)
    int b_rq[C::NB], b_rqh[C::NB], b_dst[C::NB];
    uint32_t b_x[C::NB], b_slo[C::NB], b_shi[C::NB];
    bool b_side[C::NB];
#pragma unroll
    for (int u = 0; u < C::NB; ++u) {
        const int q = tid + u * kThreads;
        const bool real = q < 2 * C::NIT;
        const int side = real && q >= C::NIT ? 1 : (real ? 0 : 1);
        const int rq = real ? (side ? q - C::NIT : q) : 0;
        const bool isL = !real || rq < C::NLD;
        const int w = real ? (isL ? rq : rq - C::NLD) : C::NLD;   // idle threads: a pad dword
        const bool more = isL ? (w + 1 < C::NLD) : (w + 1 < C::NRD);
        const int c0 = (isL ? aL : aR) + 4 * w;
        b_rq[u] = rq;
        b_rqh[u] = real && more ? rq + 1 : rq;
        b_side[u] = side;
        b_dst[u] = side * 3 * (C::SLOT / 4) + (isL ? 0 : C::SIDE / 4) + w;
        // L' = L ^ 0x80 both sides; R side: ~R' = R ^ 0x7f entering, R' = R ^ 0x80 leaving
        b_x[u] = (isL || side) ? 0x80808080u : 0x7F7F7F7Fu;
        b_slo[u] = edge_sel(c0, W);
        b_shi[u] = real && more ? edge_sel(c0 + 4, W) : b_slo[u];
    }
    auto build = [&](int ks, int r0, int r1) {   // slot ks from ring rows r0 (entering), r1 (leaving)
#pragma unroll
        for (int u = 0; u < C::NB; ++u) {
            const uint32_t* p = raw + (b_side[u] ? r1 : r0) * C::RAWD;
            const uint32_t lo = __builtin_amdgcn_perm(p[b_rq[u]], p[b_rq[u]], b_slo[u]) ^ b_x[u];
            const uint32_t hi = __builtin_amdgcn_perm(p[b_rqh[u]], p[b_rqh[u]], b_shi[u]) ^ b_x[u];
            uint32_t* d = sm32 + ks * (C::SLOT / 4) + b_dst[u];
#pragma unroll
            for (int sh = 0; sh < 4; ++sh) d[sh * DWC] = __builtin_amdgcn_alignbyte(hi, lo, sh);
        }
    };

    // the taps i >= win are zero on the L side (the MFMA's B operand) and in the hsq sums
    v4i wmask;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int nb = min(max(win - 4 * q, 0), 4);
        wmask[q] = nb >= 4 ? -1 : (int)((1u << (8 * nb)) - 1u);
    }

    // ---- A(k): hsq of step k's entering row (its ~R' copies), SR2 and U(k).  Thread-owned
    // columns (hsq needs no barrier); columns past XPW compute into the pad column block
    // LDS dword offset of the 16 operand bytes at stream byte p: copy p & 3, dword p >> 2; p
    // advancing by 32 (one tile) moves it by 8 dwords, so one per-lane base serves every tile
    // of a wave through the instructions' immediate offsets
    auto lane_off = [](int p) { return (p & 3) * DWC + (p >> 2); };
    const int offA = C::SIDE / 4 + lane_off(tid + oR);
    int sr2[C::NJ];
#pragma unroll
    for (int jj = 0; jj < C::NJ; ++jj) sr2[jj] = 0;
    auto phaseA = [&](int ks, int he, int hl, int ub, bool leave) {
        const uint32_t* er = sm32 + ks * (C::SLOT / 4) + offA;   // ~R' of column tid
        int32_t* hs_e = hsq + he * XPP;
        const int32_t* hs_l = hsq + hl * XPP;
        uint32_t* U = Ub + ub * XPP;
        const int lm = leave ? -1 : 0;
#pragma unroll
        for (int jj = 0; jj < C::NJ; ++jj) {
            // column tid + 256 jj: its copy dwords sit 64 jj further (immediate offsets)
            const int ix = min(tid + jj * kThreads, C::XPW + (tid & 31));
            const uint32_t* e = er + 64 * jj;
            const v4i v = v4i{(int)e[0], (int)e[1], (int)e[2], (int)e[3]};
            int hs = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int m = ~v[q] & wmask[q];   // R' = ~(~R')
                hs = __builtin_amdgcn_sdot4(m, m, hs, false);
            }
            const int old = hs_l[ix];
            hs_e[ix] = hs;
            sr2[jj] += hs - (old & lm);
            // unsigned keys: + off (a multiple of M >= the key range's half-width)
            U[ix] = (uint32_t)((sr2[jj] - bias) * M - ix) + off;
        }
    };

    // ---- accumulators; lane-constant selection of the edge tiles: cell (x' row i, x column j)
    // of the first x'-tile of an x-tile is a valid disparity iff i >= j, of the last iff i < j
    // (D % 32 == 0).  BM: the invalid cells start at 2^(30 - MB), i.e. their keys sit 2^31 above
    // the true ones (the sliding sums only add and remove rows, so the offset stays): the valid
    // keys lie in [0, 2R], the invalid ones in [2^31, 2^31 + 2R] — above every valid one
    bool sel0[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) sel0[q] = ((q & 3) + 8 * (q >> 2) + 4 * h) >= j;
    v16i acc[XT][NT];
#pragma unroll
    for (int k = 0; k < XT; ++k)
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                int v = 0;
                if (BM && t == 0) v = sel0[q] ? 0 : (1 << (30 - MB));
                if (BM && t == NT - 1) v = sel0[q] ? (1 << (30 - MB)) : 0;
                acc[k][t][q] = v;
            }

    // ---- B(s): A = R' rows (32 x' of an x'-tile), B = L' columns (32 x of an x-tile): a lane
    // holds ONE x column and 16 x' rows, so the minimum over x' stays inside the lane.  K =
    // [16 taps of the entering row (lanes 0..31) | 16 of the leaving row (lanes 32..63)];
    // entering ~R' (= -R' - 1), leaving R': the accumulator holds -X - Cor(x)
    const int hside = h * 3 * (C::SLOT / 4);               // the lane's half: entering / leaving slot
    const int hmask = h ? 0 : -1;
    const int offL = hside + lane_off(32 * wave * XT + j + oL);
    const int offR = hside + C::SIDE / 4 + lane_off(32 * wave * XT + j + oR);
    auto phaseB = [&](int ks, bool leave) {
        const uint32_t* lp = sm32 + ks * (C::SLOT / 4) + offL;
        const uint32_t* rp = sm32 + ks * (C::SLOT / 4) + offR;
        const int lm = hmask | (leave ? -1 : 0);          // warm-up: the leaving half adds nothing
        const v4i wm = wmask & lm;
        v4i lop[XT];
#pragma unroll
        for (int k = 0; k < XT; ++k) lop[k] = v4i{(int)lp[8 * k], (int)lp[8 * k + 1], (int)lp[8 * k + 2], (int)lp[8 * k + 3]} & wm;
#pragma unroll
        for (int gi = 0; gi < XT + NT - 1; ++gi) {
            const uint32_t* q = rp + 8 * gi;
            const v4i rop = v4i{(int)q[0], (int)q[1], (int)q[2], (int)q[3]};
#pragma unroll
            for (int k = 0; k < XT; ++k) {
                const int t = gi - k;
                if (t >= 0 && t < NT) acc[k][t] = __builtin_amdgcn_mfma_i32_32x32x32_i8(rop, lop[k], acc[k][t], 0, 0, 0);
            }
        }
    };

    // ---- E(s): key = U(x') + 2M * acc; the minimum over the lane's x' rows and x'-tiles, x'-tile
    // by x'-tile (its U rows serve every x-tile it pairs with); without BM a lane-constant
    // select voids the edge tiles' invalid cells.  The two lane halves hold the two x' row
    // halves of one x: v_permlane32_swap exchanges the upper half of one register with the lower
    // half of the other, so with two x-tiles lanes 0..31 end with x-tile 0 and lanes 32..63 with
    // x-tile 1 — 64 consecutive output columns, one buffer store (lanes with nothing to write
    // store past the descriptor's range: dropped, no exec branch, one store per step exactly)
    const auto orsrc = __builtin_amdgcn_make_buffer_rsrc(a.out + z * a.fs_out, 0, 0x7FFFFFFF, 0x00020000);
    const int kk = XT == 2 ? h : 0;
    const int cst = 32 * (wave * XT + kk) + j;             // the stored column's block index
    const bool st_ok = (XT == 2 || h == 0) && xw + cst < a.X1;
    auto phaseE = [&](int ub, int y) {
        const uint32_t* U = Ub + ub * XPP + 4 * h;
        uint32_t b0[XT], b1[XT];
#pragma unroll
        for (int k = 0; k < XT; ++k) b0[k] = b1[k] = 0xFFFFFFFFu;
#pragma unroll
        for (int gi = 0; gi < XT + NT - 1; ++gi) {
            // U of the 16 x' rows the lane holds: rows 8g + 4h + 0..3, one 16-byte LDS
            // broadcast per g (every lane of a half reads the same address)
            uint32_t u[16];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const v4i v = *reinterpret_cast<const v4i*>(U + 32 * (wave * XT + gi) + 8 * g);
#pragma unroll
                for (int e = 0; e < 4; ++e) u[4 * g + e] = (uint32_t)v[e];
            }
#pragma unroll
            for (int k = 0; k < XT; ++k) {
                const int t = gi - k;
                if (t < 0 || t >= NT) continue;
                uint32_t kv[16];
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    kv[q] = ((uint32_t)acc[k][t][q] << (MB + 1)) + u[q];
                    if (!BM && t == 0) kv[q] = sel0[q] ? kv[q] : 0xFFFFFFFFu;
                    if (!BM && t == NT - 1) kv[q] = sel0[q] ? 0xFFFFFFFFu : kv[q];
                }
#pragma unroll
                for (int q = 0; q < 16; q += 4) {
                    b0[k] = min3u(b0[k], kv[q], kv[q + 1]);
                    b1[k] = min3u(b1[k], kv[q + 2], kv[q + 3]);
                }
            }
        }
        uint32_t res;
        if constexpr (XT == 2) {
            const auto p = __builtin_amdgcn_permlane32_swap(min(b0[0], b1[0]), min(b0[1], b1[1]), false, false);
            res = min((uint32_t)p[0], (uint32_t)p[1]);
        } else {
            const uint32_t b = min(b0[0], b1[0]);
            const auto p = __builtin_amdgcn_permlane32_swap(b, b, false, false);
            res = min((uint32_t)p[0], (uint32_t)p[1]);
        }
        // d - minD = (c - ix') + D - 1 and the key's low MB bits hold -ix' (off % M == 0)
        const int drel = (int)((res + (uint32_t)(cst + D - 1)) & (uint32_t)(M - 1));
        const int o = st_ok ? 2 * (y * a.opitch + xw + cst) : (int)0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b16((uint16_t)((a.minD + drel) * 16), orsrc, o, 0, 0);
    };

    // ---- prologue: raw rows 0 .. PRE - 1; copies of steps 0 and 1; A(0)
    const int nsteps = (y1 - y0) + win - 1;
    auto inc = [](int v, int n) { return v + 1 == n ? 0 : v + 1; };
    static_assert(PRE == 5, "vmcnt immediates below");
#pragma unroll
    for (int k = 0; k < PRE; ++k) issue_raw(k, k);
    asm volatile("s_waitcnt vmcnt(3)" ::: "memory");   // rows 0 and 1
    lds_barrier();
    build(0, 0, 0);                                     // (no leaving row yet: its half is masked)
    lds_barrier();
    phaseA(0, 0, 2 % hr, 0, false);
    build(1, 1 % rawr, (1 + PRE) % rawr);
    asm volatile("s_waitcnt vmcnt(2)" ::: "memory");   // row 2
    lds_barrier();

    // ring indices, advanced incrementally (a runtime modulo is a VALU reciprocal chain):
    // si = s % 3, ha = (s + 1) % hr, hl = (s + 3) % hr (the row leaving at step s + 1, hr = win
    // + 2), rp = (s + PRE) % rawr, rb = (s + 2) % rawr, rbl = (s + 2 - win) % rawr
    int si = 0, ha = 1 % hr, hl = 3 % hr, rp = PRE % rawr, rb = 2 % rawr, rbl = (2 + PRE) % rawr;
    // raw row s + 3 (issued at iteration s - 2) is retired at the end of iteration s; the ops
    // younger than it: the DMAs of iterations s - 1 and s and, once outputs are stored (one
    // store per iteration from step win - 1 on), the stores of iterations s - 2 .. s
    auto iteration = [&](int s, auto epi) {
        constexpr bool EPI = decltype(epi)::value;
        const int s1 = inc(si, 3), s2 = inc(s1, 3);
        issue_raw(s + PRE, rp);
        phaseB(si, s >= win);
        phaseA(s1, ha, hl, (s + 1) & 1, s + 1 >= win);
        build(s2, rb, rbl);
        if constexpr (EPI) {
            phaseE(s & 1, y0 + s - (win - 1));
            const int e = s - (win - 1);                 // stored steps before this one
            if (e >= 2) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
            else if (e == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        }
        lds_barrier();
        si = s1;
        ha = inc(ha, hr);
        hl = inc(hl, hr);
        rp = inc(rp, rawr);
        rb = inc(rb, rawr);
        rbl = inc(rbl, rawr);
    };
    int s = 0;
    for (; s < win - 1; ++s) iteration(s, std::false_type{});
    for (; s < nsteps; ++s) iteration(s, std::true_type{});
    // the DMAs still in flight land in this block's LDS: drain them before the block ends
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
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
    bool big;       // edge cells masked by the accumulator offset (R < 2^30)
    uint32_t off;   // key offset (a multiple of M): R rounded up (big) or 2^31
};

// Whether the MFMA kind runs (win, D) and its tile / band shape.  Key range: val - bias in
// [-hw, hw] (val = SR2 - 2X, bias = its centre), the leaving-row term bounded by the band height
// hb: |2M * Cor| <= 2M * (hb + win) * win * 128 (one term per entering row); the half-width
// R = M * hw + that + the x' index.  The keys are exact modulo 2^32 (the shift may wrap, the
// sum lands back in [off - R, off + R]): R < 2^31 with off = 2^31, and R < 2^30 for the offset
// masking (off = R; 1080p D=128: windows <= 13; D=160: <= 9).
bool ssd_shape(int win, int D, int rows, SsdShape* sh) {
    // D up to 256 (9 x'-tiles of accumulators, 194 VGPRs at one x-tile per wave); the key
    // range below decides the windows (D > 128 takes 8 index bits: up to win 13)
    if (win < 1 || win > 15 || (win & 1) == 0 || D < 32 || D > 256 || D % 32 != 0) return false;
    static const bool on = [] {
        const char* e = std::getenv("SV_SSD_MFMA");
        return !(e && e[0] == '0');
    }();
    if (!on) return false;
    const int nt = D / 32 + 1;
    // x-tiles per wave: one (<= 128 VGPRs: 3 blocks per CU) unless the edge masking needs the
    // per-cell select (no offset room: w15 at D=128), where two amortise the operand loads
    // better — 1080p D=128, one stream, 26 frames: w9 767 vs 847 us, w15 458 vs 424 us; VGA
    // D=64 w9 136 vs 161 us (profiles/r06_ssd)
    const int xt = nt >= 4 && nt <= 5 ? 2 : 1;   // refined below once the key range is known
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
    const long long R = M * hw + 2 * M * cor + xpw + 64;
    if (R >= (1LL << 31)) return false;
    // the offset is a multiple of M: the disparity index is read from the key's low bits
    const long long off = (R + M - 1) / M * M;
    const bool big = off < (1LL << 30);
    *sh = SsdShape{big ? 1 : xt, nt, mb, hb, (int)bias, big, big ? (uint32_t)off : 0x80000000u};
    return true;
}

template <int XT, int NT, int MB, bool BM>
int launch_t(const MatchParams& a, const SsdShape& sh, hipStream_t s) {
    using C = SsdCfg<XT, NT, MB>;
    const int nf = a.nf > 1 ? a.nf : 1;
    const int rows = a.row1 - a.row0;
    dim3 grid((a.X1 - a.X0 + C::XW - 1) / C::XW, (rows + sh.hb - 1) / sh.hb, nf);
    if (C::lds(a.win) > 65536) {   // opt in to > 64 KiB of dynamic LDS (per device: every launch)
        const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_ssd_mfma<XT, NT, MB, BM>),
                                                    hipFuncAttributeMaxDynamicSharedMemorySize, C::lds(a.win));
        if (attr != hipSuccess) return (int)attr;
    }
    hipLaunchKernelGGL((k_ssd_mfma<XT, NT, MB, BM>), grid, dim3(kThreads), C::lds(a.win), s, a, sh.hb, sh.bias, sh.off);
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
    // the output stores are 32-bit byte offsets from one buffer descriptor per frame
    const bool ofits = 2LL * ((long long)a.row1 * a.opitch + a.W) < 0x7FFFFFFFLL;
    return ssd_mfma(cost, a.win, a.D) && a.r == a.win / 2 && (al & 3) == 0 && ofits;
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
    const auto go = [&](auto bm) {
        constexpr bool BM = decltype(bm)::value;
        switch (sh.nt * 4 + sh.xt) {
            case 2 * 4 + 1: return launch_t<1, 2, 7, BM>(b, sh, s);
            case 2 * 4 + 2: return launch_t<2, 2, 7, BM>(b, sh, s);
            case 3 * 4 + 1: return launch_t<1, 3, 7, BM>(b, sh, s);
            case 3 * 4 + 2: return launch_t<2, 3, 7, BM>(b, sh, s);
            case 4 * 4 + 1: return launch_t<1, 4, 7, BM>(b, sh, s);
            case 4 * 4 + 2: return launch_t<2, 4, 7, BM>(b, sh, s);
            case 5 * 4 + 1: return launch_t<1, 5, 7, BM>(b, sh, s);
            case 5 * 4 + 2: return launch_t<2, 5, 7, BM>(b, sh, s);
            case 6 * 4 + 1: return launch_t<1, 6, 8, BM>(b, sh, s);
            case 7 * 4 + 1: return launch_t<1, 7, 8, BM>(b, sh, s);
            case 8 * 4 + 1: return launch_t<1, 8, 8, BM>(b, sh, s);
            case 9 * 4 + 1: return launch_t<1, 9, 8, BM>(b, sh, s);
        }
        return (int)hipErrorInvalidValue;
    };
    return sh.big ? go(std::true_type{}) : go(std::false_type{});
}

}  // namespace sv
