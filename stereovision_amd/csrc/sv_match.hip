// sv_match.hip — the disparity cost-volume + winner-take-all kernel for gfx950.
//
// Replaces the reference's `cv2.StereoSGBM_create(...).compute(gray_left, gray_right)`
// (depth_map.py:894-909, fused_depth_map.py:988-1004) with the build-defined SAD / SSD /
// HOG winner-take-all engine specified in DESIGN.md ("Semantics").  Output: int16 = d*16,
// invalid = (minD-1)*16 outside the matched band [X0, X1).
//
// Work decomposition (one wave = ROWS output rows (1 or 4), one run of output columns):
//   * the wave is split into G = 64/LPG groups of LPG lanes; group g walks its segment of
//     S columns left to right;
//   * lane l of a group owns the DPL consecutive disparities d = minD + l*DPL + k, so the
//     LPG*DPL candidates of one pixel sit across one group, and the argmin is an in-lane
//     min3 chain over (cost << dbits | d) keys + a DPP row reduction (first-min tie-break);
//   * image data is staged ONCE per wave in LDS as "column packs": the window rows of one
//     column packed 4 bytes per dword (zero padded).  One v_sad_u8 sums 4 vertical taps;
//   * the horizontal window is a running sum along x: per step the group adds the column
//     entering the window and subtracts the column leaving it;
//   * the right-image column a lane needs for disparity k at step t is the column it
//     loaded for k-1 at step t-1, so each lane keeps a DPL-deep register ring and loads
//     ONE new right pack per step (plus one for the leaving column);
//   * right packs are stored with a 1-in-DPL slot gap (rslot) so the 16 lanes of a group,
//     whose columns are DPL apart, hit distinct LDS banks, and a lane's reads inside a
//     DPL-step chunk use static offsets;
//   * the per-pixel DPP reductions of a DPL-step chunk are batched (independent chains)
//     before one coalesced store per lane.
// Cost kinds:
//   SAD   1 row/wave, pack = ceil(win/4) byte dwords, ceil(win/4) v_sad_u8 per column cell;
//   SAD4  4 rows/wave for win >= 5: packs of the 2r-2 rows the four windows share + one
//         word per row for its 3 others; the metric configs run the ring kind below
//         (k_match_ring: a register ring of entering-column costs, v_sad_u32 updates);
//   SSD   v_dot4_u32_u8: sum (L-R)^2 = sum L^2 + sum R^2 - 2 sum L*R (squares per pack);
//   HOG   9-bin u16 window histograms as packs compared with v_sad_u16 (no running window).
#include "sv_internal.h"
#include "sv_xcd.h"

#include <algorithm>
#include <cstdlib>
#include <vector>
#include <cstdio>
#include <type_traits>

namespace sv {
namespace {

constexpr int COST_SAD4 = 4;          // internal kind: SAD, four output rows per wave

// Segment width per lane group: 4*LPG columns rounded up to a multiple of DPL so that
// every group of a wave shares the same right-pack slot phase (rslot).
// `sm` = segment length in units of LPG columns (4; SV_SAD4_SEG overrides it for the
// 4-row kind, for A/B measurements).
__host__ __device__ __forceinline__ int seg_width(int lpg, int dpl, int sm = 4) { return (sm * lpg + dpl - 1) / dpl * dpl; }
__host__ __device__ __forceinline__ int wave_cols(int lpg, int dpl, int sm = 4) { return (64 / lpg) * seg_width(lpg, dpl, sm); }
// 4-row kind: full-length segments when the common words are split into their own array
// (24-B packs, r <= 5); half-length for the 28-B packs of r 6..7, which would otherwise
// hold the LDS to 1.5 waves per SIMD.
int seg_mult(int kind, int r) {
    static const int sm4 = [] {
        const char* e = std::getenv("SV_SAD4_SEG");
        const int v = e ? std::atoi(e) : 0;
        return v >= 1 && v <= 8 ? v : 0;
    }();
    if (kind != COST_SAD4) return 4;
    if (sm4) return sm4;
    return (2 * r - 2 + 3) / 4 <= 2 ? 4 : 2;
}

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return min(max(v, lo), hi); }

struct Word3 { uint32_t x, y, z; };   // a 12-byte common-word slot (4-byte aligned)

// A column pack holds NW live dwords inside a 16*Q-byte LDS slot.
template <int COST, int ND> struct PackCfg {
    // ND is the kind's width parameter: byte dwords (SAD, SSD), unused (HOG), the window
    // radius r (SAD4: ceil((2r-2)/4) common dwords + 4 per-row dwords)
    static constexpr int NW = COST == COST_SAD ? ND : COST == COST_SSD ? ND + 1
                            : COST == COST_SAD4 ? (2 * ND - 2 + 3) / 4 + 4 : 5;
    static constexpr int Q = (NW + 3) / 4;
    static constexpr int ROWS = COST == COST_SAD4 ? 4 : 1;
    // waves per block: the 4-row kind's packs are large, one wave per block lets the LDS
    // hold as many waves as the register file does
    static constexpr int WPB = COST == COST_SAD4 ? 1 : 4;
    // SPLIT (4-row kind with <= 2 common words): the common words live in a separate
    // 8-byte-per-slot array, the 4 per-row words in the 16-byte array: 24 B per pack
    // instead of a 32-byte slot, so a 4-LPG segment still fits 2 waves per SIMD in LDS
    // HOG (5 words) splits too: word 0 in the 8-byte array, words 1-4 in a 16-byte slot, so
    // a group's 16 lanes (slots DPL+1 apart) read disjoint banks (32-byte slots: 2-way)
    static constexpr int NC = COST == COST_SAD4 ? NW - 4 : (COST == COST_HOG || (COST == COST_SSD && NW == 5)) ? 1 : 0;
    // (r 6..7: 3 common words in a 12-byte slot of their own: 28-B packs, so the ring kind's
    // LDS holds ~40% longer segments than with a padded 16-byte slot)
    static constexpr bool SPLIT = (COST == COST_SAD4 && NC <= 3) || COST == COST_HOG ||
                                  (COST == COST_SSD && NW == 5);
    // (the 4-row kind with one common word, r 2..3: a 4-byte slot, 20-B packs)
    static constexpr int CW = (COST == COST_SAD4 && NC == 1) ? 1 : NC <= 2 ? 2 : 3;   // words per common slot
    using CT = typename std::conditional<CW == 1, uint32_t,
                                         typename std::conditional<CW == 2, uint2, Word3>::type>::type;
    static constexpr int QX = SPLIT ? 1 : Q;          // uint4 per slot in the main array
    static constexpr int SLOT_BYTES = 16 * QX + (SPLIT ? 4 * CW : 0);
};
template <int NW> struct Pk { uint32_t w[NW]; };

// 4-row kind with r <= 5 (win <= 11): argmin keys are (cost << 16) | idx, maintained with
// v_sad_hi_u8 (cost max 30855: keys incl. the padding offset stay below 2^32).
__host__ __device__ constexpr bool hi_keys(int cost, int r) { return cost == COST_SAD4 && r <= 5; }

// Pointer to a column-pack slot (main array + the split common-word array).
template <int COST, int ND, typename X, typename C> struct PackPtrT {
    X* x;
    C* c;
    __device__ __forceinline__ PackPtrT operator+(int s) const {
        return {x + s * PackCfg<COST, ND>::QX, PackCfg<COST, ND>::SPLIT ? c + s : c};
    }
};
template <int COST, int ND>
using PackPtr = PackPtrT<COST, ND, const uint4, const typename PackCfg<COST, ND>::CT>;
template <int COST, int ND> using PackOut = PackPtrT<COST, ND, uint4, typename PackCfg<COST, ND>::CT>;

// B128: the 16-byte slot as one ds_read_b128 (the ring kind, whose 32-lane groups read
// slots 80 B apart: as two dword pairs, lanes l and l+16 of a b32 cycle share banks).  The
// other kinds keep the split dword loads the compiler pairs into ds_read2_b64 (HOG: b128
// measured 518 -> 655 us per 4K frame).
template <int COST, int ND, bool B128 = false>
__device__ __forceinline__ Pk<PackCfg<COST, ND>::NW> ld(PackPtr<COST, ND> p) {
    using P = PackCfg<COST, ND>;
    Pk<P::NW> v;
    if constexpr (P::SPLIT) {
        if constexpr (P::CW == 1) {
            v.w[0] = *p.c;
        } else {
            const typename P::CT c = *p.c;
            v.w[0] = c.x;
            if constexpr (P::NC > 1) v.w[1] = c.y;
            if constexpr (P::NC > 2) v.w[2] = c.z;
        }
        if constexpr (B128) {
            const uint4 m = *p.x;
            v.w[P::NC] = m.x;
            v.w[P::NC + 1] = m.y;
            v.w[P::NC + 2] = m.z;
            v.w[P::NC + 3] = m.w;
        } else {
            const uint32_t* q = reinterpret_cast<const uint32_t*>(__builtin_assume_aligned(p.x, 16));
#pragma unroll
            for (int i = 0; i < 4; ++i) v.w[P::NC + i] = q[i];
        }
    } else {
        const uint32_t* q = reinterpret_cast<const uint32_t*>(__builtin_assume_aligned(p.x, 16));
#pragma unroll
        for (int i = 0; i < P::NW; ++i) v.w[i] = q[i];
    }
    return v;
}

// Store the NW words w[0..NW) of one pack.
template <int COST, int ND>
__device__ __forceinline__ void put(PackOut<COST, ND> p, const uint32_t (&w)[8]) {
    using P = PackCfg<COST, ND>;
    if constexpr (P::SPLIT) {
        if constexpr (P::CW == 1) *p.c = w[0];
        else if constexpr (P::CW == 2) *p.c = make_uint2(w[0], P::NC > 1 ? w[1] : 0u);
        else *p.c = Word3{w[0], w[1], w[2]};
        p.x[0] = make_uint4(w[P::NC], w[P::NC + 1], w[P::NC + 2], w[P::NC + 3]);
    } else {
        p.x[0] = make_uint4(w[0], w[1], w[2], w[3]);
        if constexpr (P::Q > 1) p.x[1] = make_uint4(w[4], w[5], w[6], w[7]);
    }
}

// Column cost(s) of one (left pack, right pack) pair: v[0] (v[0..3]: the four rows of SAD4).
template <int COST, int ND, int NW>
__device__ __forceinline__ void ccol(const Pk<NW>& l, const Pk<NW>& r, uint32_t* v) {
    if constexpr (COST == COST_SAD) {
        uint32_t a = 0u;
#pragma unroll
        for (int i = 0; i < ND; ++i) a = __builtin_amdgcn_sad_u8(l.w[i], r.w[i], a);
        v[0] = a;
    } else if constexpr (COST == COST_SAD4) {
        constexpr int NC = NW - 4;
        uint32_t s = 0u;
#pragma unroll
        for (int i = 0; i < NC; ++i) s = __builtin_amdgcn_sad_u8(l.w[i], r.w[i], s);
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = __builtin_amdgcn_sad_u8(l.w[NC + q], r.w[NC + q], s);
    } else if constexpr (COST == COST_SSD) {
        uint32_t dot = 0u;
#pragma unroll
        for (int i = 0; i < ND; ++i) dot = __builtin_amdgcn_udot4(l.w[i], r.w[i], dot, false);
        v[0] = (l.w[ND] + r.w[ND]) - (dot << 1);
    } else {  // HOG: 9 u16 bins in 5 dwords; the cost IS the cell value
        uint32_t a = 0u;
#pragma unroll
        for (int i = 0; i < 5; ++i) a = __builtin_amdgcn_sad_u16(l.w[i], r.w[i], a);
        v[0] = a;
    }
}

// h + d * m (m = 1 << dbits, |d| < 2^23: one column's cost difference) as ONE
// v_mad_i32_i24.  Through the mul24 intrinsic LLVM does not factor the per-step updates
// into running diff sums (which `h += d << s` in plain C gets: an extra add per cell).
__device__ __forceinline__ uint32_t shl_add(uint32_t d, int m, uint32_t h) {
    return h + (uint32_t)__mul24((int)d, m);
}

// Build one column pack for logical column c around output row y (replicate-clamped).
template <int COST, int ND>
__device__ __forceinline__ void build_pack(const MatchParams& a, const uint8_t* img,
                                           const uint16_t* hist, int c, int y, PackOut<COST, ND> dst) {
    const int cc = clampi(c, 0, a.W - 1);
    if constexpr (COST == COST_HOG) {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(hist + ((size_t)y * a.W + cc) * 10);
        const uint32_t w[8] = {src[0], src[1], src[2], src[3], src[4], 0u, 0u, 0u};
        put<COST, ND>(dst, w);
    } else if constexpr (COST == COST_SAD4) {
        // rows y-r .. y+r+3 (j = 0 .. 2r+3): j in [3, 2r] -> common word (j-3)/4; the 3
        // rows of output q outside the common block -> byte positions of word ND+q
        constexpr int NC = PackCfg<COST, ND>::NW - 4;
        uint32_t w[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
        const int r = ND;
        for (int j = 0; j <= 2 * r + 3; ++j) {
            const int yy = clampi(y - r + j, 0, a.H - 1);
            const uint32_t v = img[(size_t)yy * a.pitch + cc];
            if (j >= 3 && j <= 2 * r) {
                const int q = (j - 3) >> 2;
                const uint32_t sh = v << (8 * ((j - 3) & 3));
#pragma unroll
                for (int i = 0; i < NC; ++i) w[i] |= q == i ? sh : 0u;
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                // custom rows of output q: j = q .. 2 (before the common block), then
                // j = 2r+1 .. 2r+q (after it); byte position = order within the 3
                const int pos = j <= 2 ? j - q : (j >= 2 * r + 1 ? (3 - q) + (j - 2 * r - 1) : -1);
                const bool in = j <= 2 ? (j >= q) : (j >= 2 * r + 1 && j <= 2 * r + q);
                w[NC + q] |= in ? v << (8 * pos) : 0u;
            }
        }
        put<COST, ND>(dst, w);
    } else {
        uint32_t w[5] = {0u, 0u, 0u, 0u, 0u};
        uint32_t sq = 0;
        for (int j = 0; j < a.win; ++j) {
            const int yy = clampi(y - a.r + j, 0, a.H - 1);
            const uint32_t v = img[(size_t)yy * a.pitch + cc];
            sq += v * v;
            const uint32_t sh = v << (8 * (j & 3));
            const int q = j >> 2;
            w[0] |= q == 0 ? sh : 0u;
            w[1] |= q == 1 ? sh : 0u;
            w[2] |= q == 2 ? sh : 0u;
            w[3] |= q == 3 ? sh : 0u;
        }
        if constexpr (COST == COST_SSD) w[ND] = sq;
        const uint32_t o[8] = {w[0], w[1], w[2], w[3], w[4], 0u, 0u, 0u};
        put<COST, ND>(dst, o);
    }
}

// ---- vectorised pack building: one lane = 4 consecutive in-bounds columns -------------
// Each window row is read as ONE dword (4 columns) and 4 rows x 4 columns are transposed
// with v_perm_b32 into the 4 columns' pack words (8 perms per 16 bytes), instead of one
// clamped byte load + shift/select chain per (row, column).
__device__ __forceinline__ void transpose4(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t (&o)[4]) {
    const uint32_t t0 = __builtin_amdgcn_perm(b, a, 0x05010400u);   // a0 b0 a1 b1
    const uint32_t t1 = __builtin_amdgcn_perm(b, a, 0x07030602u);   // a2 b2 a3 b3
    const uint32_t t2 = __builtin_amdgcn_perm(d, c, 0x05010400u);   // c0 d0 c1 d1
    const uint32_t t3 = __builtin_amdgcn_perm(d, c, 0x07030602u);   // c2 d2 c3 d3
    o[0] = __builtin_amdgcn_perm(t2, t0, 0x05040100u);              // a0 b0 c0 d0
    o[1] = __builtin_amdgcn_perm(t2, t0, 0x07060302u);
    o[2] = __builtin_amdgcn_perm(t3, t1, 0x05040100u);
    o[3] = __builtin_amdgcn_perm(t3, t1, 0x07060302u);
}

// 4-row kind: the pack words of 4 columns from their 2r+4 window rows (one dword = the 4
// columns of a row, rows y-r .. y+r+3); same layout as build_pack.
template <int R>
__device__ __forceinline__ void sad4_group_words(const uint32_t (&rw)[2 * R + 4],
                                                 uint32_t (&w)[PackCfg<COST_SAD4, R>::NW][4]) {
    constexpr int NC = PackCfg<COST_SAD4, R>::NW - 4, NCR = 2 * R - 2;
#pragma unroll
    for (int m = 0; m < NC; ++m) {
        uint32_t d[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) d[t] = 4 * m + t < NCR ? rw[3 + 4 * m + t] : 0u;
        transpose4(d[0], d[1], d[2], d[3], w[m]);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        uint32_t d[3];
        int n = 0;
#pragma unroll
        for (int j = q; j <= 2; ++j) d[n++] = rw[j];
#pragma unroll
        for (int j = 2 * R + 1; j <= 2 * R + q; ++j) d[n++] = rw[j];
        transpose4(d[0], d[1], d[2], 0u, w[NC + q]);
    }
}

// Pack words of the 4 columns cg..cg+3 (all inside [0, W), 4-byte aligned rows) around
// output row y; same layout as build_pack.
template <int COST, int ND>
__device__ __forceinline__ void build_group(const MatchParams& a, const uint8_t* img, int cg, int y,
                                            uint32_t (&w)[PackCfg<COST, ND>::NW][4]) {
    const int r = COST == COST_SAD4 ? ND : a.r;
    auto row = [&](int j) -> uint32_t {
        const int yy = clampi(y - r + j, 0, a.H - 1);
        return *reinterpret_cast<const uint32_t*>(img + (size_t)yy * a.pitch + cg);
    };
    if constexpr (COST == COST_SAD4) {
        uint32_t rw[2 * ND + 4];
#pragma unroll
        for (int j = 0; j < 2 * ND + 4; ++j) rw[j] = row(j);
        sad4_group_words<ND>(rw, w);
        return;
    }
    const int nsh = a.win;                                   // transposed rows
#pragma unroll
    for (int q = 0; q < ND; ++q) {
        uint32_t d[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) d[t] = (4 * q + t < nsh) ? row(4 * q + t) : 0u;
        transpose4(d[0], d[1], d[2], d[3], w[q]);
    }
    if constexpr (COST == COST_SSD) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            uint32_t sq = 0u;
#pragma unroll
            for (int q = 0; q < ND; ++q) sq = __builtin_amdgcn_udot4(w[q][k], w[q][k], sq, false);
            w[ND][k] = sq;
        }
    }
}

// Logical right-pack index i -> LDS slot: one empty slot after every DPL packs, phased by
// c0 so that every DPL-step chunk of a lane's "entering column" reads is DPL consecutive
// slots (static ds_read offsets) and the 16 lanes of a group, DPL packs apart, land DPL+1
// slots apart (DPL+1 odd -> distinct 16-byte bank groups for ds_read_b128).
__device__ __forceinline__ int rslot(int i, int c0, int dpl) { return i + (i + c0) / dpl; }

// All column packs of one wave: L packs i -> column cL0 + i (slot i), R packs i -> column
// cR0 + i (slot rslot(i)).  Interior 4-column groups take the vectorised path; groups
// touching the image border (replicate clamp), HOG, and unaligned images take build_pack.
template <int COST, int ND, int DPL>
__device__ __forceinline__ void build_all_packs(const MatchParams& a, int y, int cL0, int NL, int cR0,
                                                int NRlog, int c0, PackOut<COST, ND> Lp,
                                                PackOut<COST, ND> Rp, int lane) {
    constexpr int NW = PackCfg<COST, ND>::NW;
    bool aligned = ((reinterpret_cast<uintptr_t>(a.L) | reinterpret_cast<uintptr_t>(a.R) |
                     (uintptr_t)a.pitch) & 3u) == 0;
    if constexpr (COST == COST_HOG) aligned = false;
    if (!aligned) {
        for (int i = lane; i < NL; i += 64) build_pack<COST, ND>(a, a.L, a.HL, cL0 + i, y, Lp + i);
        for (int i = lane; i < NRlog; i += 64)
            build_pack<COST, ND>(a, a.R, a.HR, cR0 + i, y, Rp + rslot(i, c0, DPL));
        return;
    }
    if constexpr (COST != COST_HOG) {
    const int aL = cL0 & ~3, aR = cR0 & ~3;                  // floor to a multiple of 4
    const int gL = (cL0 + NL - aL + 3) >> 2, gR = (cR0 + NRlog - aR + 3) >> 2;
    for (int gi = lane; gi < gL + gR; gi += 64) {
        const bool right = gi >= gL;
        const int cg = right ? aR + 4 * (gi - gL) : aL + 4 * gi;
        const int cfirst = right ? cR0 : cL0, n = right ? NRlog : NL;
        const uint8_t* img = right ? a.R : a.L;
        const PackOut<COST, ND> base = right ? Rp : Lp;
        if (cg >= 0 && cg + 4 <= a.W) {
            uint32_t w[NW][4];
            build_group<COST, ND>(a, img, cg, y, w);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int idx = cg + k - cfirst;
                if (idx < 0 || idx >= n) continue;
                uint32_t v[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) v[i] = i < NW ? w[i < NW ? i : 0][k] : 0u;
                put<COST, ND>(base + (right ? rslot(idx, c0, DPL) : idx), v);
            }
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int idx = cg + k - cfirst;
                if (idx < 0 || idx >= n) continue;
                build_pack<COST, ND>(a, img, nullptr, cg + k, y, base + (right ? rslot(idx, c0, DPL) : idx));
            }
        }
    }
    }
}

// The ring kind's packs (4-row kind, radius R): as build_all_packs, but each lane issues
// the row loads of up to MF of its 4-column groups before it transposes any of them, so a
// wave waits for its global loads once per MF groups instead of once per group (the
// per-group form left ~8% of k_match's time in the segment prologue).  Groups touching the
// image border load from column 0 (unused) and take build_pack afterwards.
template <int R, int MF, int DPL>
__device__ __forceinline__ void build_ring_packs(const MatchParams& a, int y, int cL0, int NL, int cR0,
                                                 int NRlog, int c0, PackOut<COST_SAD4, R> Lp,
                                                 PackOut<COST_SAD4, R> Rp, int lane) {
    constexpr int NW = PackCfg<COST_SAD4, R>::NW, NRW = 2 * R + 4;
    const bool aligned = ((reinterpret_cast<uintptr_t>(a.L) | reinterpret_cast<uintptr_t>(a.R) |
                           (uintptr_t)a.pitch) & 3u) == 0;
    if (!aligned) {
        build_all_packs<COST_SAD4, R, DPL>(a, y, cL0, NL, cR0, NRlog, c0, Lp, Rp, lane);
        return;
    }
    const int aL = cL0 & ~3, aR = cR0 & ~3;                  // floor to a multiple of 4
    const int gL = (cL0 + NL - aL + 3) >> 2, gR = (cR0 + NRlog - aR + 3) >> 2;
    const int G = gL + gR;
    uint32_t roff[NRW];                                      // row offsets (wave-uniform)
#pragma unroll
    for (int j = 0; j < NRW; ++j) roff[j] = (uint32_t)clampi(y - R + j, 0, a.H - 1) * (uint32_t)a.pitch;
    for (int g0 = 0; g0 < G; g0 += 64 * MF) {
        uint32_t rw[MF][NRW];
#pragma unroll
        for (int m = 0; m < MF; ++m) {
            const int gi = g0 + lane + 64 * m;
            const bool right = gi >= gL;
            const int cg = right ? aR + 4 * (gi - gL) : aL + 4 * gi;
            const bool in = gi < G && cg >= 0 && cg + 4 <= a.W;
            const uint8_t* img = (right ? a.R : a.L) + (in ? cg : 0);
#pragma unroll
            for (int j = 0; j < NRW; ++j) rw[m][j] = *reinterpret_cast<const uint32_t*>(img + roff[j]);
        }
#pragma unroll
        for (int m = 0; m < MF; ++m) {
            const int gi = g0 + lane + 64 * m;
            if (gi >= G) continue;
            const bool right = gi >= gL;
            const int cg = right ? aR + 4 * (gi - gL) : aL + 4 * gi;
            const int cfirst = right ? cR0 : cL0, n = right ? NRlog : NL;
            const PackOut<COST_SAD4, R> base = right ? Rp : Lp;
            if (cg >= 0 && cg + 4 <= a.W) {
                uint32_t w[NW][4];
                sad4_group_words<R>(rw[m], w);
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int idx = cg + k - cfirst;
                    if (idx < 0 || idx >= n) continue;
                    uint32_t v[8];
#pragma unroll
                    for (int i = 0; i < 8; ++i) v[i] = i < NW ? w[i < NW ? i : 0][k] : 0u;
                    put<COST_SAD4, R>(base + (right ? rslot(idx, c0, DPL) : idx), v);
                }
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int idx = cg + k - cfirst;
                    if (idx < 0 || idx >= n) continue;
                    build_pack<COST_SAD4, R>(a, right ? a.R : a.L, nullptr, cg + k, y,
                                             base + (right ? rslot(idx, c0, DPL) : idx));
                }
            }
        }
    }
}

template <int COST, int ND, int DPL>
__device__ __forceinline__ void match_chunk(
    const int cut, const int dbits, PackPtr<COST, ND> rnb, PackPtr<COST, ND> rob, PackPtr<COST, ND> lnb,
    PackPtr<COST, ND> lob,
    Pk<PackCfg<COST, ND>::NW> (&rn)[DPL], Pk<PackCfg<COST, ND>::NW> (&ro)[DPL],
    uint32_t (&h)[DPL][PackCfg<COST, ND>::ROWS], const uint32_t (&mk)[DPL],
    uint32_t (&bk)[PackCfg<COST, ND>::ROWS][DPL]) {
    constexpr int NW = PackCfg<COST, ND>::NW;
    constexpr int ROWS = PackCfg<COST, ND>::ROWS;
    constexpr bool RUN = COST != COST_HOG;            // running horizontal window
    constexpr bool HI = hi_keys(COST, ND);            // dbits == 16 (plan_match)
#pragma unroll
    for (int u = 0; u < DPL; ++u) {
        // ring slot u receives this step's entering right column; its previous content
        // (k = DPL-1 of the last step) is dead.  Static offsets inside the chunk; `cut` is
        // the wave-uniform phase of the old ring's slot gap.
        rn[u] = ld<COST, ND>(rnb + u);
        const Pk<NW> L = ld<COST, ND>(lnb + u);
        Pk<NW> LO;
        if constexpr (RUN) {
            ro[u] = ld<COST, ND>(rob + (u + (u >= cut ? 1 : 0)));
            LO = ld<COST, ND>(lob + u);
        }
#pragma unroll
        for (int k = 0; k < DPL; ++k) {
            const int sk = (u - k + DPL) % DPL;
            if constexpr (HI) {
                // keys (cost << 16) | idx updated by v_sad_hi_u8, which adds (SAD << 16):
                // m = (old row-q SAD + old common - new common) << 16, then
                // h = h + (new row-q SAD << 16) - m: 2 v_sad + 1 v_sub per cell, 1 v_sub
                // per 4 cells (instead of 2 v_sad + v_sub + v_mad per cell)
                constexpr int NC = PackCfg<COST, ND>::NC;
                uint32_t cn = 0u, co = 0u;
#pragma unroll
                for (int i = 0; i < NC; ++i) {
                    cn = __builtin_amdgcn_sad_hi_u8(L.w[i], rn[sk].w[i], cn);
                    co = __builtin_amdgcn_sad_hi_u8(LO.w[i], ro[sk].w[i], co);
                }
                const uint32_t nch = co - cn;
#pragma unroll
                for (int q = 0; q < ROWS; ++q) {
                    const uint32_t m = __builtin_amdgcn_sad_hi_u8(LO.w[NC + q], ro[sk].w[NC + q], nch);
                    h[k][q] = __builtin_amdgcn_sad_hi_u8(L.w[NC + q], rn[sk].w[NC + q], h[k][q]) - m;
                }
                continue;
            }
            uint32_t vn[ROWS];
            ccol<COST, ND, NW>(L, rn[sk], vn);
            if constexpr (RUN) {
                // running keys: h = (window cost << dbits) + base; one shift-add per cell
                uint32_t vo[ROWS];
                ccol<COST, ND, NW>(LO, ro[sk], vo);
#pragma unroll
                for (int q = 0; q < ROWS; ++q) h[k][q] = shl_add(vn[q] - vo[q], 1 << dbits, h[k][q]);
            } else {
                h[k][0] = (vn[0] << dbits) | mk[k];
            }
        }
#pragma unroll
        for (int q = 0; q < ROWS; ++q) {
            uint32_t b = 0xFFFFFFFFu;
#pragma unroll
            for (int k = 0; k < DPL; ++k) b = min(b, h[k][q]);
            bk[q][u] = b;
        }
        // one scheduling region per step: without it hipcc hoists every step's LDS reads
        // to the top of the chunk and the register file doubles
        __builtin_amdgcn_sched_barrier(0);
    }
}

// Batched per-pixel reductions of one chunk, branch-free per LPG so the independent DPP
// chains interleave.
// The min lands in the group's LAST lane (every lane for LPG = 16): row_ror within 16-lane
// rows, then row_bcast:15 / row_bcast:31 across rows.
template <int LPG, int N>
__device__ __forceinline__ void reduce_batch(uint32_t* v) {
#define SV_ROR_STEP(CTRL)                                                                     \
    _Pragma("unroll") for (int i = 0; i < N; ++i)                                             \
        v[i] = min(v[i], (uint32_t)__builtin_amdgcn_update_dpp(0u, (int)v[i], CTRL, 0xF, 0xF, false));
    SV_ROR_STEP(0x121)  // row_ror:1
    SV_ROR_STEP(0x122)  // row_ror:2
    SV_ROR_STEP(0x124)  // row_ror:4
    SV_ROR_STEP(0x128)  // row_ror:8
#undef SV_ROR_STEP
    if constexpr (LPG >= 32) {
#pragma unroll
        for (int i = 0; i < N; ++i)
            v[i] = min(v[i], (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v[i], 0x142, 0xA, 0xF, false));
    }
    if constexpr (LPG == 64) {
#pragma unroll
        for (int i = 0; i < N; ++i)
            v[i] = min(v[i], (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)v[i], 0x143, 0xC, 0xF, false));
    }
}

// Reduce-scatter of 16 keys over the 16 lanes of a row (LPG = 16, ROWS * DPL = 16):
// on return lane l's v[0] is the min over the row of key index l.  Four butterfly steps
// with XOR partners 15, 7, 3, 1 (row_mirror, row_half_mirror, quad perms); at each step a
// lane keeps the half of its keys selected by the partner bit and sends the other half:
// 8+4+2+1 fused v_min_u32_dpp plus 2 selects each, instead of 16 x 4 row_ror steps.
__device__ __forceinline__ void reduce_scatter16(uint32_t (&v)[16], int l) {
#define SV_RS_STEP(HALF, BIT, CTRL)                                                            \
    {                                                                                          \
        const bool hi = (l & (BIT)) != 0;                                                      \
        _Pragma("unroll") for (int k = 0; k < (HALF); ++k) {                                   \
            const uint32_t send = hi ? v[k] : v[k + (HALF)];                                   \
            const uint32_t keep = hi ? v[k + (HALF)] : v[k];                                   \
            v[k] = min(keep, (uint32_t)__builtin_amdgcn_update_dpp(0u, (int)send, CTRL, 0xF, 0xF, false)); \
        }                                                                                      \
    }
    SV_RS_STEP(8, 8, 0x140)   // row_mirror:      partner l ^ 15
    SV_RS_STEP(4, 4, 0x141)   // row_half_mirror: partner l ^ 7
    SV_RS_STEP(2, 2, 0x1B)    // quad_perm 3210:  partner l ^ 3
    SV_RS_STEP(1, 1, 0xB1)    // quad_perm 1032:  partner l ^ 1
#undef SV_RS_STEP
}

// reduce_scatter16 with the first two butterfly steps as bank-masked DPP: the partner bit of
// those steps (lane bit 3, then bit 2) is a DPP bank bit, so a lane's keep/send choice is
// made by which lanes an instruction writes (bank_mask) instead of two v_cndmask per pair:
// 2 v_min_u32_dpp per pair instead of 1 + 2 selects (33 ops instead of 45 for 16 keys).
// Inline asm because the masked write must preserve the disabled lanes' destination; each
// block starts with s_nop 1 (VALU write -> DPP read of the same VGPR needs 2 wait states).
__device__ __forceinline__ void reduce_scatter16_bm(uint32_t (&v)[16], int l) {
#define SV_BM_PAIR(A, B, CTRL, M0, M1)                                                          \
    "v_min_u32_dpp %" #A ", %" #A ", %" #A " " CTRL " row_mask:0xf bank_mask:" M0 "\n\t"      \
    "v_min_u32_dpp %" #A ", %" #B ", %" #B " " CTRL " row_mask:0xf bank_mask:" M1 "\n\t"
    // step 1, row_mirror (partner 15 - l): lanes 0-7 (banks 0,1) keep v[k], lanes 8-15 v[k+8]
    asm volatile("s_nop 1\n\t"
                 SV_BM_PAIR(0, 8, "row_mirror", "0x3", "0xc") SV_BM_PAIR(1, 9, "row_mirror", "0x3", "0xc")
                 SV_BM_PAIR(2, 10, "row_mirror", "0x3", "0xc") SV_BM_PAIR(3, 11, "row_mirror", "0x3", "0xc")
                 SV_BM_PAIR(4, 12, "row_mirror", "0x3", "0xc") SV_BM_PAIR(5, 13, "row_mirror", "0x3", "0xc")
                 SV_BM_PAIR(6, 14, "row_mirror", "0x3", "0xc") SV_BM_PAIR(7, 15, "row_mirror", "0x3", "0xc")
                 : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7])
                 : "v"(v[8]), "v"(v[9]), "v"(v[10]), "v"(v[11]), "v"(v[12]), "v"(v[13]), "v"(v[14]), "v"(v[15]));
    // step 2, row_half_mirror (partner l ^ 7): bit-2-clear lanes (banks 0,2) keep v[k]
    asm volatile("s_nop 1\n\t"
                 SV_BM_PAIR(0, 4, "row_half_mirror", "0x5", "0xa") SV_BM_PAIR(1, 5, "row_half_mirror", "0x5", "0xa")
                 SV_BM_PAIR(2, 6, "row_half_mirror", "0x5", "0xa") SV_BM_PAIR(3, 7, "row_half_mirror", "0x5", "0xa")
                 : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3])
                 : "v"(v[4]), "v"(v[5]), "v"(v[6]), "v"(v[7]));
#undef SV_BM_PAIR
#define SV_RS_STEP(HALF, BIT, CTRL)                                                            \
    {                                                                                          \
        const bool hi = (l & (BIT)) != 0;                                                      \
        _Pragma("unroll") for (int k = 0; k < (HALF); ++k) {                                   \
            const uint32_t send = hi ? v[k] : v[k + (HALF)];                                   \
            const uint32_t keep = hi ? v[k + (HALF)] : v[k];                                   \
            v[k] = min(keep, (uint32_t)__builtin_amdgcn_update_dpp(0u, (int)send, CTRL, 0xF, 0xF, false)); \
        }                                                                                      \
    }
    SV_RS_STEP(2, 2, 0x1B)    // quad_perm 3210:  partner l ^ 3
    SV_RS_STEP(1, 1, 0xB1)    // quad_perm 1032:  partner l ^ 1
#undef SV_RS_STEP
}

// Reduce-scatter of 8 keys over the 16 lanes of a row: on return lanes 2j and 2j+1 hold the
// min over the row of key j = (l >> 1) & 7 in v[0].  Bank-masked DPP for lane bits 3 and 2,
// selects for bit 1, then one all-reduce step with lane l ^ 1: 16 ops for 8 keys.
__device__ __forceinline__ void reduce_scatter8_bm(uint32_t (&v)[8], int l) {
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

// Occupancy target: LDS admits ~3 blocks/CU for the common configs (D <= 128, win <= 11),
// so cap registers at 3 waves/SIMD (<= 168 VGPRs); the widest packs get 2 waves/SIMD.
template <int COST, int ND> struct Occ {
    static constexpr int W = COST == COST_SAD4 ? 2 : (COST == COST_SAD || ND <= 3) ? 3 : 2;
};

template <int COST, int ND, int DPL>
__global__ __launch_bounds__((64 * PackCfg<COST, ND>::WPB), (Occ<COST, ND>::W)) void k_match(MatchParams a) {
    constexpr int NW = PackCfg<COST, ND>::NW;
    constexpr int ROWS = PackCfg<COST, ND>::ROWS;
    extern __shared__ __attribute__((aligned(16))) uint4 smem[];
    if (blockIdx.z) {   // frame batch
        a.L += blockIdx.z * a.fs_in;
        a.R += blockIdx.z * a.fs_in;
        a.out += blockIdx.z * a.fs_out;
        if constexpr (COST == COST_HOG) {
            a.HL += blockIdx.z * a.fs_hist;
            a.HR += blockIdx.z * a.fs_hist;
        }
    }
    const int lane = threadIdx.x & 63;
    const int wid = PackCfg<COST, ND>::WPB == 1 ? 0 : (int)(threadIdx.x >> 6);
    const int LPG = a.lpg;
    const int S = seg_width(LPG, DPL, a.segm);      // segment width per group
    const int WC = wave_cols(LPG, DPL, a.segm);
    const int r = a.r;
    const int W2 = 2 * r + 1;
    const int c0 = (DPL - (4 * r + 1) % DPL) % DPL;      // (iR0 + W2 + c0) % DPL == 0
    const int NL = WC + 4 * r + DPL + 1;
    const int NRlog = WC + 4 * r + LPG * DPL + DPL;
    const int NRphys = NRlog + (NRlog + c0) / DPL + 1;
    // per-wave LDS region: [L main | R main | L common | R common] (common arrays: SPLIT)
    using P = PackCfg<COST, ND>;
    uint4* wbase = reinterpret_cast<uint4*>(reinterpret_cast<char*>(smem) + (size_t)wid * (NL + NRphys) * P::SLOT_BYTES);
    typename P::CT* cbase = reinterpret_cast<typename P::CT*>(wbase + (size_t)(NL + NRphys) * P::QX);
    const PackOut<COST, ND> Lw{wbase, cbase};
    const PackOut<COST, ND> Rw{wbase + (size_t)NL * P::QX, cbase + NL};
    const PackPtr<COST, ND> Lp{Lw.x, Lw.c};
    const PackPtr<COST, ND> Rp{Rw.x, Rw.c};

    const int y = a.row0 + ((int)blockIdx.y * PackCfg<COST, ND>::WPB + wid) * ROWS;
    const int yc = min(y, a.row1 - 1);
    const int xw = a.X0 + (int)blockIdx.x * WC;
    const int cL0 = xw - 3 * r - 1;
    const int cR0 = cL0 - a.minD - (LPG * DPL - 1);

    build_all_packs<COST, ND, DPL>(a, yc, cL0, NL, cR0, NRlog, c0, Lw, Rw, lane);

    if (blockIdx.x == 0) {  // columns outside the matched band are invalid
        const int16_t inv = (int16_t)((a.minD - 1) * 16);
#pragma unroll
        for (int q = 0; q < ROWS; ++q) {
            if (y + q >= a.row1) break;
            int16_t* orow = a.out + (size_t)(y + q) * a.opitch;
            for (int x = lane; x < a.X0; x += 64) orow[x] = inv;
            for (int x = a.X1 + lane; x < a.W; x += 64) orow[x] = inv;
        }
    }
    __syncthreads();
    if (y >= a.row1) return;

    const int g = lane >> a.lpg_log2;
    const int l = lane & (LPG - 1);
    // disparity slot of the lane inside its group: lanes of odd 16-lane rows are rotated by
    // 8, which makes the per-step right-pack ds_read_b128 conflict-free across the two
    // groups that share a b128 lane group (the min over a group does not depend on the
    // order; emission uses the physical lane)
    const int sl = l ^ (((lane >> 4) & 1) << 3);
    const int xs = xw + g * S;
    const int iL0 = g * S + 2 * r + 1;                   // L index of the window's first column
    const int iR0 = g * S + 2 * r + (LPG - sl) * DPL;  // R index of (first column, k = 0)
    const uint32_t dmask = (1u << a.dbits) - 1u;
    const int dbits = a.dbits;
    const int j = l - (LPG - 16);                        // emitting lane -> step within a chunk

    // argmin keys (cost << dbits) | idx.  Running kinds keep the key itself in h, starting
    // from its base: idx, or for padding disparities (idx >= D) idx + (cmax + 1) << dbits so
    // they can never win (plan_match checks the range).  HOG forms keys with mk.
    uint32_t mk[DPL];
    uint32_t h[DPL][ROWS], bk[ROWS][DPL];
#pragma unroll
    for (int k = 0; k < DPL; ++k) {
        const int idx = sl * DPL + k;
        mk[k] = idx < a.D ? (uint32_t)idx : 0xFFFFFFFFu;
#pragma unroll
        for (int q = 0; q < ROWS; ++q) h[k][q] = idx < a.D ? (uint32_t)idx : a.pad_key | (uint32_t)idx;
    }

    // ---- prologue: window of output column xs = the W2 columns xs-r .. xs+r, added directly
    for (int t = 0; t < W2; ++t) {
        const Pk<NW> L = ld<COST, ND>(Lp + (iL0 + t));
#pragma unroll
        for (int k = 0; k < DPL; ++k) {
            uint32_t vn[ROWS];
            ccol<COST, ND, NW>(L, ld<COST, ND>(Rp + rslot(iR0 + t - k, c0, DPL)), vn);
            if constexpr (COST == COST_HOG) h[k][0] = (vn[0] << dbits) | mk[k];
            else {
#pragma unroll
                for (int q = 0; q < ROWS; ++q) h[k][q] += vn[q] << dbits;
            }
        }
    }
    {
        const bool emit0 = j == 0 && xs < a.X1;
#pragma unroll
        for (int q = 0; q < ROWS; ++q) {
            uint32_t b = 0xFFFFFFFFu;
#pragma unroll
            for (int k = 0; k < DPL; ++k) b = min(b, h[k][q]);
            if (LPG == 16) reduce_batch<16, 1>(&b);
            else if (LPG == 32) reduce_batch<32, 1>(&b);
            else reduce_batch<64, 1>(&b);
            if (emit0 && y + q < a.row1)
                a.out[(size_t)(y + q) * a.opitch + xs] = (int16_t)(((int)(b & dmask) + a.minD) * 16);
        }
    }

    // ---- main loop: step t' adds column xs+r+1+t' and drops column xs-r+t' (output
    // xs+1+t'), in chunks of DPL steps with static ring slots and static LDS offsets.
    // c0 aligns chunk starts with the right-pack slot gaps (see rslot); the leaving
    // column's reads trail by W2 packs, so their gap phase is (-W2) mod DPL for every lane.
    const int phi = (DPL - W2 % DPL) % DPL;
    const int cut = DPL - phi;                           // old slot offsets u >= cut skip a gap
    const int iN = iR0 + W2;                             // R index of the entering column, t' = 0
    Pk<NW> rn[DPL], ro[DPL];
#pragma unroll
    for (int s = 1; s < DPL; ++s) {                      // virtual steps t' = s - DPL
        rn[s] = ld<COST, ND>(Rp + rslot(iN - (DPL - s), c0, DPL));
        if constexpr (COST != COST_HOG) ro[s] = ld<COST, ND>(Rp + rslot(iR0 - (DPL - s), c0, DPL));
    }
    const PackPtr<COST, ND> rn0 = Rp + rslot(iN, c0, DPL);
    const PackPtr<COST, ND> ro0 = Rp + rslot(iR0, c0, DPL);
    const PackPtr<COST, ND> ln0 = Lp + (iL0 + W2);
    const PackPtr<COST, ND> lo0 = Lp + iL0;
    const int T = (S - 1 + DPL - 1) / DPL * DPL;

    for (int t0 = 0, c = 0; t0 < T; t0 += DPL, ++c) {
        match_chunk<COST, ND, DPL>(cut, dbits, rn0 + c * (DPL + 1), ro0 + c * (DPL + 1), ln0 + t0, lo0 + t0, rn,
                                   ro, h, mk, bk);
        if constexpr (ROWS * DPL == 16 || ROWS * DPL == 32) {
            if (LPG == 16) {   // reduce-scatter: lane l ends with key (row l / DPL, step l % DPL)
#pragma unroll
                for (int half = 0; half < ROWS * DPL / 16; ++half) {
                    uint32_t v[16];
#pragma unroll
                    for (int i = 0; i < 16; ++i) v[i] = bk[(16 * half + i) / DPL][i % DPL];
                    reduce_scatter16(v, l);
                    const int q = (16 * half) / DPL + l / DPL, e = t0 + l % DPL + 1, x = xs + e;
                    if (e < S && x < a.X1 && y + q < a.row1)
                        a.out[(size_t)(y + q) * a.opitch + x] = (int16_t)(((int)(v[0] & dmask) + a.minD) * 16);
                }
                continue;
            }
        }
        if constexpr (ROWS * DPL == 8) {
            // 8 keys (HOG, 1-row SAD/SSD with DPL 8, 2-row SAD2 with DPL 4): bank-masked
            // reduce-scatter over each 16-lane row, then the rows of a group joined by
            // permlane swaps; lanes 2i of the group's first row emit key i
            uint32_t v[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = bk[i / DPL][i % DPL];
            reduce_scatter8_bm(v, lane & 15);
            uint32_t key = v[0];
            if (LPG >= 32) {
                const auto p = __builtin_amdgcn_permlane16_swap(key, key, false, false);
                key = min(p[0], p[1]);
            }
            if (LPG == 64) {
                const auto p = __builtin_amdgcn_permlane32_swap(key, key, false, false);
                key = min(p[0], p[1]);
            }
            const int i = (l >> 1) & 7, q = i / DPL, e = t0 + i % DPL + 1, x = xs + e;
            if (l < 16 && (l & 1) == 0 && e < S && x < a.X1 && y + q < a.row1)
                a.out[(size_t)(y + q) * a.opitch + x] = (int16_t)(((int)(key & dmask) + a.minD) * 16);
            continue;
        }
        const int e = t0 + j + 1;
        const int x = xs + e;
        const bool emit = j >= 0 && j < DPL && e < S && x < a.X1;
        // ROWS*DPL independent group reductions (ILP instead of a serial DPP chain per step)
        if (LPG == 16) reduce_batch<16, ROWS * DPL>(&bk[0][0]);
        else if (LPG == 32) reduce_batch<32, ROWS * DPL>(&bk[0][0]);
        else reduce_batch<64, ROWS * DPL>(&bk[0][0]);
#pragma unroll
        for (int q = 0; q < ROWS; ++q) {
            uint32_t v = bk[q][0];
#pragma unroll
            for (int u = 1; u < DPL; ++u) v = (j == u) ? bk[q][u] : v;
            if (emit && y + q < a.row1)
                a.out[(size_t)(y + q) * a.opitch + x] = (int16_t)(((int)(v & dmask) + a.minD) * 16);
        }
    }
}

// ---- ring kind: SAD, four rows per lane, win 5..11 (r 2..5) -----------------------------
// k_match's four-row kind recomputes the LEAVING column's cost at every step (12 v_sad_hi per
// 4 cells).  Here each lane owns RG_DPL = 4 consecutive disparities and keeps the entering
// column's four row costs (hi-shifted, as in the key) in a register ring of W2 = 2r+1 steps,
// so the leaving column's costs are read back instead of recomputed: a step costs 6 v_sad_hi
// + 4 v_sad_u32 per 4 cells (key = |key - leaving| + entering; r 5 on 16/64-lane groups: 4
// v_sub + 4 v_add).  Both rings (the M-slot cost ring and the 4-deep right pack ring) have
// static register indices inside a body of lcm(4, M) unrolled steps.
// The first 2r steps of a segment fill the window (ring starts at zero) and emit nothing.
// Keys are (cost << 16) | idx; padding disparities (idx >= D)
// start at cost 0x8000, above every real window cost (<= 121*255 = 30855 for win 11).
constexpr int RG_DPL = 4;

// two u16 lanes of a word (v_pk_add_u16 / v_pk_sub_u16, wrapping mod 2^16)
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_add16(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, a) + __builtin_bit_cast(u16x2, b));
}
__device__ __forceinline__ uint32_t pk_sub16(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, a) - __builtin_bit_cast(u16x2, b));
}


// DEFER: a chunk's second step pair is not reduced at the chunk's end (where its DPP /
// permlane chain ran alone before the next basic block) but in the next chunk's step 1,
// beside that chunk's first pair: two independent reduce-scatter chains interleaved, +9
// loop-carried VGPRs (off for r 5, which would spill).
// KEYS (split ring, D > 256): the reduced argmin keys (cost << 16 | idx) go to a.keys as u32
// (the merge kernel picks the smaller of the two passes' keys), no band-edge fill.
// SSD (r <= 4): the same packs and ring with squared differences, Σ(L-R)² = ΣL² + ΣR² - 2ΣLR
// over each output row's window column: v_dot4_u32_u8 on the common and per-row words (the
// packs' zero bytes add nothing), ΣL² once per step, ΣR² per disparity slot; the column cost
// enters pre-shifted by dbits, (ΣL² + ΣR²) << dbits - ΣLR << (dbits + 1) by one
// v_mad_i32_i24, and the window update is the same v_sad_u32.
template <int R, int LPGT, bool DEFER, bool KEYS, bool SSD = false>
__global__ __launch_bounds__(64, 2) void k_match_ring(MatchParams a) {
    using P = PackCfg<COST_SAD4, R>;
    constexpr int NW = P::NW, NC = P::NC, W2 = 2 * R + 1;
    // PK (r 6..7): window and column costs of rows 2j, 2j+1 share a register as two u16
    // (a window costs at most 57375), updated with v_pk_add/sub_u16: 15 ring steps x 16
    // cells fit in 120 VGPRs; the argmin keys (cost << 16) | idx are built per step
    constexpr bool PK = R >= 6;
    static_assert(P::SPLIT && (P::CW == 3) == PK, "ring kind expects split packs (20 B for r 2..3, 24 B for r 4..5, 28 B for r 6..7)");
    extern __shared__ __attribute__((aligned(16))) uint4 smem[];
    // XCD-aware tile order (sv_xcd.h): horizontal and vertical neighbours share 2r of their
    // 2r+4 input rows and most right-image columns; each XCD takes a contiguous tile range
    int bx, by, bz;
    xcd_tile(a.xcd_map != 0, bx, by, bz);
    if (bz) {   // frame batch
        a.L += bz * a.fs_in;
        a.R += bz * a.fs_in;
        a.out += bz * a.fs_out;
        if constexpr (KEYS) a.keys += bz * a.fs_out;
    }
    const int lane = threadIdx.x;
    constexpr int LPG = LPGT;                           // lanes per group (template: no
                                                        // branches between the steps)
    const int S = a.segm;                               // segment width per group (multiple of 4)
    const int WC = (64 / LPG) * S;
    // SADU (r <= 4): the window update is ONE v_sad_u32 (key - leaving + entering), which
    // reads the leaving column's cost after the entering one is computed, so the two cannot
    // share a register: the cost ring gets M = W2 + 1 slots (the entering cost goes to the
    // slot whose value left the window one step earlier) and keeps static register names.
    // r 5: the 16 more ring VGPRs first spilled 4-9 VGPRs to scratch (1080p D=128 win 11:
    // 572 -> 555 us per 16 frames with 32-lane groups, VGA D=64 win 11 122 -> 139 us with
    // 16-lane ones); without the left-pack prefetch (LPF) every group width fits in 252-255.
    // r 6..7 (packed halves) take it too: 16 / 14 slots of 8 words.
    // PK: the two u16 halves of a cost word update as ONE 32-bit v_sad_u32 as well: each half
    // of the key holds its leaving cost as a summand, so key >= leaving as 32-bit integers with
    // no borrow between the halves, and key - leaving + entering stays below 2^16 per half (no
    // carry): the packed result is exact.
    constexpr bool SADU = PK || R <= 5;
    constexpr int M = SADU ? W2 + 1 : W2;               // cost ring slots
    constexpr int U = M % 4 == 0 ? M : M % 2 == 0 ? 2 * M : 4 * M;   // lcm(4, M) steps per body
    constexpr int NCH = U / 4;                          // chunks per body
    // steps per segment: S outputs + 2r warm-up, in chunks of 4; whole bodies of U steps,
    // the first body entered at chunk e0 (its first e0 chunks skipped)
    const int Tn = (S + 2 * R + 3) & ~3;
    const int nit = (Tn + U - 1) / U;
    const int e0 = (nit * U - Tn) >> 2;
    const int NL = WC - S + Tn + 1;                      // + the L prefetch past the last step
    const int NRlog = WC - S + Tn + 4 * LPG;
    constexpr int c0 = 1;                               // chunk starts (index = 3 mod 4) meet slot gaps
    const int NRphys = NRlog + (NRlog + c0) / RG_DPL + 1;
    uint4* wbase = smem;
    typename P::CT* cbase = reinterpret_cast<typename P::CT*>(wbase + (size_t)(NL + NRphys));
    const PackOut<COST_SAD4, R> Lw{wbase, cbase};
    const PackOut<COST_SAD4, R> Rw{wbase + NL, cbase + NL};
    const PackPtr<COST_SAD4, R> Lp{Lw.x, Lw.c};
    const PackPtr<COST_SAD4, R> Rp{Rw.x, Rw.c};

    const int y = a.row0 + by * 4;
    const int yc = min(y, a.row1 - 1);
    const int xw = a.X0 + bx * WC;
    const int cL0 = xw - R;                             // L index i -> column cL0 + i
    const int cR0 = cL0 - a.minD - (4 * LPG - 1);       // R index i -> column cR0 + i
    build_ring_packs<R, 3, RG_DPL>(a, yc, cL0, NL, cR0, NRlog, c0, Lw, Rw, lane);

    if (!KEYS && bx == 0) {  // columns outside the matched band are invalid
        const int16_t inv = (int16_t)((a.minD - 1) * 16);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (y + q >= a.row1) break;
            int16_t* orow = a.out + (size_t)(y + q) * a.opitch;
            for (int x = lane; x < a.X0; x += 64) orow[x] = inv;
            for (int x = a.X1 + lane; x < a.W; x += 64) orow[x] = inv;
        }
    }
    __syncthreads();
    if (y >= a.row1) return;

    const int g = lane / LPG;
    const int l = lane & (LPG - 1);
    const int xs = xw + g * S;                          // first output column of the segment
    // step t enters column xs - r + t; lane l, disparity idx 4l + k reads R index iR0 + t - k
    // r <= 5: padding disparities (idx >= D) start at cost 0x8000, above any real window.
    // r 6..7 (window costs up to 57375, no headroom; D a multiple of 4): padding lanes
    // re-match the last real group D-4..D-1 under their own, larger labels, so on equal
    // costs the real lane wins every tie
    const int dl = PK ? min(4 * l, a.D - 4) : 4 * l;
    const int iR0 = g * S + 4 * (LPG - 1) - dl + 3;
    constexpr int RQ = PK ? 2 : 4;                      // cost words per k (h and ring slots)
    uint32_t h[RG_DPL][RQ], lab[RG_DPL];
#pragma unroll
    for (int k = 0; k < RG_DPL; ++k) {
        const int idx = 4 * l + k;
        const uint32_t base = PK ? 0u : idx < a.D ? (uint32_t)idx : (SSD ? a.pad_key : 0x8000u << 16) | (uint32_t)idx;
        lab[k] = (uint32_t)idx;
#pragma unroll
        for (int q = 0; q < RQ; ++q) h[k][q] = base;
    }
    uint32_t ring[M][RG_DPL][RQ];
#pragma unroll
    for (int s = 0; s < M; ++s)
#pragma unroll
        for (int k = 0; k < RG_DPL; ++k)
#pragma unroll
            for (int q = 0; q < RQ; ++q) ring[s][k][q] = 0u;
    Pk<NW> rn[RG_DPL];
#pragma unroll
    for (int s = 1; s < RG_DPL; ++s) rn[RG_DPL - s] = ld<COST_SAD4, R, true>(Rp + rslot(iR0 - s, c0, RG_DPL));
    // pointers of body position 0 (chunk e0 of the first body is step 0; the skipped chunks'
    // offsets are never dereferenced)
    PackPtr<COST_SAD4, R> rb = Rp + (rslot(iR0, c0, RG_DPL) - e0 * (RG_DPL + 1));
    PackPtr<COST_SAD4, R> lb = Lp + (g * S - 4 * e0);
    // LPF: the left pack is loaded one step ahead (off for r 5 + SADU, whose 32-lane body is
    // 4 VGPRs over the 256 a wave of two per SIMD may hold: the 6 registers of the prefetched
    // pack take its spills out of the loop)
    constexpr bool LPF = !(R == 5 && SADU);
    Pk<NW> Lnext = ld<COST_SAD4, R, true>(lb + 4 * e0);
    // after the reduce-scatter lane l's key is (row jq, step ju) of the chunk; the first 16
    // lanes of a group emit
    // (32-bit per-lane state only: output offset of step 0 and the emit window)
    const int jq = (lane >> 2) & 3, ju = (lane >> 1) & 1;   // key (l >> 1) & 7 = 2 jq + ju
    // 32-lane groups (D 65..128) join the two DPP rows of a chunk's two step pairs with ONE
    // v_permlane16_swap of the pairs' keys (instead of a mov + swap + min per pair): the
    // rows then hold different pairs, and both rows emit.  Which row receives which pair is
    // read off the swap itself once (pofs = the step offset of the lane's pair in its chunk,
    // folded into eb).  64-lane groups (D 129..256) do the same and then join the wave's
    // halves with one v_permlane32_swap; rows 0 and 1 emit.  (r 5 fits it since LPG is a
    // template parameter and the body has no branches: 244 VGPRs; with a runtime LPG and
    // branches around the reductions the allocator spilled ~1,000.)
    constexpr bool join2 = LPG >= 32;
    int pofs = 0;
    if (join2) {
        const auto p = __builtin_amdgcn_permlane16_swap((uint32_t)lane, (uint32_t)lane + 64u, false, false);
        // min(p[0], p[1]) of a lane comes from the first operand's values iff both p[k] < 64
        pofs = (max(p[0], p[1]) < 64u) ? 0 : 2;
    }
    // step t emits column xs + t + eb (join2: the chunk starting at step t emits the lane's
    // pair at column xs + t + eb)
    const int eb = ju - 2 * R + pofs;
    constexpr int OB = KEYS ? 4 : 2;                        // bytes per output element
    const int ooff = OB * ((y + jq) * a.opitch + xs + eb);   // bytes
    // 32-bit buffer offsets from one SGPR descriptor (no 64-bit per-lane addresses to keep)
    const auto orsrc = KEYS ? __builtin_amdgcn_make_buffer_rsrc(a.keys, 0, 0x7FFFFFFF, 0x00020000)
                            : __builtin_amdgcn_make_buffer_rsrc(a.out, 0, 0x7FFFFFFF, 0x00020000);
    const int emax = ((l & 1) == 0 && l < (join2 ? 32 : 16) && y + jq < a.row1) ? max(0, min(S, a.X1 - xs)) : 0;

    // store of a reduced key for the chunk starting at step tt (join2) / of step tt
    auto emit_key = [&](uint32_t key, int tt) {
        // non-emitting lanes store past the buffer's range (dropped by the hardware bounds
        // check, as in composable_kernel): no exec-mask branch
        const int off = (unsigned)(tt + eb) < (unsigned)emax ? ooff + OB * tt : (int)0x80000000u;
        if constexpr (KEYS) __builtin_amdgcn_raw_buffer_store_b32(key, orsrc, off, 0, 0);
        else __builtin_amdgcn_raw_buffer_store_b16(
            (uint16_t)(((int)(key & (SSD ? (1u << a.dbits) - 1u : 0xFFFFu)) + a.minD) * 16), orsrc, off, 0, 0);
    };
    // join2: pair (0,1) in kA, pair (2,3) in kB: one swap joins both
    auto join_pairs = [&](uint32_t kA_, uint32_t kB_) {
        auto p = __builtin_amdgcn_permlane16_swap(kA_, kB_, false, false);
        uint32_t key = min(p[0], p[1]);
        if (LPG == 64) {   // rows 0 and 2 hold the same pair (1 and 3 the other)
            p = __builtin_amdgcn_permlane32_swap(key, key, false, false);
            key = min(p[0], p[1]);
        }
        return key;
    };
    auto join_rows = [&](uint32_t key) {   // !join2: a pair's key over the group's DPP rows
        if (LPG >= 32) {   // rows 0,1 (and 2,3) of the wave: min with lane ^ 16
            const auto p = __builtin_amdgcn_permlane16_swap(key, key, false, false);
            key = min(p[0], p[1]);
        }
        if (LPG == 64) {   // halves: min with lane ^ 32
            const auto p = __builtin_amdgcn_permlane32_swap(key, key, false, false);
            key = min(p[0], p[1]);
        }
        return key;
    };
    // DEFER state: the previous chunk's second pair (8 keys), its first pair's reduced key
    // and its first step (a first chunk has none: the sentinel step stores out of range)
    uint32_t dv[8], kA = 0xFFFFFFFFu;
    int tprev = -(1 << 24);
#pragma unroll
    for (int i = 0; i < 8; ++i) dv[i] = 0xFFFFFFFFu;

    // whole bodies of U = 4*W2 steps, no exits inside a body (an exit per chunk made LLVM
    // shuffle the rings); the first body skips its first e0 chunks by a uniform branch
    for (int it = 0, t0 = -4 * e0; it < nit; ++it) {
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch, t0 += 4) {
            if (t0 < 0) continue;            // the first body's skipped chunks (uniform)
            uint32_t bk[4][2];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                // the entering cost goes to `slot`, the leaving one (entered W2 steps ago)
                // is read from `oslot`
                const int slot = (4 * ch + u) % M, oslot = (4 * ch + u + 1) % M;
                // this step's packs: L (every k) and the entering right column (k = 0 only)
                rn[u] = ld<COST_SAD4, R, true>(rb + (ch * (RG_DPL + 1) + u));
                const Pk<NW> Lc = LPF ? Lnext : ld<COST_SAD4, R, true>(lb + (4 * ch + u));
                if constexpr (LPF) Lnext = ld<COST_SAD4, R, true>(lb + (4 * ch + u + 1));
                // SSD: ΣL² of this step's left pack per output row, pre-shifted by dbits
                uint32_t sqL[4];
                if constexpr (SSD) {
                    uint32_t sc = 0u;
#pragma unroll
                    for (int i = 0; i < NC; ++i) sc = __builtin_amdgcn_udot4(Lc.w[i], Lc.w[i], sc, false);
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        sqL[q] = __builtin_amdgcn_udot4(Lc.w[NC + q], Lc.w[NC + q], sc, false) << a.dbits;
                }
                // !SADU: the leaving column's costs need no LDS data: subtract them while the
                // loads are in flight; k = 0 (the fresh right pack) last
                if constexpr (!SADU) {
#pragma unroll
                    for (int k = 0; k < RG_DPL; ++k)
#pragma unroll
                        for (int q = 0; q < RQ; ++q)
                            h[k][q] = PK ? pk_sub16(h[k][q], ring[slot][k][q]) : h[k][q] - ring[slot][k][q];
                }
#pragma unroll
                for (int kk = 0; kk < RG_DPL; ++kk) {
                    const int k = RG_DPL - 1 - kk;
                    const Pk<NW>& Rk = rn[(u - k) & 3];
                    if constexpr (PK) {
                        // common rows once, in both halves; row 2j's sad in the low half,
                        // row 2j+1's in the high half
                        uint32_t cn = 0u;
#pragma unroll
                        for (int i = 0; i < NC; ++i) cn = __builtin_amdgcn_sad_u8(Lc.w[i], Rk.w[i], cn);
                        cn |= cn << 16;
#pragma unroll
                        for (int j = 0; j < 2; ++j) {
                            const uint32_t c = __builtin_amdgcn_sad_hi_u8(
                                Lc.w[NC + 2 * j + 1], Rk.w[NC + 2 * j + 1],
                                __builtin_amdgcn_sad_u8(Lc.w[NC + 2 * j], Rk.w[NC + 2 * j], cn));
                            if constexpr (SADU) sad_u32_acc(h[k][j], ring[oslot][k][j], c);
                            else h[k][j] = pk_add16(h[k][j], c);
                            ring[slot][k][j] = c;
                        }
                    } else if constexpr (SSD) {
                        uint32_t cn = 0u, sr = 0u;
#pragma unroll
                        for (int i = 0; i < NC; ++i) {
                            cn = __builtin_amdgcn_udot4(Lc.w[i], Rk.w[i], cn, false);
                            sr = __builtin_amdgcn_udot4(Rk.w[i], Rk.w[i], sr, false);
                        }
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            const uint32_t lr = __builtin_amdgcn_udot4(Lc.w[NC + q], Rk.w[NC + q], cn, false);
                            const uint32_t rr = __builtin_amdgcn_udot4(Rk.w[NC + q], Rk.w[NC + q], sr, false);
                            const uint32_t t = (rr << a.dbits) + sqL[q];
                            const uint32_t c = (uint32_t)__mul24((int)lr, -(2 << a.dbits)) + t;
                            sad_u32_acc(h[k][q], ring[oslot][k][q], c);
                            ring[slot][k][q] = c;
                        }
                    } else {
                        uint32_t cn = 0u;
#pragma unroll
                        for (int i = 0; i < NC; ++i) cn = __builtin_amdgcn_sad_hi_u8(Lc.w[i], Rk.w[i], cn);
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            const uint32_t c = __builtin_amdgcn_sad_hi_u8(Lc.w[NC + q], Rk.w[NC + q], cn);
                            // SADU: key - leaving + entering as ONE v_sad_u32 (|key - leaving|
                            // + entering): the key holds the leaving column's cost as one of
                            // its summands, so key >= leaving and the absolute value is the
                            // plain difference (one VOP3 instead of a VOP2 sub + add)
                            if constexpr (SADU) sad_u32_acc(h[k][q], ring[oslot][k][q], c);
                            else h[k][q] += c;
                            ring[slot][k][q] = c;
                        }
                    }
                }
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    uint32_t kq[RG_DPL];
#pragma unroll
                    for (int k = 0; k < RG_DPL; ++k)
                        kq[k] = !PK ? h[k][q] : (q & 1) ? (h[k][q >> 1] & 0xFFFF0000u) | lab[k] : (h[k][q >> 1] << 16) | lab[k];
                    bk[q][u & 1] = min(min(kq[0], kq[1]), min(kq[2], kq[3]));
                }
                __builtin_amdgcn_sched_barrier(0);
                // steps u-1, u: 8 keys (row q, step j) at v[2q + j].  Warm-up pairs are reduced
                // too (their keys are not emitted): no branch, so a chunk is one basic block and
                // the scheduler can interleave a reduction's DPP / permlane chain with the next
                // step's independent cost work
                if (DEFER && u == 3) {   // the second pair waits for the next chunk
#pragma unroll
                    for (int i = 0; i < 8; ++i) dv[i] = bk[i >> 1][i & 1];
                } else if (DEFER && u == 1) {   // this chunk's first pair + the previous chunk's second
                    uint32_t v[8];
#pragma unroll
                    for (int i = 0; i < 8; ++i) v[i] = bk[i >> 1][i & 1];
                    reduce_scatter8_bm(v, lane & 15);
                    reduce_scatter8_bm(dv, lane & 15);
                    if (join2) {
                        emit_key(join_pairs(kA, dv[0]), tprev);
                        kA = v[0];
                    } else {
                        emit_key(join_rows(dv[0]), tprev + 2);
                        emit_key(join_rows(v[0]), t0);
                    }
                    tprev = t0;
                } else if (u & 1) {
                    uint32_t v[8];
#pragma unroll
                    for (int i = 0; i < 8; ++i) v[i] = bk[i >> 1][i & 1];
                    reduce_scatter8_bm(v, lane & 15);
                    if (join2) {
                        if (u == 1) kA = v[0];
                        else emit_key(join_pairs(kA, v[0]), t0);
                    } else {
                        emit_key(join_rows(v[0]), t0 + u - 1);
                    }
                }
            }
        }
        rb = rb + NCH * (RG_DPL + 1);
        lb = lb + U;
    }
    if (DEFER) {   // the last chunk's second pair
        reduce_scatter8_bm(dv, lane & 15);
        if (join2) emit_key(join_pairs(kA, dv[0]), tprev);
        else emit_key(join_rows(dv[0]), tprev + 2);
    }
}

__global__ void k_fill_i16(int16_t* out, int opitch, int H, int W, int16_t v) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    if (x < W && y < H) out[(size_t)y * opitch + x] = v;
}

template <int COST, int ND, int DPL>
int launch_one(const MatchParams& a, size_t lds, hipStream_t s) {
    auto fn = k_match<COST, ND, DPL>;
    if (lds > 65536) {  // opt in to > 64 KiB of dynamic LDS (per device, cheap host call)
        hipError_t e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return (int)e;
    }
    const int wc = wave_cols(a.lpg, DPL, a.segm);
    const int rows_per_block = PackCfg<COST, ND>::WPB * PackCfg<COST, ND>::ROWS;
    dim3 grid((a.X1 - a.X0 + wc - 1) / wc, (a.row1 - a.row0 + rows_per_block - 1) / rows_per_block,
              a.nf > 1 ? a.nf : 1);
    hipLaunchKernelGGL(fn, grid, dim3(64 * PackCfg<COST, ND>::WPB), lds, s, a);
    return (int)hipGetLastError();
}

template <int COST, int ND>
int launch_dpl(const MatchParams& a, const MatchPlan& p, size_t lds, hipStream_t s) {
    switch (p.dpl) {
        case 4: return launch_one<COST, ND, 4>(a, lds, s);
        case 6: return launch_one<COST, ND, 6>(a, lds, s);
        case 8: return launch_one<COST, ND, 8>(a, lds, s);
    }
    return (int)hipErrorInvalidValue;
}

template <int COST>
int launch_nd(const MatchParams& a, const MatchPlan& p, size_t lds, hipStream_t s) {
    if constexpr (COST == COST_HOG) {
        return launch_dpl<COST, 5>(a, p, lds, s);
    } else if constexpr (COST == COST_SAD4) {
        switch (p.ndw) {   // = r
            case 2: return launch_dpl<COST, 2>(a, p, lds, s);
            case 3: return launch_dpl<COST, 3>(a, p, lds, s);
            case 4: return launch_dpl<COST, 4>(a, p, lds, s);
            case 5: return launch_dpl<COST, 5>(a, p, lds, s);
            case 6: return launch_dpl<COST, 6>(a, p, lds, s);
            case 7: return launch_dpl<COST, 7>(a, p, lds, s);
        }
        return (int)hipErrorInvalidValue;
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

// Kind actually launched for a public cost: SAD with win >= 5 runs four rows per wave.
int kind_of(int cost, int win) {
    if (cost == COST_SAD && win >= 5) return COST_SAD4;
    return cost;
}

// Ring kind eligibility and geometry.  SV_RING=0 disables it (A/B measurements);
bool ring_kind(int cost, int win, int num_disp) {
    static const bool on = [] {
        const char* e = std::getenv("SV_RING");
        return !(e && e[0] == '0');
    }();
    return on && kind_of(cost, win) == COST_SAD4 && win >= 5 && num_disp <= 256 &&
           (win <= 11 || (win <= 15 && num_disp % 4 == 0));
}
int ring_lpg(int num_disp) { return num_disp <= 64 ? 16 : num_disp <= 128 ? 32 : 64; }
// Segment width per group: S (a multiple of 4) minimising the steps all waves of a row
// run, ceil(band / (G*S)) * (S + 2r) (idle columns of the last wave + the 2r warm-up steps
// of every segment), among segments whose LDS leaves room for 2 waves per SIMD; ties go to
// the longer segment.  SV_RING_SEG=<S> forces a width (A/B measurements).
size_t ring_lds_bytes(int lpg, int seg, int r);
int ring_seg(int lpg, int r, int band, long long blocks) {
    static const int env = [] {
        const char* e = std::getenv("SV_RING_SEG");
        const int v = e ? std::atoi(e) : 0;
        return v >= 8 && v <= 1024 && v % 4 == 0 ? v : 0;
    }();
    (void)blocks;
    if (env) return env;
    const int G = 64 / lpg;
    int best = 8;
    long long best_cost = -1;
    for (int S = 8; S <= 1024; S += 4) {
        if (S > 8 && ring_lds_bytes(lpg, S, r) > 20 * 1024) break;
        const long long cost = (long long)((band + G * S - 1) / (G * S)) * ((S + 2 * r + 3) & ~3);
        if (best_cost < 0 || cost <= best_cost) { best = S; best_cost = cost; }
    }
    return best;
}
size_t ring_lds_bytes(int lpg, int seg, int r) {
    const int wc = (64 / lpg) * seg;
    const int tn = (seg + 2 * r + 3) & ~3;
    const int nl = wc - seg + tn + 1, nr = wc - seg + tn + 4 * lpg;
    const int nrp = nr + (nr + 1) / RG_DPL + 1;
    return (size_t)(nl + nrp) * (r <= 3 ? 20 : r <= 5 ? 24 : 28);
}

template <int R, int LPG, bool KEYS, bool SSD>
int launch_ring_rl(const MatchParams& a, size_t lds, hipStream_t s) {
    // SV_RING_DEFER=0 (A/B): every pair reduced inside its own chunk
    static const bool defer = [] {
        const char* e = std::getenv("SV_RING_DEFER");
        return !(e && e[0] == '0');
    }();
    void (*fn)(MatchParams);
    if constexpr (SSD) fn = k_match_ring<R, LPG, R != 5, false, true>;
    else if constexpr (KEYS) fn = k_match_ring<R, LPG, R != 5, true>;
    else fn = (defer && R != 5) ? k_match_ring<R, LPG, R != 5, false> : k_match_ring<R, LPG, false, false>;
    if (lds > 65536) {
        hipError_t e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return (int)e;
    }
    const int wc = (64 / a.lpg) * a.segm;
    dim3 grid((a.X1 - a.X0 + wc - 1) / wc, (a.row1 - a.row0 + 3) / 4, a.nf > 1 ? a.nf : 1);
    // SV_XCD_MAP=0 (A/B): tiles in plain dispatch order
    static const bool xcd = [] {
        const char* e = std::getenv("SV_XCD_MAP");
        return !(e && e[0] == '0');
    }();
    MatchParams b = a;
    b.xcd_map = xcd ? 1 : 0;
    hipLaunchKernelGGL(fn, grid, dim3(64), lds, s, b);
    return (int)hipGetLastError();
}
template <int R, bool KEYS, bool SSD = false>
int launch_ring_r(const MatchParams& a, size_t lds, hipStream_t s) {
    switch (a.lpg) {
        case 16: return launch_ring_rl<R, 16, KEYS, SSD>(a, lds, s);
        case 32: return launch_ring_rl<R, 32, KEYS, SSD>(a, lds, s);
        case 64: return launch_ring_rl<R, 64, KEYS, SSD>(a, lds, s);
    }
    return (int)hipErrorInvalidValue;
}

template <bool KEYS, bool SSD = false>
int launch_ring(const MatchParams& a0, hipStream_t s) {
    MatchParams a = a0;
    a.lpg = ring_lpg(a.D);
    a.lpg_log2 = a.lpg == 16 ? 4 : a.lpg == 32 ? 5 : 6;
    a.dbits = SSD ? a.lpg_log2 + 2 : 16;   // SSD keys: (cost << log2(4 LPG)) | idx
    if (SSD) a.pad_key = (uint32_t)((max_cost(a.win, COST_SSD) + 1) << a.dbits);
    a.segm = ring_seg(a.lpg, a.r, a.X1 - a.X0, (long long)((a.row1 - a.row0 + 3) / 4) * (a.nf > 1 ? a.nf : 1));
    const size_t lds = ring_lds_bytes(a.lpg, a.segm, a.r);
    if (lds > 160 * 1024) return (int)hipErrorInvalidValue;
    if constexpr (SSD) {
        switch (a.r) {
            case 2: return launch_ring_r<2, false, true>(a, lds, s);
            case 3: return launch_ring_r<3, false, true>(a, lds, s);
            case 4: return launch_ring_r<4, false, true>(a, lds, s);
        }
        return (int)hipErrorInvalidValue;
    } else {
        switch (a.r) {
            case 2: return launch_ring_r<2, KEYS>(a, lds, s);
            case 3: return launch_ring_r<3, KEYS>(a, lds, s);
            case 4: return launch_ring_r<4, KEYS>(a, lds, s);
            case 5: return launch_ring_r<5, KEYS>(a, lds, s);
            case 6: return launch_ring_r<6, KEYS>(a, lds, s);
            case 7: return launch_ring_r<7, KEYS>(a, lds, s);
        }
        return (int)hipErrorInvalidValue;
    }
}

// Split ring merge: per pixel the smaller of the two passes' keys (pass B's indices shifted
// past pass A's 256: on equal costs pass A's smaller disparity wins, the first minimum), and
// the band-edge columns' invalid value.  4 pixels per thread (16-B key loads, one 8-B store)
// when the pitch, frame stride and map allow it.
__device__ __forceinline__ int16_t merge_px(uint32_t ka, uint32_t kb, int x, int X0, int X1, int minD) {
    const uint32_t k = min(ka, kb + 256u);
    return (int16_t)(x >= X0 && x < X1 ? ((int)(k & 0xFFFFu) + minD) * 16 : (minD - 1) * 16);
}
__global__ __launch_bounds__(256) void k_merge_ring_keys(const uint32_t* __restrict__ ka,
                                                         const uint32_t* __restrict__ kb, int16_t* __restrict__ out,
                                                         int opitch, long long fs_out, int row0, int W, int X0, int X1,
                                                         int minD, int vec) {
    const int x = 4 * (int)(blockIdx.x * 256 + threadIdx.x);
    if (x >= W) return;
    const size_t i = (size_t)blockIdx.z * fs_out + (size_t)(row0 + (int)blockIdx.y) * opitch + x;
    if (vec && x + 4 <= W) {
        const uint4 a = *reinterpret_cast<const uint4*>(ka + i);
        const uint4 b = *reinterpret_cast<const uint4*>(kb + i);
        const uint32_t lo = (uint16_t)merge_px(a.x, b.x, x, X0, X1, minD) |
                            ((uint32_t)(uint16_t)merge_px(a.y, b.y, x + 1, X0, X1, minD) << 16);
        const uint32_t hi = (uint16_t)merge_px(a.z, b.z, x + 2, X0, X1, minD) |
                            ((uint32_t)(uint16_t)merge_px(a.w, b.w, x + 3, X0, X1, minD) << 16);
        *reinterpret_cast<uint2*>(out + i) = make_uint2(lo, hi);
        return;
    }
    for (int q = 0; q < 4 && x + q < W; ++q) out[i + q] = merge_px(ka[i + q], kb[i + q], x + q, X0, X1, minD);
}


}  // namespace

// D in (256, 512]: the ring kind twice, d in [0, 256) (64-lane groups) and [256, D) (its
// own group width), each into a key plane, then k_merge_ring_keys — the four-row kind it
// replaces ran 2.3x slower per cell (1080p D=320 w7: 2,322 us per 16 frames against 805 for
// D=256, round 4)
// SSD windows 5..9 with D <= 256 take the ring kind's SSD form when the keys (cost << dbits |
// idx, padding lanes above every real key) fit 32 bits
bool ring_ssd(int cost, int win, int num_disp) {
    if (cost != COST_SSD || win < 5 || win > 9 || num_disp < 1 || num_disp > 256) return false;
    if (!ring_kind(COST_SAD, win, num_disp)) return false;   // (SV_RING=0 switches it off too)
    const int lpg = ring_lpg(num_disp), dbits = (lpg == 16 ? 4 : lpg == 32 ? 5 : 6) + 2;
    const uint64_t cmax = max_cost(win, COST_SSD);
    const uint64_t top = num_disp < 4 * lpg ? (2 * cmax + 2) << dbits : (cmax << dbits) + (uint64_t)(4 * lpg);
    return top < (1ull << 32);
}
bool ring_split(int cost, int win, int num_disp) {
    return num_disp > 256 && num_disp <= 512 && ring_kind(cost, win, 256) && ring_kind(cost, win, num_disp - 256);
}
long long ring_split_elems(int nf, long long fs_out, int row1, int opitch) {
    return ((long long)(nf > 1 ? nf - 1 : 0) * fs_out + (long long)(row1 + 3) * opitch + 64 + 3) & ~3LL;
}

uint64_t max_cost(int win, int cost) {
    return cost == COST_SAD ? (uint64_t)win * win * 255
         : cost == COST_SSD ? (uint64_t)win * win * 255 * 255
                            : (uint64_t)9 * win * win * 255;
}

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
    const int kind = kind_of(cost, win);
    plan->ndw = kind == COST_HOG ? 5 : kind == COST_SAD4 ? win / 2
              : (win + 3) / 4;
    int n = plan->dpl * plan->lpg - 1, bits = 0;
    while (n > 0) { ++bits; n >>= 1; }
    plan->dbits = bits < 1 ? 1 : bits;
    if (hi_keys(kind, win / 2)) plan->dbits = 16;
    const uint64_t cmax = max_cost(win, cost);
    // the other kinds' keys (cost << dbits | idx) must fit 32 bits; padding disparities (idx >=
    // D) carry keys above (cmax + 1) << dbits
    const bool over = (cmax << plan->dbits) >= (1ull << 32) ||
                      (num_disp < plan->dpl * plan->lpg && cost != COST_HOG &&
                       ((2 * cmax + 2) << plan->dbits) >= (1ull << 32));
    plan->mfma_only = 0;
    if (over) {
        // SSD the matrix-core kind holds (centred keys, sv_ssd_mfma.hip): only that kind runs
        // it (launch_match refuses the call where it cannot: unaligned images)
        if (!ssd_mfma(cost, win, num_disp)) return -34;   // ERANGE: key would overflow
        plan->mfma_only = 1;
    }
    return 0;
}

size_t match_lds_bytes(const MatchPlan& p, int r, int cost) {
    const int kind = kind_of(cost, 2 * r + 1);
    const int nw = kind == COST_SAD ? p.ndw : kind == COST_SSD ? p.ndw + 1
                 : kind == COST_SAD4 ? (2 * p.ndw - 2 + 3) / 4 + 4 : 5;
    const int wpb = kind == COST_SAD4 ? 1 : 4;
    const bool split = (kind == COST_SAD4 && nw - 4 <= 3) || kind == COST_HOG || (kind == COST_SSD && nw == 5);
    const int cw = kind == COST_SAD4 && nw - 4 == 3 ? 3 : kind == COST_SAD4 && nw - 4 == 1 ? 1 : 2;
    const int Q = (nw + 3) / 4;
    const int c0 = (p.dpl - (4 * r + 1) % p.dpl) % p.dpl;
    const int wc = wave_cols(p.lpg, p.dpl, seg_mult(kind, r));
    const int NL = wc + 4 * r + p.dpl + 1;
    const int NRlog = wc + 4 * r + p.lpg * p.dpl + p.dpl;
    const int NRphys = NRlog + (NRlog + c0) / p.dpl + 1;
    return (size_t)wpb * (NL + NRphys) * (split ? 16 + 4 * cw : Q * 16);
}

int launch_fill_i16(int16_t* out, int opitch, int H, int W, int16_t v, hipStream_t s) {
    if (H <= 0 || W <= 0) return 0;
    hipLaunchKernelGGL(k_fill_i16, dim3((W + 255) / 256, H), dim3(256), 0, s, out, opitch, H, W, v);
    return (int)hipGetLastError();
}

int launch_match(const MatchParams& a, const MatchPlan& p, int cost, hipStream_t s) {
    if (a.row1 <= a.row0) return 0;
    if (a.X1 <= a.X0) {
        for (int z = 0; z < (a.nf > 1 ? a.nf : 1); ++z) {
            int e = launch_fill_i16(a.out + z * a.fs_out + (size_t)a.row0 * a.opitch, a.opitch,
                                    a.row1 - a.row0, a.W, (int16_t)((a.minD - 1) * 16), s);
            if (e) return e;
        }
        return 0;
    }
    // the ring kind stores through one buffer descriptor with 32-bit byte offsets
    // (2 * (row * out_pitch + x) per frame); maps whose last row lies past 2^31 bytes take
    // the size_t-addressed four-row kind instead
    const bool ring_fits = 2LL * ((long long)(a.row1 + 3) * a.opitch + a.W + 64) < 0x7FFFFFFFLL;
    if (ring_kind(cost, a.win, a.D) && ring_fits) return launch_ring<false>(a, s);
    if (ssd_mfma_fits(a, cost)) return launch_ssd_mfma(a, s);
    if (p.mfma_only) return (int)hipErrorInvalidValue;   // no other kind holds these keys
    if (ring_ssd(cost, a.win, a.D) && ring_fits) return launch_ring<false, true>(a, s);
    if (ring_split(cost, a.win, a.D) && a.keys) {
        // (key planes: 4-byte elements, so half the 2^31-byte range of the int16 maps)
        if (4LL * ((long long)(a.row1 + 3) * a.opitch + a.W + 64) >= 0x7FFFFFFFLL) return (int)hipErrorInvalidValue;
        MatchParams pa = a, pb = a;
        pa.D = 256;
        pb.minD = a.minD + 256;
        pb.D = a.D - 256;
        pb.keys = a.keys + a.keys_stride;
        int e = launch_ring<true>(pa, s);
        if (!e) e = launch_ring<true>(pb, s);
        if (e) return e;
        const int nf = a.nf > 1 ? a.nf : 1;
        const long long fso = nf > 1 ? a.fs_out : 0LL;
        const int vec = (a.opitch % 4 == 0 && fso % 4 == 0 && a.keys_stride % 4 == 0 &&
                         ((uintptr_t)a.out & 7) == 0 && ((uintptr_t)a.keys & 15) == 0) ? 1 : 0;
        hipLaunchKernelGGL(k_merge_ring_keys, dim3((a.W + 1023) / 1024, a.row1 - a.row0, nf), dim3(256), 0, s, pa.keys,
                           pb.keys, a.out, a.opitch, fso, a.row0, a.W, a.X0, a.X1, a.minD, vec);
        return (int)hipGetLastError();
    }
    const size_t lds = match_lds_bytes(p, a.r, cost);
    if (lds > 160 * 1024) return (int)hipErrorInvalidValue;
    MatchParams b = a;
    b.segm = seg_mult(kind_of(cost, a.win), a.r);
    switch (kind_of(cost, a.win)) {
        case COST_SAD: return launch_nd<COST_SAD>(b, p, lds, s);
        case COST_SAD4: return launch_nd<COST_SAD4>(b, p, lds, s);
        case COST_SSD: return launch_nd<COST_SSD>(b, p, lds, s);
        case COST_HOG: return launch_nd<COST_HOG>(b, p, lds, s);
    }
    return (int)hipErrorInvalidValue;
}

}  // namespace sv
