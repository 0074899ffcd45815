// Internal declarations shared by the HIP kernel files and the C-ABI (sv_capi.cpp).
// gfx950 (CDNA4, wave64) only.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

struct sv_comm;

namespace sv {

// v_sad_u32: a = |a - b| + c (unsigned) — a running window sum's update `sum - leaving +
// entering` in ONE VOP3 whenever sum >= leaving (the sum holds the leaving term as a summand);
// also exact on two u16 halves per word when each half's sum holds its own leaving term and
// stays below 2^16 (no borrow, no carry).  No clang builtin, and the umax - umin + c pattern
// is split into several ops inside large bodies, so inline asm (plain VOP3: no hazards).
__device__ __forceinline__ void sad_u32_acc(uint32_t& a, uint32_t b, uint32_t c) {
    asm("v_sad_u32 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));
}

// Sets the calling thread's sv_last_error() message; returns `code`.
int set_error(int code, const std::string& msg);

// RCCL transfers of the multi-device entry points (sv_comm.cpp; librccl loaded on first use).
int comm_group_start();
int comm_group_end();
int comm_send(sv_comm* c, const void* buf, size_t bytes, int peer, hipStream_t s);
int comm_recv(sv_comm* c, void* buf, size_t bytes, int peer, hipStream_t s);
int comm_rank(const sv_comm* c);
int comm_size(const sv_comm* c);
int comm_device(const sv_comm* c);

enum Cost { COST_SAD = 0, COST_SSD = 1, COST_HOG = 2, COST_SGBM = 3 };

// Disparity lanes: each wave is split into groups of LPG lanes (16/32/64); every lane of a
// group owns DPL consecutive disparities of the same output pixel, so one group covers
// LPG*DPL candidates and the per-pixel argmin is an in-lane min3 chain plus a
// log2(LPG)-step DPP reduction.
struct MatchPlan {
    int dpl;     // disparities per lane: 4, 6 or 8
    int lpg;     // lanes per group: 16, 32 or 64
    int ndw;     // dwords per column pack: ceil(win/4) (SAD/SSD), 5 for HOG
    int dbits;   // argmin key index bits
    int mfma_only = 0;   // SSD whose keys only the matrix-core kind holds (its own key form)
};

struct MatchParams {
    const uint8_t* L;      // left gray (device), row pitch `pitch` bytes
    const uint8_t* R;      // right gray
    const uint16_t* HL;    // HOG window histograms [H][W][10] (cost == HOG)
    const uint16_t* HR;
    int H, W, pitch;
    int minD, D, r;        // r = win/2 (0 for HOG: the window lives in the histograms)
    int win;
    int X0, X1;            // matched column band [X0, X1)
    int row0, row1;        // output rows [row0, row1)
    int lpg, lpg_log2, dbits;
    int16_t* out;
    int opitch;            // elements
    // frame batch (grid.z): frame z reads L/R + z*fs_in bytes, HL/HR + z*fs_hist elements
    // and writes out + z*fs_out elements
    int nf;
    long long fs_in, fs_out, fs_hist;
    uint32_t pad_key;      // (max_cost + 1) << dbits: key offset of padding disparities
    int segm;              // segment length in LPG units (set by launch_match)
    // persistent kinds: the launching context's work counters (16 B, zero between launches;
    // the kernel's last wave resets them), so concurrent launches on other contexts never
    // share one
    unsigned* work_ctr;
    int xcd_map;           // ring kind: XCD-aware tile order (launch_ring_rl)
    // split ring (SAD, 256 < D <= 512): two argmin-key planes laid out like `out` (opitch,
    // fs_out) as u32, `keys_stride` elements apart; the caller owns them (ring_split_elems)
    uint32_t* keys;
    long long keys_stride;
};

// Host-side launchers (return hipError_t as int).
int plan_match(int num_disp, int win, int cost, MatchPlan* plan);
uint64_t max_cost(int win, int cost);   // largest window cost of a (win, cost) pair
size_t match_lds_bytes(const MatchPlan& p, int r, int cost);
int launch_match(const MatchParams& a, const MatchPlan& p, int cost, hipStream_t s);
// D > 256 SAD windows run the ring kind twice (d < 256, d >= 256) into key planes and merge:
// whether a launch takes that form, and the elements of one key plane it needs
bool ring_split(int cost, int win, int num_disp);
bool ring_ssd(int cost, int win, int num_disp);   // SSD windows 5..9, D <= 256: the ring kind
// SSD on the matrix cores (sv_ssd_mfma.hip): odd windows <= 15, D a multiple of 32 up to 256
// (the key range decides: D > 128 up to win 13)
bool ssd_mfma(int cost, int win, int num_disp);
bool ssd_mfma_fits(const MatchParams& a, int cost);   // + operand alignment, r == win / 2
int launch_ssd_mfma(const MatchParams& a, hipStream_t s);
long long ring_split_elems(int nf, long long fs_out, int row1, int opitch);
int launch_fill_i16(int16_t* out, int opitch, int H, int W, int16_t v, hipStream_t s);

int launch_gray(const uint8_t* bgr, int H, int W, int pitch, uint8_t* gray, hipStream_t s);
// nf frames (grid.z): frame z reads g + z*fs_in bytes and writes out + z*fs_out floats.
int launch_harris(const uint8_t* g, int H, int W, int pitch, float* out, hipStream_t s, int nf = 1,
                  long long fs_in = 0, long long fs_out = 0);
int launch_hog_hist(const uint8_t* g, int H, int W, int pitch, int win, int row0, int row1,
                    uint16_t* hist, hipStream_t s);
// Both images of nf frame pairs in one launch (grid.z = 2 nf): frame z's left/right images at
// g0/g1 + z*fs_in bytes, their histograms at h0/h1 + z*fs_hist elements.
int launch_hog_hist_pairs(const uint8_t* g0, const uint8_t* g1, int H, int W, int pitch, int win, int row0,
                          int row1, uint16_t* h0, uint16_t* h1, int nf, long long fs_in, long long fs_hist,
                          hipStream_t s);

// Rectification (sv_rectify.hip).  ir = inv(P[:, :3] * R) row-major; k = k1 k2 p1 p2 k3 k4
// k5 k6 s1 s2 s3 s4 (OpenCV distCoeffs order, zero-padded).
struct UndistortParams {
    double ir[9];
    double fx, fy, u0, v0;
    double k[12];
    int H, W;
};
int launch_undistort_map(const UndistortParams& p, short2* map1, uint16_t* map2, hipStream_t s);
int launch_remap(const uint8_t* src, int sH, int sW, int channels, int spitch, long long sfs,
                 const short2* map1, const uint16_t* map2, int H, int W, bool gray_out, uint8_t* dst,
                 int dpitch, long long dfs, int nf, hipStream_t s);

// u8 (f32 = false) or float32 images; pitches and frame strides in bytes.
int launch_resize_linear(const void* src, int sH, int sW, int cn, int spitch, long long sfs, void* dst,
                         int dH, int dW, int dpitch, long long dfs, int nf, bool f32, hipStream_t s);

// Reductions (sv_stats.hip).
struct FrameStatsArgs {
    const uint8_t* img0;
    const uint8_t* img1;      // grid.z = 2: the second image of the pair
    int H, W, pitch, cn;
    int bh, bw;               // blocks of compute_block_homogeneity: max(1, H/48) x max(1, W/48)
    uint32_t* block_sum;      // [nimg][bh][bw]
    uint32_t* block_sq;
    uint32_t* hist;           // [nimg][256], written whole by the fold kernel
    uint32_t* hist_copies;    // accumulators [kHistCopies][nimg][256], zero on entry and exit
    // frame batches: image z of the launch (grid.z) is image z % per (img0 / img1) of frame
    // z / per, at + (z / per) * fs bytes; outputs are dense per image z
    int per;                  // images per frame: 1 or 2
    long long fs;
};
// Global histograms are accumulated into kHistCopies copies (block b adds into copy
// b % kHistCopies: hundreds of same-address atomics serialise at L2) and folded after.
constexpr int kHistCopies = 8;
int launch_frame_stats(const FrameStatsArgs& a, int nimg, hipStream_t s);

enum SelectMask { SEL_ALL = 0, SEL_POSITIVE = 1, SEL_MASK_GT = 2 };
constexpr int kMaxRanks = 4;
constexpr int kSelBatch = 16;   // arrays per batched select launch
struct SelectArgs {
    const float* x;
    const float* mask;        // SEL_MASK_GT: element i selected iff mask[i] > thr
    float thr;
    int mask_mode;
    size_t n;
    int shift, bits;          // digit = (key >> shift) & ((1 << bits) - 1)
    int nranks;
    // batches (grid.y = array y of narr): x + y * xstride, mask + y * mstride; every
    // accumulator / output below is per array (array y's block at + y * its size)
    int narr;
    size_t xstride, mstride;
    uint32_t prefix[kSelBatch][kMaxRanks];   // key >> (shift + bits) of each rank's target
    uint32_t* ghist;          // accumulators [narr][kHistCopies][kMaxRanks][2048], zero on entry and exit
    unsigned long long* counts;   // accumulators [narr][kCountSlots][16] (slot = {selected, nan, pad})
    uint32_t* hist_out;       // [narr][kMaxRanks][2048], folded by the launcher's second kernel
    unsigned long long* counts_out;   // [narr][2]: selected, nan
};
constexpr int kCountSlots = 32;   // blocks add their counts into slot blockIdx % 32 (128 B apart)
int launch_select_hist(const SelectArgs& a, hipStream_t s);

enum AffineMode { AFF_F32 = 0, AFF_F64 = 1, AFF_FILL = 2 };
struct AffineArgs {
    const float* x;
    float* out;
    size_t n;
    int mode;
    float fa, fb, fc, fd;     // AFF_F32: fc + ((x - fa) / fb) * fd;  AFF_FILL: fc
    double ds, doff;          // AFF_F64: float(double(x) * ds + doff)
};
int launch_affine_f32(const AffineArgs& a, hipStream_t s);

// SGBM-3WAY mode (sv_sgbm.hip).
struct SgbmArgs {
    const uint8_t* L;
    const uint8_t* R;
    int H, W, pitch;
    int minD, D, r;            // r = blockSize / 2
    int Dp;                    // per-pixel stride of the volumes: sgbm_dp(D)
    int X0, Wb;                // band [X0, X0 + Wb)
    int cap, P1, P2, uniq, disp12;
    uint16_t* hsum;            // [H][Wb][D] window-column sums of the pixel cost
    uint16_t* C;               // [H][Wb][D] window sums
    void* Llr;                 // [H][Wb][D] path costs, int16 (l32 = 0) or int32
    void* Lrl;
    void* Ltb;                 // [H][Wb][Dp] top->bottom path costs (same type as Llr)
    int l32;
    int fused;                 // R->L path fused with the WTA (L_rl never stored; see sgbm_fused)
    uint4* recs;               // [2][H][W] per-pixel BT records of L, R (k_sgbm_cost path)
    void* band;                // [H][Wb] {int16 x16 disparity after uniqueness + sub-pixel,
                               //  int16 argmin index, int32 min cost (INT_MAX: not unique)}
    int16_t* out;              // [H][opitch] final int16 x16 map
    int opitch;
    void* dummy;               // >= 64 x 128 bytes: store target of the padding lanes
    // frame batch (grid.z = frame): frame z reads L/R + z*fs_in bytes, writes out + z*fs_out
    // elements, and owns volume z (H*Wb*Dp elements of each volume's type) and band z
    long long fs_in, fs_out;
    __device__ __forceinline__ void select_frame(int z) {
        const size_t vol = (size_t)H * Wb * Dp * z;
        L += z * fs_in;
        R += z * fs_in;
        out += z * fs_out;
        hsum += vol;
        C += vol;
        const size_t lb = vol * (l32 ? 4 : 2);
        Llr = static_cast<char*>(Llr) + lb;
        Lrl = static_cast<char*>(Lrl) + lb;
        Ltb = static_cast<char*>(Ltb) + lb;
        band = static_cast<char*>(band) + (size_t)H * Wb * 8 * z;
        if (recs) recs += (size_t)2 * H * W * z;
    }
};
int sgbm_dp(int D);   // per-pixel volume stride for D disparities, -1 if D > 512
// Whether launches of nf frames of D disparities fuse the R->L path with the WTA
// (k_sgbm_rl_wta, L_rl never stored): batches of >= 8 frames with D <= 128, where the extra
// work per step hides behind other waves' chains.  Otherwise both horizontal directions run
// in k_sgbm_hpath, and for D > 128 the vertical path is fused with the WTA instead
// (k_sgbm_vpath_wta, L_tb never stored; measured faster at every batch size there: D=320
// 412 -> 459 frames/s at batch 8, 449 -> 491 at 16).  SV_SGBM_FUSED=0 / 1 forces either form.
bool sgbm_fused(int nf, int D);
// r <= 4: pixel cost and both window sums in one pass (k_sgbm_cost, no hsum
// volume); SV_SGBM_COST=0 restores k_sgbm_hsum_tiled + k_sgbm_vsum8
bool sgbm_cost_fused(int D, int r);
// aux / fork / join: a second stream and two events for the concurrent vertical path (aux =
// nullptr: everything on s)
// nf frames per launch (grid.z), laid out as described at SgbmArgs::select_frame
int launch_sgbm(const SgbmArgs& a, int nf, hipStream_t s, hipStream_t aux, hipEvent_t fork, hipEvent_t join);
// nf maps, map z at img + z*fimg; parent/size hold H*W ints per map
int launch_speckles(int16_t* img, int H, int W, int pitch, int newv, int maxsize, int maxdiff, int* parent,
                    int* size, hipStream_t s, int nf = 1, long long fimg = 0);

// Post-processing modes for the median kernel.
enum PostMode { POST_NONE = 0, POST_DEPTH = 1, POST_SCALED = 2 };
struct PostParams {
    int mode;
    float minf, maxf, rangef, min_disp_global;   // POST_DEPTH (depth_map.py:915-937)
    int min_disp, num_disp;                       // POST_SCALED (fused_depth_map.py:1010-1029)
    float* out_a;      // DEPTH: depth_final        SCALED: disparity_normalized (f32)
    uint8_t* out_u8;   // DEPTH: depth_normalized   SCALED: disparity_normalized (u8)
    float* out_b;      // SCALED: confidence
    // Optional display colormap of out_u8 (cv2.applyColorMap: TURBO at depth_map.py:937, JET
    // at fused_depth_map.py:1013), fused into the median kernel's epilogue: out_bgr[3i..3i+2]
    // = the B, G, R bytes of cmap[out_u8[i]] (cmap: 256 entries B | G << 8 | R << 16).
    uint8_t* out_bgr;
    const uint32_t* cmap;
    // Optional int16 x16 median map (the host paths expand it with the table on the host:
    // 2 B/px over PCIe instead of 9-11); the f32 disparity output of the median kernel is
    // then optional (disp == nullptr).
    int16_t* out_m16;
    // Optional u8 disparity index map: m / 16 - d8_base, for integer-disparity costs (SAD / SSD /
    // HOG: every median is a multiple of 16) with D <= 255 — 1 B/px for a gather over xGMI.
    uint8_t* out_d8;
    int d8_base;
    // Optional lookup table of the post-processing as a function of the int16 x16 median
    // value m in [lut_m0, lut_m0 + lut_n), built by launch_post_lut with the same f32 ops
    // (bit-identical to evaluating post_one per pixel; replaces two IEEE divisions).
    const float* lut_a;
    const uint8_t* lut_u8;
    const float* lut_b;
    int lut_m0, lut_n;
    // 4: the table holds whole disparities only (entry i = value lut_m0 + 16 i), for maps whose
    // medians are all multiples of 16 (integer-disparity costs): (D + 1) entries instead of
    // 16 (D + 1), so the epilogue's lookups stay in L1 at large D
    int lut_shift;
};
// Harris response computed by extra blocks of the median launch (C2): the left gray frames
// at g (+ z*fs_in bytes, row pitch `pitch`), f32 responses at out (+ z*fs_out floats, row
// pitch W).  Needs W, H >= 8 (the DPP form).  mbx is set by the launcher.
struct HarrisParams {
    const uint8_t* g;
    int pitch;
    long long fs_in;
    float* out;
    long long fs_out;
    int mbx;
    int form;   // 0: 60-column waves, 1: 248-column waves (set by the launcher)
};
// nf frames (grid.z): frame z reads in + z*fs_in and writes disp/out_* + z*fs_out elements.
// harris (nullable): also the Harris response of rows [row0, row1) of each frame.
int launch_median_i16(const int16_t* in, int H, int W, int row0, int row1, float* disp,
                      const PostParams& pp, hipStream_t s, int nf = 1, long long fs_in = 0,
                      long long fs_out = 0, const HarrisParams* harris = nullptr);
int launch_median_f32(const float* in, int H, int W, float* out, hipStream_t s);
// The median kernel's post-processing epilogue over an int16 x16 median map of n pixels
// (disp = m / 16 and the pp outputs, element-wise; the table must be attached).
int launch_post_m16(const int16_t* in, long long n, float* disp, const PostParams& pp, hipStream_t s);
int launch_post(const float* disp, int n, const PostParams& pp, hipStream_t s);
// Evaluates the post-processing of pp.mode for m = m0 .. m0+n-1 (d = m/16) into the tables.
int launch_post_lut(const PostParams& pp, int m0, int n, int step, float* lut_a, uint8_t* lut_u8,
                    float* lut_b, hipStream_t s);

}  // namespace sv
