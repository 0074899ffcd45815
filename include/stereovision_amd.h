/*
 * stereovision_amd.h — C ABI of the MI355X (gfx950) stereo-disparity engine.
 *
 * Drop-in boundary for the reference's disparity hot path.  Every entry point names the
 * reference call it replaces (file:line under AlexGr5/StereoVision):
 *
 *   sv_gray / sv_gray_dev            cv2.cvtColor(img, cv2.COLOR_BGR2GRAY)
 *                                    depth_map.py:871-880, fused_depth_map.py:979-980
 *   sv_disparity / sv_disparity_dev  cv2.StereoSGBM_create(...).compute(gl, gr)
 *                                    depth_map.py:894-909, fused_depth_map.py:988-1004
 *                                    (replaced by the north_star SAD/SSD/HOG WTA engine;
 *                                    same int16 x16 output convention)
 *   sv_median5_f32, sv_median_rows_dev   cv2.medianBlur(disparity, 5)
 *                                    depth_map.py:912, fused_depth_map.py:1007
 *   sv_depth_post                    depth/clip/mask/normalise NumPy block, depth_map.py:915-937
 *   sv_scaled_post                   clip/normalise/confidence NumPy block,
 *                                    fused_depth_map.py:1010-1029
 *   sv_depth_map                     the whole numeric body of create_depth_map
 *                                    (depth_map.py:868-937) minus the colormap
 *   sv_depth_map_color               ... including the colormap (depth_map.py:937)
 *   sv_stereo_scaled                 the whole numeric body of create_depth_map_stereo_scaled
 *                                    (fused_depth_map.py:976-1029) minus colormap/putText
 *   sv_harris, sv_hog_hist           north_star stages with no reference counterpart
 *   sv_init_undistort_rectify_map    cv2.initUndistortRectifyMap(K, dist, R, P, size, CV_16SC2)
 *                                    depth_map.py:636-641, fused_depth_map.py:402-407
 *   sv_remap / sv_remap_dev          cv2.remap(img, map1, map2, cv2.INTER_LINEAR)
 *                                    depth_map.py:815-826, fused_depth_map.py:480-491
 *   sv_resize_linear                 cv2.resize(img, size) INTER_LINEAR (fused_depth_map.py:474-476)
 *   sv_frame_stats                   image statistics of detect_camera_occlusion
 *                                    (fused_depth_map.py:131-301)
 *   sv_select_count/ranks            order statistics of np.percentile in
 *                                    calibrate_midas_to_stereo / normalize_to_stereo_range
 *                                    (fused_depth_map.py:1169-1257, 1503-1554)
 *   sv_multi_gpu_batch               the per-frame create_depth_map loop, frame-sharded over
 *                                    several devices from one process
 *   sv_rectify_pair                  the two remap calls of apply_stereo_rectification
 *                                    (depth_map.py:779-834, fused_depth_map.py:444-500) with
 *                                    the maps resident on the device
 *
 * Conventions
 *   - plain pointers and sizes only; images are row-major uint8, `stride` in bytes;
 *   - host (`sv_x`) entry points take caller-owned host buffers and block until the result
 *     is in them; device (`sv_x_dev`) entry points take device pointers and a hipStream_t
 *     passed as void* (NULL = the context's own stream) and return after enqueueing;
 *   - return 0 on success, a negative errno-style code otherwise; no C++ exception crosses
 *     the ABI; sv_last_error() gives the calling thread's last message;
 *   - a context is bound to one device; calls on one context are serialised by an internal
 *     mutex and each call selects the context's device first (device selection is
 *     per-thread in HIP), so contexts may be used from any thread (the reference calls the
 *     disparity path from a ThreadPoolExecutor worker, fused_depth_map.py:2591-2598);
 *   - the context owns its device buffers and pinned staging, grown on demand and reused.
 */
#ifndef STEREOVISION_AMD_H
#define STEREOVISION_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SV_API_VERSION 1

typedef struct sv_ctx sv_ctx;

/* SAD / SSD / HOG: the north_star winner-take-all engine.  SGBM: OpenCV's SGBM-3WAY
 * algorithm restated (the reference's own matcher), with the reference's parameters
 * P1 = 24 win^2, P2 = 96 win^2, disp12MaxDiff 1, uniquenessRatio 10, speckle 100 / 32,
 * preFilterCap 63 (depth_map.py:894-906) when selected through the generic entry points;
 * sv_sgbm / sv_sgbm_dev take every parameter.  SGBM is frame-only (no row bands). */
enum sv_cost { SV_COST_SAD = 0, SV_COST_SSD = 1, SV_COST_HOG = 2, SV_COST_SGBM = 3 };

enum sv_status {
    SV_OK = 0,
    SV_EHIP = -5,     /* HIP runtime error (message in sv_last_error) */
    SV_ENOMEM = -12,
    SV_ENODEV = -19,
    SV_EINVAL = -22,
    SV_ERANGE = -34   /* parameters whose argmin key would overflow 32 bits: (cmax << dbits)
                         >= 2^32, or ((2 cmax + 2) << dbits) >= 2^32 when num_disp leaves
                         padding disparities in the lane plan (cmax = largest window cost) */
};

/* post-processing modes of sv_map_out.mode / sv_post_m16_dev */
enum sv_post { SV_POST_NONE = 0, SV_POST_DEPTH = 1, SV_POST_SCALED = 2 };

/* kernel ids for the profiling counters */
enum sv_kernel {
    SV_K_GRAY = 0, SV_K_HARRIS = 1, SV_K_HOG = 2, SV_K_MATCH = 3, SV_K_MEDIAN = 4, SV_K_POST = 5,
    SV_K_REMAP = 6, SV_K_UNDISTORT = 7, SV_K_RESIZE = 8, SV_K_STATS = 9, SV_K_SELECT = 10,
    SV_K_AFFINE = 11, SV_K_SGBM = 12, SV_K_SPECKLE = 13,
    SV_K_GATHER = 14,   /* multi-GPU gathers to the root (RCCL / peer copies), root stream */
    SV_K_SCATTER = 15,  /* multi-GPU input scatters (row bands + halos), per context stream */
    SV_K_H2D = 16,      /* host-buffer entry points: the frame pair's upload (per image) */
    SV_K_D2H = 17,      /* host-buffer entry points: the outputs' download */
    SV_NKERNELS = 18
};

int sv_version(void);
const char* sv_last_error(void);
int sv_device_count(int* n);
int sv_create(int device, sv_ctx** out);
void sv_destroy(sv_ctx* ctx);
int sv_synchronize(sv_ctx* ctx);
/* Waits for the context's work and frees its grow-only device scratch (disparity, HOG and
 * SGBM volumes, band buffers); the next call allocates what it needs again.  SGBM batches
 * size their volumes to SV_SGBM_BUDGET_GB, default a quarter of the device's free memory
 * (at most 48 GiB). */
int sv_release_scratch(sv_ctx* ctx);
/* Cross-stream ordering on the context's device (NULL stream = the context stream), with 16
 * event slots per context: sv_event_record marks the work enqueued on `stream` so far;
 * sv_stream_wait_event makes work enqueued on `stream` afterwards wait for that mark (e.g.
 * a gather on a communication stream overlapping the next frame batch's kernels). */
int sv_event_record(sv_ctx* ctx, int slot, void* stream);
int sv_stream_wait_event(sv_ctx* ctx, int slot, void* stream);
void* sv_stream(sv_ctx* ctx);

/* Engine plan for a configuration: disparities per lane, lanes per group, LDS bytes per
 * 256-thread block of the matching kernel. */
int sv_plan(int num_disp, int win, int cost, int* dpl, int* lpg, int* lds_bytes);

/* ---- host-memory entry points (drop-in path) ------------------------------------- */
int sv_gray(sv_ctx* ctx, const uint8_t* bgr, int H, int W, int stride, uint8_t* gray);

/* left/right: HxW (channels = 1) or HxWx3 BGR (channels = 3).  disp16: HxW int16 = d*16,
 * invalid = (min_disp-1)*16.  harris (nullable): HxW f32 Harris response of the left
 * gray image. */
int sv_disparity(sv_ctx* ctx, const uint8_t* left, const uint8_t* right, int H, int W,
                 int channels, int stride, int min_disp, int num_disp, int win, int cost,
                 int16_t* disp16, float* harris);

int sv_median5_f32(sv_ctx* ctx, const float* in, int H, int W, float* out);

/* min_depth/max_depth: float32 of the caller's bounds; depth_range: float32 of
 * (max_depth - min_depth) computed in double (NumPy-2 semantics of depth_map.py:936);
 * min_disp_global: the module global MIN_DISP (depth_map.py:932). */
int sv_depth_post(sv_ctx* ctx, const float* disparity, int n, float min_depth, float max_depth,
                  float depth_range, float min_disp_global, float* depth_final,
                  uint8_t* depth_normalized);

int sv_scaled_post(sv_ctx* ctx, const float* disparity, int n, int min_disp, int num_disp,
                   float* disparity_normalized, uint8_t* normalized_u8, float* confidence);

int sv_depth_map(sv_ctx* ctx, const uint8_t* left, const uint8_t* right, int H, int W,
                 int channels, int stride, int min_disp, int num_disp, int win, int cost,
                 float min_depth, float max_depth, float depth_range, float min_disp_global,
                 float* depth_final, float* disparity, uint8_t* depth_normalized);

int sv_stereo_scaled(sv_ctx* ctx, const uint8_t* left, const uint8_t* right, int H, int W,
                     int channels, int stride, int min_disp, int num_disp, int win, int cost,
                     float* disparity_normalized, float* disparity, uint8_t* normalized_u8,
                     float* confidence);

/* The same two entry points with the display colormap of the drop-ins fused into the
 * median/post kernel (cv2.applyColorMap(depth_normalized, COLORMAP_TURBO) at depth_map.py:937;
 * COLORMAP_JET of the normalised disparity at fused_depth_map.py:1013): cmap_bgr is the
 * 256 x 3 BGR table (the drop-ins pass cv2's own table, read back from cv2.applyColorMap, when
 * cv2 is importable), depth_colormap the H x W x 3 BGR output.  depth_normalized /
 * normalized_u8 are nullable here. */
int sv_depth_map_color(sv_ctx* ctx, const uint8_t* left, const uint8_t* right, int H, int W,
                       int channels, int stride, int min_disp, int num_disp, int win, int cost,
                       float min_depth, float max_depth, float depth_range, float min_disp_global,
                       const uint8_t* cmap_bgr, float* depth_final, float* disparity,
                       uint8_t* depth_normalized, uint8_t* depth_colormap);
int sv_stereo_scaled_color(sv_ctx* ctx, const uint8_t* left, const uint8_t* right, int H, int W,
                           int channels, int stride, int min_disp, int num_disp, int win, int cost,
                           const uint8_t* cmap_bgr, float* disparity_normalized, float* disparity,
                           uint8_t* normalized_u8, float* confidence, uint8_t* depth_colormap);

int sv_harris(sv_ctx* ctx, const uint8_t* gray, int H, int W, int stride, float* out);

/* Row band [row0, row1) of the disparity map (halo rows read from the full frame, so the
 * bands of a row-tiled multi-GPU split reassemble bit-exactly); only those rows of
 * disp16 (HxW) are written. */
int sv_disparity_rows(sv_ctx* ctx, const uint8_t* left, const uint8_t* right, int H, int W,
                      int channels, int stride, int min_disp, int num_disp, int win, int cost,
                      int row0, int row1, int16_t* disp16);

/* out: [H][W][10] uint16 (9 bins + 1 zero pad) window histograms */
int sv_hog_hist(sv_ctx* ctx, const uint8_t* gray, int H, int W, int stride, int win,
                uint16_t* out);

/* ---- device-memory entry points (zero-copy, row bands for multi-GPU sharding) ---- */
int sv_gray_dev(sv_ctx* ctx, const uint8_t* d_bgr, int H, int W, int pitch, uint8_t* d_gray,
                void* stream);

/* Computes output rows [row0, row1) of the disparity map of full-frame gray device images
 * (halo rows are read from the full frame, so bands tile the frame bit-exactly). */
int sv_disparity_dev(sv_ctx* ctx, const uint8_t* d_left, const uint8_t* d_right, int H, int W,
                     int pitch, int min_disp, int num_disp, int win, int cost, int row0,
                     int row1, int16_t* d_disp16, int out_pitch, void* stream);

/* Outputs of the median + post-processing epilogue: cv2.medianBlur(disparity, 5) of an int16
 * x16 disparity map (depth_map.py:909-912, fused_depth_map.py:1004-1007) and the NumPy post
 * that follows it — SV_POST_DEPTH: depth/clip/mask/normalise (depth_map.py:915-937),
 * SV_POST_SCALED: clip/normalise/confidence (fused_depth_map.py:1010-1029).  Every pointer is
 * nullable (not written) and, except cmap_bgr, a device pointer; at least one output must be
 * set.  One descriptor serves every median launch (row bands, frame batches, the root of a
 * multi-device call) instead of one entry point per output combination. */
typedef struct sv_map_out {
    int mode;                  /* sv_post: what out_a / out_u8 / out_b hold */
    float min_depth;           /* SV_POST_DEPTH: float32 of the caller's bounds */
    float max_depth;
    float depth_range;         /* float32 of (max_depth - min_depth) computed in double
                                  (NumPy-2 semantics of depth_map.py:936) */
    float min_disp_global;     /* the module global MIN_DISP (depth_map.py:932) */
    float* disparity;          /* f32 median / 16 (create_depth_map's `disparity`) */
    float* out_a;              /* DEPTH: depth_final       SCALED: disparity_normalized */
    uint8_t* out_u8;           /* DEPTH: depth_normalized  SCALED: its u8 image */
    float* out_b;              /* SCALED: confidence */
    int16_t* med16;            /* int16 x16 median map (OpenCV's fixed point; disparity =
                                  med16 / 16 exactly): 2 B/px for a gather or a download */
    uint8_t* d8;               /* u8 disparity index median / 16 - (min_disp - 1), 0 =
                                  invalid: integer-disparity costs (SAD / SSD / HOG) with
                                  num_disp <= 255, else -EINVAL (1 B/px) */
    const uint8_t* cmap_bgr;   /* with bgr: the 256 x 3 BGR colormap table (host memory) */
    uint8_t* bgr;              /* cv2.applyColorMap(out_u8, cmap) (TURBO at depth_map.py:937,
                                  JET at fused_depth_map.py:1013), H x W x 3 */
    float* harris;             /* sv_depth_map_batch_dev only: the Harris response of every
                                  LEFT frame, computed by extra blocks of the median launch */
} sv_map_out;

/* Median (+ post) of output rows [row0, row1) of an H x W int16 x16 map (halo rows read from
 * the full map, so row bands of a multi-GPU split reassemble bit-exactly); outputs at their
 * full-frame offsets.  cost: the matcher that produced the map (integer-disparity maps use the
 * whole-disparity post table; SGBM's sub-pixel maps the full one). */
int sv_median_rows_dev(sv_ctx* ctx, const int16_t* d_disp16, int H, int W, int row0, int row1,
                       int min_disp, int num_disp, int cost, const sv_map_out* out, void* stream);
/* The post-processing of n median values d_med16 (int16 x16, e.g. maps gathered over xGMI):
 * d_disparity = m / 16 (nullable), and mode's outputs element-wise, exactly as the median
 * kernel's epilogue writes them (depth_map.py:915-936 / fused_depth_map.py:1010-1024). */
int sv_post_m16_dev(sv_ctx* ctx, const int16_t* d_med16, int64_t n, int mode, float min_depth,
                    float max_depth, float depth_range, float min_disp_global, int min_disp,
                    int num_disp, float* d_disparity, float* d_out_a, uint8_t* d_out_u8,
                    float* d_out_b, void* stream);

/* ---- frame batches (one launch per kernel over grid.z) ------------------------------
 * A batch of n_frames equally-shaped gray pairs, frame z at d_left/d_right + z*frame_stride
 * bytes.  Replaces the reference's per-frame loop over the same calls (depth_map.py:837-946
 * called once per captured frame, fused_depth_map.py:2591-2598) when frames are queued:
 * one launch per kernel fills the GPU even for small frames.  The context's internal scratch
 * is ordered across streams (a call on another stream waits for the previous user of the
 * scratch).  cost = SV_COST_SGBM runs every SGBM stage once per chunk of up to 32 frames
 * (volumes of ~1.5 GB per 1080p D=128 frame, within the scratch budget of
 * sv_release_scratch); chunks of >= 8 frames fuse the right-to-left path with the
 * winner-take-all.
 *
 * sv_disparity_batch_dev: the int16 x16 maps only, at an explicit out_pitch /
 * out_frame_stride (elements). */
int sv_disparity_batch_dev(sv_ctx* ctx, const uint8_t* d_left, const uint8_t* d_right,
                           int n_frames, int H, int W, int pitch, int64_t frame_stride,
                           int min_disp, int num_disp, int win, int cost, int16_t* d_disp16,
                           int out_pitch, int64_t out_frame_stride, void* stream);
/* sv_depth_map_batch_dev: the whole device path (disparity -> median -> post) over the batch,
 * every output of `out` dense per frame (frame z at + z*H*W elements).  stages:
 *   SV_STAGE_ALL     both launches; d_disp16 nullable (the context's scratch, else the raw
 *                    int16 x16 maps are kept there, dense per frame)
 *   SV_STAGE_MATCH   the disparity launch only, into d_disp16 (required); out unused
 *   SV_STAGE_MEDIAN  the median launch only, from d_disp16 (required; d_left read only for
 *                    out->harris) — with SV_STAGE_MATCH on another stream or context, the two
 *                    launches of consecutive batches overlap (the HBM-bound median beside the
 *                    VALU-bound match). */
#define SV_STAGE_MATCH 1
#define SV_STAGE_MEDIAN 2
#define SV_STAGE_ALL 3
int sv_depth_map_batch_dev(sv_ctx* ctx, const uint8_t* d_left, const uint8_t* d_right,
                           int n_frames, int H, int W, int pitch, int64_t frame_stride,
                           int min_disp, int num_disp, int win, int cost, int stages,
                           int16_t* d_disp16, const sv_map_out* out, void* stream);

/* Frame-sharded batch over several devices from ONE host process:
 * replaces the reference's per-frame loop over create_depth_map (depth_map.py:837-946,
 * called once per captured frame; fused_depth_map.py:2591-2598 submits frames to a worker
 * pool).  Host frames f of left/right at + f*H*W*channels (channels 1 = gray, 3 = BGR);
 * outputs dense per frame (+ f*H*W).  Frames are split into ndev contiguous shards; context
 * k (its own device and stream) stages, computes and returns shard k on its own host
 * thread, concurrently with the others.  Every context must be distinct; the post-
 * processing is create_depth_map's (depth_final, disparity, depth_normalized). */
int sv_multi_gpu_batch(sv_ctx* const* ctxs, int ndev, const uint8_t* left, const uint8_t* right, int n_frames,
                       int H, int W, int channels, int min_disp, int num_disp, int win, int cost, float min_depth,
                       float max_depth, float depth_range, float min_disp_global, float* depth_final,
                       float* disparity, uint8_t* depth_normalized);
/* ---- multi-GPU: RCCL communicators + device-side gathers --------
 * The reference has no distributed code; its unit of work is one frame pair per call
 * (fused_depth_map.py:2591-2598 submits frames to a worker pool, depth_map.py:1181-1183
 * calls create_depth_map once per frame).  The MI355X build shards frames (C4) or the row
 * bands of one frame (C5) over GPUs and gathers the finished maps to one device over xGMI.
 * RCCL (librccl.so.1) is loaded with dlopen on first use.
 *   sv_comm_init_rank   one process per GPU (ncclCommInitRank; the id comes from one rank's
 *                       sv_comm_unique_id, shared out of band)
 *   sv_comm_init_all    one process, ndev distinct devices (ncclCommInitAll); comms[k] has
 *                       rank k
 *   sv_comm_barrier / sv_comm_allreduce_max_f64   blocking, one communicator per process
 *   sv_comm_gatherv     rank k's send_bytes land at d_recv + recv_offsets[k] on `root`
 *                       (ncclSend/ncclRecv in one group; the root's own block is a device
 *                       copy unless it is already in place); enqueued on `stream` (NULL =
 *                       the communicator's own stream, which nothing orders against the
 *                       caller's compute streams: pass the stream the data was produced on) */
typedef struct sv_comm sv_comm;
#define SV_COMM_ID_BYTES 128
int sv_comm_available(void);
int sv_comm_unique_id(uint8_t* id);
/* sv_comm_init_rank: non-blocking ncclCommInitRankConfig polled until it completes or
 * timeout_s seconds pass (<= 0: no limit); on an error or the deadline the half-built
 * communicator is aborted (ncclCommAbort) and -EHIP returned, so a rank whose peers failed
 * during bootstrap comes back instead of blocking forever. */
int sv_comm_init_rank(int device, int nranks, int rank, const uint8_t* id, double timeout_s,
                      sv_comm** out);
int sv_comm_init_all(int ndev, const int* devices, sv_comm** comms);
void sv_comm_destroy(sv_comm* comm);
int sv_comm_rank(sv_comm* comm, int* rank, int* nranks, int* device);
int sv_comm_barrier(sv_comm* comm);
int sv_comm_allreduce_max_f64(sv_comm* comm, double* value);
int sv_comm_gatherv(sv_comm* comm, const void* d_send, uint64_t send_bytes, void* d_recv,
                    const uint64_t* recv_offsets, const uint64_t* recv_bytes, int root, void* stream);
/* The inverse of sv_comm_gatherv: the root's send_bytes[k] bytes at d_send + send_offsets[k]
 * land in rank k's d_recv (recv_bytes); the root's own block is a device copy unless it is
 * already in place.  Enqueued on `stream` (NULL = the communicator's stream: the caller then
 * orders it against its own streams). */
int sv_comm_scatterv(sv_comm* comm, const void* d_send, const uint64_t* send_offsets,
                     const uint64_t* send_bytes, void* d_recv, uint64_t recv_bytes, int root,
                     void* stream);
int sv_comm_synchronize(sv_comm* comm);

/* Gather-only map formats (north_star: "a trivial RCCL gather of the final disparity rows"):
 *   SV_MAP_M16  int16 x16 medians (OpenCV's fixed-point disparity after medianBlur,
 *               depth_map.py:909-912), 2 B/px over xGMI
 *   SV_MAP_D8   u8 disparity indices median / 16 - (min_disp - 1) (0 = invalid), 1 B/px:
 *               exact for the integer-disparity costs (SAD / SSD / HOG) with num_disp <= 255 */
#define SV_MAP_M16 1
#define SV_MAP_D8 2

/* One process driving ndev contexts; replaces the reference's per-frame loop
 * over create_depth_map (depth_map.py:837-946; fused_depth_map.py:2591-2598 submits frames to a
 * worker pool) and returns the disparity rows the reference returns (depth_map.py:909-912).
 *   shard SV_SHARD_FRAMES (C4): context k computes its n_frames[k] frames at left[k] / right[k]
 *         (+ z*frame_stride bytes, on its own device); outputs dense in context order (frame z
 *         of context k at index sum(n_frames[:k]) + z).
 *   shard SV_SHARD_ROWS (C5): ONE frame; context k computes output rows
 *         [H*k/ndev, H*(k+1)/ndev) (window and median halos read locally, so the bands
 *         reassemble bit-exactly); n_frames and frame_stride unused.  inputs:
 *           SV_INPUTS_RESIDENT  every context holds the full gray frame (left[k] on its device)
 *           SV_INPUTS_SCATTER   the frame is on the root only (left[0]); context k > 0 first
 *                               receives the input rows its band reads (sv_band_rows_in) over
 *                               RCCL / peer copies (profiled as SV_K_SCATTER on the root)
 *           SV_INPUTS_HOST      the frame is in HOST memory (left[0], pinned for overlap: see
 *                               sv_host_register); every context uploads its own band's input
 *                               rows over its own PCIe link (no xGMI scatter; SV_K_H2D)
 *         Frames mode takes SV_INPUTS_RESIDENT only.
 * out (on ctxs[0]'s device) selects what the root holds: create_depth_map's outputs
 * (mode SV_POST_DEPTH with disparity, out_a, out_u8: the peers' maps cross xGMI as int16 x16
 * and are expanded on the root, k_post_m16 profiled as SV_K_POST), or gather-only the map of
 * every frame / the full frame as med16 (SV_MAP_M16) or d8 (SV_MAP_D8), nothing expanded.
 * comms (nullable; else comms[k] is rank k of an ndev-rank communicator on ctxs[k]'s device):
 * gathers / scatters as RCCL send/recv over xGMI; NULL: hipMemcpyPeerAsync (a plain device copy
 * when two contexts share a device).  Returns after enqueueing: the outputs are complete once
 * ctxs[0]'s stream is (sv_synchronize(ctxs[0])). */
#define SV_SHARD_FRAMES 0
#define SV_SHARD_ROWS 1
#define SV_INPUTS_RESIDENT 0
#define SV_INPUTS_SCATTER 1
#define SV_INPUTS_HOST 2
int sv_multi_gpu_dev(sv_ctx* const* ctxs, sv_comm* const* comms, int ndev, int shard, int inputs,
                     const uint8_t* const* left, const uint8_t* const* right, const int* n_frames,
                     int H, int W, int pitch, int64_t frame_stride, int min_disp, int num_disp,
                     int win, int cost, const sv_map_out* out);

/* Row bands of a `world`-way row tiling for rank `rank`: out6 = {r0, r1 (output rows), h0, h1
 * (disparity rows incl. the median halo), in0, in1 (input rows the band reads)}.  Device
 * buffers holding only input rows [in0, in1) must keep SV_BAND_MARGIN spare rows above and
 * below them (read-ahead of the row pipelines; never used as data). */
#define SV_BAND_MARGIN 8
int sv_band_rows_in(int H, int rank, int world, int win, int cost, int* out6);

int sv_harris_dev(sv_ctx* ctx, const uint8_t* d_gray, int H, int W, int pitch, float* d_out,
                  void* stream);
/* Harris response of n_frames gray frames (frame z at d_gray + z*frame_stride bytes, output
 * dense at d_out + z*H*W floats), one launch for the batch (C2: Harris beside the disparity
 * of a frame stream). */
int sv_harris_batch_dev(sv_ctx* ctx, const uint8_t* d_gray, int n_frames, int H, int W, int pitch,
                        int64_t frame_stride, float* d_out, void* stream);
int sv_hog_hist_dev(sv_ctx* ctx, const uint8_t* d_gray, int H, int W, int pitch, int win,
                    int row0, int row1, uint16_t* d_out, void* stream);

/* ---- rectification ---------------------------------------
 * K: 3x3 camera matrix, row-major doubles.  dist: ndist in {0, 4, 5, 8, 12, 14} OpenCV
 * distCoeffs (k1 k2 p1 p2 [k3 [k4 k5 k6 [s1 s2 s3 s4 [tx ty]]]]; a nonzero tilt is
 * SV_EINVAL).  R: 3x3 rectification rotation or NULL (identity).  P: new camera matrix,
 * 3 x p_cols row-major (p_cols 3 or 4; NULL = K).  Maps (CV_16SC2 + CV_16UC1 layout, dense
 * H x W): map1 = int16 (x, y) pairs of the source pixel, map2 = (y & 31) * 32 + (x & 31) of
 * the 1/32-pixel fraction.  Rounding of the f64 source position follows cvRound. */
int sv_init_undistort_rectify_map(sv_ctx* ctx, const double* K, const double* dist, int ndist,
                                  const double* R, const double* P, int p_cols, int H, int W,
                                  int16_t* map1, uint16_t* map2);
int sv_init_undistort_rectify_map_dev(sv_ctx* ctx, const double* K, const double* dist, int ndist,
                                      const double* R, const double* P, int p_cols, int H, int W,
                                      int16_t* d_map1, uint16_t* d_map2, void* stream);

/* remap INTER_LINEAR, BORDER_CONSTANT 0: src sH x sW x channels (1 or 3) u8 with row pitch
 * `stride` bytes; map1/map2 (map2 nullable = integer maps) and dst are H x W.  Host memory. */
int sv_remap(sv_ctx* ctx, const uint8_t* src, int sH, int sW, int channels, int stride,
             const int16_t* map1, const uint16_t* map2, int H, int W, uint8_t* dst);
/* Device version over a batch of n_frames sources (frame z at d_src + z*src_frame_stride,
 * output at d_dst + z*dst_frame_stride), one launch.  gray_out (channels == 3 only) writes
 * cvtColor(remap(src), BGR2GRAY) instead of the BGR result: the rectified gray image the
 * matcher reads, in one pass. */
int sv_remap_dev(sv_ctx* ctx, const uint8_t* d_src, int sH, int sW, int channels, int src_pitch,
                 int64_t src_frame_stride, const int16_t* d_map1, const uint16_t* d_map2, int H, int W,
                 int gray_out, uint8_t* d_dst, int dst_pitch, int64_t dst_frame_stride, int n_frames,
                 void* stream);
/* apply_stereo_rectification with device-resident maps: host left/right (sH x sW x channels,
 * row pitch `stride`) -> host rectified left/right (H x W x channels, dense). */
int sv_rectify_pair(sv_ctx* ctx, const int16_t* d_map1_left, const uint16_t* d_map2_left,
                    const int16_t* d_map1_right, const uint16_t* d_map2_right, int H, int W,
                    const uint8_t* left, const uint8_t* right, int sH, int sW, int channels, int stride,
                    uint8_t* out_left, uint8_t* out_right);

/* cv2.resize(src, (dW, dH)) INTER_LINEAR for u8 gray/BGR (fused_depth_map.py:474-476 and
 * :2498-2507, depth_map.py:757-776, ensure_same_size depth_map.py:39-71): OpenCV's
 * fixed-point two-pass bilinear; an exact 2x downscale is OpenCV's INTER_AREA fast path. */
int sv_resize_linear(sv_ctx* ctx, const uint8_t* src, int sH, int sW, int channels, int stride,
                     uint8_t* dst, int dH, int dW);
int sv_resize_linear_dev(sv_ctx* ctx, const uint8_t* d_src, int sH, int sW, int channels,
                         int src_pitch, int64_t src_frame_stride, uint8_t* d_dst, int dH, int dW,
                         int dst_pitch, int64_t dst_frame_stride, int n_frames, void* stream);

/* ---- SGBM-3WAY mode -----------------------------------------
 * cv2.StereoSGBM_create(minDisparity, numDisparities, blockSize, P1, P2, disp12MaxDiff,
 * preFilterCap, uniquenessRatio, speckleWindowSize, speckleRange, MODE_SGBM_3WAY)
 * .compute(left, right) (depth_map.py:894-909): int16 x16 map, invalid = (minD-1)*16.
 * Semantics in oracle/sv_sgbm_oracle.py (one stripe; int32 aggregation).  Limits:
 * num_disp <= 512, block_size odd <= 15, P2 < 349525, P1 < P2 (P2 = max(P2, P1+1)).
 * disp12MaxDiff < 0 disables the left-right check; speckleWindowSize <= 0 the filter. */
int sv_sgbm(sv_ctx* ctx, const uint8_t* left, const uint8_t* right, int H, int W, int channels,
            int stride, int min_disp, int num_disp, int block_size, int P1, int P2,
            int disp12_max_diff, int pre_filter_cap, int uniqueness_ratio,
            int speckle_window_size, int speckle_range, int16_t* disp16);
int sv_sgbm_dev(sv_ctx* ctx, const uint8_t* d_left, const uint8_t* d_right, int H, int W, int pitch,
                int min_disp, int num_disp, int block_size, int P1, int P2, int disp12_max_diff,
                int pre_filter_cap, int uniqueness_ratio, int speckle_window_size,
                int speckle_range, int16_t* d_disp16, int out_pitch, void* stream);

/* cv2.filterSpeckles(img, newVal, maxSpeckleSize, maxDiff) on an int16 map, in place: the
 * speckle stage of StereoSGBM (OpenCV calib3d, called from stereo.compute at
 * depth_map.py:909).  4-connected regions whose neighbours differ by <= max_diff and that
 * hold <= max_speckle_size pixels are set to new_val; max_speckle_size <= 0 is a no-op. */
int sv_filter_speckles(sv_ctx* ctx, int16_t* img, int H, int W, int new_val, int max_speckle_size, int max_diff);
int sv_filter_speckles_dev(sv_ctx* ctx, int16_t* d_img, int H, int W, int pitch, int new_val,
                           int max_speckle_size, int max_diff, void* stream);

/* ---- reductions around the path ----------------------------
 * Image statistics of detect_camera_occlusion (fused_depth_map.py:131-301) for one image
 * or a pair (img1 nullable): per 48x48 block of compute_block_homogeneity
 * (bh = max(1, H/48) x bw = max(1, W/48) blocks, partial edge tiles excluded as in the
 * reference) the exact sum and sum of squares of the gray values, and the 256-bin
 * histogram of the whole image (cv2.calcHist).  channels 3 = BGR, converted with the
 * cvtColor BGR2GRAY fixed point first.  Outputs per image: block_sum/block_sq [bh*bw],
 * hist [256]; the pair's second image follows the first. */
int sv_frame_stats(sv_ctx* ctx, const uint8_t* img0, const uint8_t* img1, int H, int W, int channels,
                   int stride, uint32_t* block_sum, uint32_t* block_sq, uint32_t* hist);
/* The device version, over a batch of n_frames images or pairs in one launch (image z of the
 * batch: img0 / img1 of frame z / per at + (z / per) * frame_stride bytes, per = 2 with
 * d_img1, else 1); outputs dense per image z: block moments [n_img][bh*bw], hist [n_img][256].
 * detect_camera_occlusion runs once per checked frame (fused_depth_map.py:2515-2522); a
 * stream of queued frames is one launch plus one fold. */
int sv_frame_stats_batch_dev(sv_ctx* ctx, const uint8_t* d_img0, const uint8_t* d_img1, int n_frames,
                             int64_t frame_stride, int H, int W, int channels, int pitch,
                             uint32_t* d_block_sum, uint32_t* d_block_sq, uint32_t* d_hist,
                             void* stream);

/* Order statistics of a float32 device array for np.percentile (calibrate_midas_to_stereo
 * fused_depth_map.py:1169-1257, normalize_to_stereo_range :1503-1554) with the reference's
 * masks as predicates: mask_mode 0 = all elements, 1 = elements > 0 (stereo_disparity > 0),
 * 2 = elements whose d_mask value > thr (stereo_confidence > 0.7).  sv_select_count_batch gives
 * the number of selected elements and of NaNs among them (np.percentile returns nan if
 * any); sv_select_ranks_batch gives the values of the given 0-based ranks of the ascending
 * sorted selection (nranks <= 4; radix select in three passes of 11/11/10 bits).  Both
 * block until the result is on the host and take a batch of n_arrays <= 16 arrays of n
 * elements (array y at d_x + y * x_stride elements, its mask at d_mask + y * mask_stride; one
 * array: n_arrays = 1): one launch + one fold per radix pass for the whole batch (e.g. the
 * disparity maps of queued frames).  selected / nans: [n_arrays]; ranks / values:
 * [n_arrays][nranks]. */
int sv_select_count_batch(sv_ctx* ctx, const float* d_x, int64_t n, int64_t x_stride, int n_arrays,
                          int mask_mode, const float* d_mask, int64_t mask_stride, float thr,
                          int64_t* selected, int64_t* nans);
int sv_select_ranks_batch(sv_ctx* ctx, const float* d_x, int64_t n, int64_t x_stride, int n_arrays,
                          int mask_mode, const float* d_mask, int64_t mask_stride, float thr,
                          const int64_t* ranks, int nranks, float* values);
/* Elementwise epilogues: mode 0: out = fc + ((x - fa) / fb) * fd in float32, op by op;
 * mode 1: out = float32(float64(x) * ds + doff); mode 2: out = fc. */
int sv_affine_f32_dev(sv_ctx* ctx, const float* d_x, int64_t n, int mode, float fa, float fb,
                      float fc, float fd, double ds, double doff, float* d_out, void* stream);

/* cv2.resize(x, (dW, dH), INTER_LINEAR) of a float32 HxW map (calibrate_midas_to_stereo,
 * fused_depth_map.py:1216-1217): OpenCV's float path, S0*b0 + S1*b1 without contraction.
 * Pitches in bytes. */
int sv_resize_linear_f32_dev(sv_ctx* ctx, const float* d_src, int sH, int sW, int src_pitch,
                             float* d_dst, int dH, int dW, int dst_pitch, void* stream);

/* ---- device memory helpers ----------------------------------------------------------
 * sv_copy_to_device / sv_copy_to_host: stream NULL = synchronous on the context stream (the
 * download first waits for the context's enqueued work); a stream = enqueued on it and
 * returned at once (the host buffer must stay valid until the stream reaches the copy, and be
 * page-locked — sv_host_register — for the copy to overlap device work). */
int sv_dev_alloc(sv_ctx* ctx, uint64_t bytes, void** out);
int sv_dev_free(sv_ctx* ctx, void* p);
int sv_copy_to_device(sv_ctx* ctx, void* dst, const void* src, uint64_t bytes, void* stream);
int sv_copy_to_host(sv_ctx* ctx, void* dst, const void* src, uint64_t bytes, void* stream);

/* Page-lock a host range and make it device-visible (hipHostRegister, portable).  Output
 * arrays of the host-buffer entry points (sv_depth_map, sv_depth_map_color,
 * sv_stereo_scaled, sv_stereo_scaled_color) that lie inside registered ranges are filled by
 * DMA from the device epilogue instead of by the host expansion of the int16 medians; the
 * results are identical.  A range stays registered until sv_host_unregister(ptr), which
 * takes the same start pointer.  No reference counterpart: an engine-side optimisation of
 * the numpy outputs depth_map.py:937-939 returns. */
int sv_host_register(void* ptr, uint64_t bytes);
int sv_host_unregister(void* ptr);

/* Host-side stage timings of the host-buffer entry points (process-wide, off by default):
 * ms6 = accumulated {prepare, stage + issue (the pageable uploads are synchronous), wait for
 * the first output piece, host expansion, wait for the rest, total} milliseconds over `calls`
 * calls since the last reset.  The device side of the same calls is the context's event
 * profile (sv_profile_enable): SV_K_H2D (one event pair per image upload), SV_K_GRAY,
 * SV_K_MATCH, SV_K_MEDIAN and SV_K_D2H. */
int sv_host_profile_enable(int enable);
int sv_host_profile_read(double* ms6, long long* calls, int reset);

/* ---- profiling: HIP events around every kernel this context launches -------------- */
int sv_profile_enable(sv_ctx* ctx, int on);
/* Waits for the recorded events and returns the accumulated device time and launch count
 * of kernel `kernel` (sv_kernel) since the last reset. */
int sv_profile_read(sv_ctx* ctx, int kernel, double* total_ms, long long* count);
int sv_profile_reset(sv_ctx* ctx);
/* Device time between two points of a stream (HIP events): sv_timer_begin records the
 * first, sv_timer_end the second, waits for it and returns the elapsed milliseconds.  For
 * timing a run of back-to-back launches (one event pair, so small kernels are not
 * dominated by per-launch event overhead). */
int sv_timer_begin(sv_ctx* ctx, void* stream);
int sv_timer_end(sv_ctx* ctx, void* stream, double* ms);
/* Caller-delimited profiling region on `stream` (NULL = the context's stream), counted under
 * `kernel` like a launch when profiling is enabled (a no-op otherwise): e.g. the RCCL gather a
 * process enqueues itself through sv_comm_gatherv (SV_K_GATHER).  Regions do not nest. */
int sv_profile_region_begin(sv_ctx* ctx, int kernel, void* stream);
int sv_profile_region_end(sv_ctx* ctx, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* STEREOVISION_AMD_H */
