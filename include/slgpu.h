/*
 * slgpu.h -- C ABI of libslgpu.so, the MI355X (gfx950) implementation of the
 * structured-light reconstruction hot path of
 * Nuttoty/Structured_Light_for_3D_Model_Replication:
 *
 *   gray_decode(folder, n_cols, n_rows)          server/sl_system.py:508-580
 *   reconstruct_point_cloud(col, row, mask, tex, calib)  server/sl_system.py:584-653
 *   generate_cloud(scan_dir, calib_file)         server/sl_system.py:483-694
 *
 * The reference has no FFI; its boundary is the Python function triple above
 * (called from server/gui.py:563, multi_point_cloud_process.py:206-212 and
 * Old/process_cloud.py:231-233).  This header is what a ctypes binding of that
 * triple calls; see INTEGRATION.md for the binding.
 *
 * Conventions
 *  - Every entry point returns SL_OK (0) or a negative SL_E* code; the message
 *    of the last failure on a context is sl_ctx_last_error().
 *  - Pointers named "device" are HIP device pointers owned by the caller.  The
 *    library owns only the calibration tables and scratch inside a context.
 *  - A context belongs to one device; calls on one context must be serialised
 *    by the caller (one context per thread or per device).  There is no global
 *    state, so independent contexts may be used concurrently.
 *  - Work is enqueued on `stream` (a hipStream_t; NULL = default stream) and is
 *    asynchronous unless the function says otherwise.
 */
#ifndef SLGPU_H
#define SLGPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SL_ABI_VERSION 1

#define SL_OK 0
#define SL_EINVAL (-1)    /* bad argument -> Python ValueError                          */
#define SL_EINDEX (-2)    /* dangling odd image reached: the IndexError of
                             sl_system.py:553-554                                      */
#define SL_EHIP (-3)      /* HIP runtime failure -> RuntimeError                        */
#define SL_ENOCALIB (-4)  /* sl_set_calib not called / shape mismatch -> ValueError       */
#define SL_ETIMEOUT (-5)  /* reserved                                                     */
#define SL_ECAPACITY (-6) /* output capacity smaller than the pixel count -> ValueError   */
#define SL_EIO (-7)       /* file could not be written -> OSError                        */

/* mask_mode */
#define SL_MASK_ADAPTIVE 0 /* white > 1.5*pct95(black) & contrast > 0.05*max(contrast):
                              sl_system.py:526-535                                      */
#define SL_MASK_FIXED 1    /* white > 40 & contrast > 10:
                              multi_point_cloud_process.py:36-38, Old/process_cloud.py:47-49 */

/* xyz_dtype */
#define SL_XYZ_F32 0 /* 12 B/point, the round-to-nearest fp32 of the reference's f64   */
#define SL_XYZ_F64 1 /* 24 B/point, bit-identical to the reference's f64              */
/* 12 B/point, f32 arithmetic: per-coordinate relative error vs the reference's f64
 * <= (11 + 10*16) * 2^-24 ~ 1.0e-5 (north-star tolerance 1e-4).  Points with
 * condition number sum|n_i r_i| / |n.r| > 16 are computed exactly.  Applies when
 * Oc = 0, no Nc table and no pose; otherwise identical to SL_XYZ_F32.          */
#define SL_XYZ_F32_FAST 2

typedef struct sl_ctx sl_ctx;

int sl_abi_version(void);

/* Create a context on HIP device `device`.  Replaces nothing in the reference
 * (which keeps no state); the context holds the calibration tables. */
int sl_ctx_create(int device, sl_ctx** out);
void sl_ctx_destroy(sl_ctx* ctx);
const char* sl_ctx_last_error(const sl_ctx* ctx);

/* Pre-size the context's scratch for up to `max_views` views of `max_px`
 * pixels each (and the histograms of a whole launch group) so that later calls
 * allocate nothing (required before stream capture into a hipGraph).  Calls
 * grow scratch on demand otherwise.
 * Graphs: any sequence of calls captured on one stream replays any number of
 * times, in any order with other work on the context.  Nothing a launch group
 * accumulates into depends on the host's view of the sequence: the super-block
 * sums live in two buffers whose alternation is kept on the device (the
 * producer, k_decode or k_count, reads a selector word, accumulates into that
 * buffer and zeroes the OTHER one, whose last reader -- the previous group's
 * k_cloud -- is done; the consumer only flips the selector, so the buffer it
 * read keeps its sums until the next producer zeroes it); the adaptive mask's
 * histograms are zeroed by their last reader (an arrival counter).  The one
 * thing that crosses a call boundary, a histogram pass queued by
 * sl_stack_next, is taken only by a call in the same capture (a graph's first
 * call therefore runs its own histogram pass; a pass the graph's last call
 * queues is cleared by the next call that does not take it). */
int sl_ctx_reserve(sl_ctx* ctx, int64_t max_views, int64_t max_px);

/* Upload calibration for an H x W camera (the calib.mat fields loaded at
 * sl_system.py:493-504).  Host pointers:
 *   cam_K   3x3 row-major f64            (calib["cam_K"])
 *   Oc      3 f64                         (calib["Oc"], zeros from calibrate_final)
 *   planes  Wp x 4 row-major f64 (n0,n1,n2,d) (calib["wPlaneCol"] transposed as at
 *           sl_system.py:591)
 *   Nc      3 x (H*W) row-major f64, or NULL (calib["Nc"]).  When Nc equals the
 *           pinhole rays of cam_K bit for bit (always, for calibrate_final output)
 *           it is not uploaded and rays are recomputed on the fly; otherwise it
 *           is kept on the device and read per pixel, as sl_system.py:605-606. */
int sl_set_calib(sl_ctx* ctx, int H, int W, const double* cam_K, const double* Oc,
                 const double* planes, int Wp, const double* Nc);

/* Fused gray_decode + reconstruct_point_cloud over `n_views` views.
 *
 * stack      device, view v at stack + v*stack_view_stride: n_img planes of H*W
 *            uint8 in the reference's sorted-file order [white, black, (pattern,
 *            inverse) x bits...] (sl_system.py:510-520, 553-557).
 * n_cols/n_rows  projector stripes; ceil(log2()) gives the bit counts exactly as
 *            sl_system.py:538-539 (each must be in [1, 65536]).
 * tex_bgr    device, [H][W][3] BGR per view (the colour imread of file 0,
 *            sl_system.py:580), or NULL to use the white plane replicated.
 * poses      device, n_views x 4x4 row-major f64 applied to every point of the
 *            view (turntable merge epilogue), or NULL.
 * col_out, row_out  device int32 [n_views][H][W], full frame, unmasked (may be
 *            NULL).  mask_out device uint8 (0/1) [n_views][H][W] (may be NULL).
 * xyz_out    device, out_capacity x 3 of f32 or f64 (xyz_dtype), NULL for
 *            decode only.  bgr_out device uint8 out_capacity x 3 (NULL allowed
 *            only together with xyz_out).  Both 16-byte aligned.
 * view_offsets  device int64 [n_views+1]: points of view v occupy
 *            [view_offsets[v], view_offsets[v+1]) of the merged cloud, in
 *            ascending pixel order inside each view (np.where order,
 *            sl_system.py:601).  Required when xyz_out is given.
 * out_capacity  must be >= n_views*H*W.
 *
 * Row planes are read only if row_out is non-NULL (the cloud does not use the
 * row code: sl_system.py:584-653 reads only col_map).
 * Returns SL_EINDEX / SL_EINVAL for the stack lengths on which the reference
 * raises IndexError / ValueError. */
int sl_decode_triangulate(sl_ctx* ctx, const uint8_t* stack, int64_t stack_view_stride,
                          int n_views, int n_img, int H, int W, int n_cols, int n_rows,
                          const uint8_t* tex_bgr, int64_t tex_view_stride, int mask_mode,
                          const double* poses, int32_t* col_out, int32_t* row_out,
                          uint8_t* mask_out, void* xyz_out, int xyz_dtype, uint8_t* bgr_out,
                          int64_t out_capacity, int64_t* view_offsets, void* stream);

/* Masked-pixel counts (the "Processing {N} valid pixels..." line of
 * reconstruct_point_cloud, sl_system.py:601-602: N = np.count_nonzero(mask)):
 * arms the NEXT sl_decode_triangulate on this context (that call only; it is
 * consumed even when the call fails) to write the number of pixels of view v
 * that pass the mask into device_counts[v] (device int64 [n_views], 8-byte
 * aligned), asynchronously on that call's stream.  NULL disarms.  Without it
 * the kernels count nothing. */
int sl_mask_counts_to(sl_ctx* ctx, int64_t* device_counts);

/* Stack readiness for the NEXT sl_decode_triangulate on this context (that
 * call only; consumed even when the call fails): the stack and texture are in
 * place once `event` (a hipEvent_t recorded by the caller) has completed --
 * the call's work waits for it on its stream -- or already now when `event`
 * is NULL.  Results are unchanged.  (Round 3 ran the histogram pass of such a
 * call on a side stream beside the previous call's triangulation: measured
 * slower than sl_stack_next's pre-stats, DESIGN.md 5.2, and removed.) */
int sl_stack_ready(sl_ctx* ctx, void* event);

/* The call AFTER the coming one (a stream of views): arms the NEXT
 * sl_decode_triangulate on this context (that call only; consumed even when it
 * fails) to compute, beside its own triangulation (extra workgroups of its last
 * k_cloud launch), the adaptive-mask histograms (sl_system.py:526-528) of the
 * first launch group of `stack` [n_views][...] (view stride stack_view_stride,
 * 16-byte aligned, the same frame size as the coming call).  The call after it
 * then starts with its decode -- when it is on this context, reads that same
 * stack pointer, stride, view count and frame size with the adaptive mask,
 * nothing ran on the context in between, and both calls are enqueued in the
 * same stream capture (or both outside one); otherwise it computes its
 * histograms itself.  The caller promises that `stack` holds the next call's images, in
 * place by the time the coming call's work starts on its stream, and unchanged
 * until the next call.  Results are unchanged.  NULL disarms, and also drops a
 * pass an earlier call queued for the next one (that call then computes its
 * own histograms: e.g. after a failed graph capture of chained calls).  A
 * queued pass is taken or dropped by the very next call on the context, even
 * one that fails its argument checks (never by a later one).
 * Within one call of several launch groups (more than 65536 chunks of 1024
 * pixels) the same happens without any declaration: group g's k_cloud computes
 * group g + 1's histograms, so only the first group can need a k_stats launch. */
int sl_stack_next(sl_ctx* ctx, const uint8_t* stack, int64_t stack_view_stride, int n_views);

/* A prepared call: sl_decode_triangulate's arguments (without the stream),
 * checked once and kept, so that a stream of views through the same resident
 * buffers (a ring of stack slots, reused outputs) re-enqueues it with two
 * arguments -- what a host-bound caller of small frames spends its time on is
 * the per-call argument marshalling, not the kernels.  sl_call_run is exactly
 * sl_decode_triangulate with the kept arguments on `stream` (the same checks,
 * results and errors); the buffers must stay valid until sl_call_destroy. */
typedef struct sl_call sl_call;
int sl_call_prepare(sl_ctx* ctx, const uint8_t* stack, int64_t stack_view_stride, int n_views, int n_img,
                    int H, int W, int n_cols, int n_rows, const uint8_t* tex_bgr, int64_t tex_view_stride,
                    int mask_mode, const double* poses, int32_t* col_out, int32_t* row_out, uint8_t* mask_out,
                    void* xyz_out, int xyz_dtype, uint8_t* bgr_out, int64_t out_capacity, int64_t* view_offsets,
                    sl_call** out);
int sl_call_run(sl_call* call, void* stream);
void sl_call_destroy(sl_call* call);

/* reconstruct_point_cloud on caller-supplied maps (sl_system.py:584-653).
 * col_map device int32 [n_views][H][W]; mask device uint8 [n_views][H][W]
 * (non-zero = valid); tex_bgr device [n_views][H][W][3].  Outputs as above. */
int sl_triangulate_maps(sl_ctx* ctx, const int32_t* col_map, const uint8_t* mask,
                        const uint8_t* tex_bgr, int n_views, int H, int W,
                        const double* poses, void* xyz_out, int xyz_dtype, uint8_t* bgr_out,
                        int64_t out_capacity, int64_t* view_offsets, void* stream);

/* Synchronise `stream` and report any HIP failure of the work enqueued so far
 * on this context.  Blocking. */
int sl_sync(sl_ctx* ctx, void* stream);

/* Adaptive-mask diagnostics of the last sl_decode_triangulate (blocking):
 * noise_floor = np.percentile(black, 95) and dynamic_range = max(white-black)
 * as float32 (sl_system.py:527-528), and the integer thresholds the kernel
 * compared against (white > thr_white, contrast > thr_contrast). */
int sl_last_thresholds(sl_ctx* ctx, int view, float* noise_floor, float* dynamic_range,
                       int* thr_white, int* thr_contrast);

/* Timing: with max_calls > 0, each later call (up to that many) records HIP
 * events on its stream before k_decode, k_count, k_cloud and after the call.
 * 0 disables.  Events between kernels add launch gaps: keep them out of
 * throughput measurements. */
int sl_profile_enable(sl_ctx* ctx, int max_calls);

/* Blocking: summed event time (ms) of k_decode, k_count and k_cloud over the
 * recorded calls since the last read, and their count; restarts recording. */
int sl_profile_read(sl_ctx* ctx, double* decode_ms, double* count_ms, double* cloud_ms, int* calls);

/* The last call's kernel path -- 0: k_decode + k_count + k_cloud; 1: [k_stats]
 * + k_decode + k_cloud, k_decode applying the mask and the point decision
 * (frames with W % 16 == 0, W, H <= 4096 and Wp <= 2048; sl_profile_* and
 * sl_time_kernels then report k_stats in the k_count slot) -- its number of
 * launch groups, and the pixels of its last launch group (what
 * sl_time_kernels re-runs).  Host only. */
int sl_last_launch_info(sl_ctx* ctx, int* path, int64_t* launches, int64_t* last_launch_px);

/* Blocking, measurement only: re-launches the kernels of the last launch group
 * of the previous sl_decode_triangulate / sl_triangulate_maps call `reps`
 * times each, back to back on its stream, and returns each kernel's average
 * duration from HIP events around the `reps` launches (the events' own cost
 * amortised).  The inputs the call consumed (histograms, block sums) are
 * rebuilt once first, untimed; k_cloud and k_count run first: the call's
 * outputs are rewritten with the same values.  Afterwards the context's
 * scratch is clean again: a histogram pass queued by sl_stack_next is dropped
 * (the next call computes its own).  Eager only: SL_EINVAL while that stream
 * is capturing into a graph. */
int sl_time_kernels(sl_ctx* ctx, int reps, double* decode_ms, double* count_ms, double* cloud_ms);

/* ASCII PLY of a cloud exactly as the reference writes it (sl_system.py:665-691,
 * multi_point_cloud_process.py:121-131): header, then per point
 * "%.4f %.4f %.4f %d %d %d\n" of x, y, z and the colour swapped from BGR to
 * RGB; %.4f correctly rounded, ties to even (what Python's f"{x:.4f}" prints).
 * Host memory, host code (no device needed); formatted on `threads` threads.
 * xyz is n x 3 f32 or f64 (xyz_dtype), bgr n x 3 uint8.
 * sl_format_ply: with out == NULL only *out_len is set (the byte size). */
int sl_format_ply(const void* xyz, int xyz_dtype, const uint8_t* bgr, int64_t n, int threads, char* out,
                  int64_t out_capacity, int64_t* out_len);
/* Write that text to `path` (replaces save_ply, sl_system.py:665-691).  A
 * large regular file already at `path` is renamed away and unlinked beside the
 * write rather than truncated in place (the same file results, faster);
 * symlinks and hard-linked files are written through / truncated as
 * open(path, "w") does.  The same for sl_write_ply_device / _binary. */
int sl_write_ply(const char* path, const void* xyz, int xyz_dtype, const uint8_t* bgr, int64_t n, int threads);

/* The same file from a cloud in device memory (xyz / bgr device pointers,
 * e.g. a call's outputs): the text is formatted on the device (one thread
 * per point, the host formatter's digit code) into context scratch, copied
 * back through a pinned buffer in chunks and written, the host formatting
 * nothing; byte-identical to sl_write_ply.  A cloud with a non-finite
 * coordinate or |x| >= 9e11 (printed through libc's %.4f) is copied back and
 * formatted on the host instead.  Blocking on `stream` (hipStream_t). */
int sl_write_ply_device(sl_ctx* ctx, const char* path, const void* xyz, int xyz_dtype, const uint8_t* bgr, int64_t n,
                        void* stream);

/* Binary little-endian PLY with the same header properties (float x y z,
 * uchar red green blue; colour swapped from BGR): 15-byte records, xyz rounded
 * to float32 when xyz_dtype is SL_XYZ_F64.  A compact binary form of the
 * reference's ASCII file (the merged cloud's Open3D-layout file, double xyz
 * and normals, is ply.save_ply_open3d). */
int sl_write_ply_binary(const char* path, const void* xyz, int xyz_dtype, const uint8_t* bgr, int64_t n,
                        int threads);

/* ---- merge stage (server/processing.py:116-182) ----
 * Open3D's PointCloud::VoxelDownSample and RemoveStatisticalOutliers on a
 * device cloud (xyz f64 [n][3], bgr u8 [n][3] or NULL).  Blocking on `stream`;
 * counts are returned on the host.  Parity vs Open3D is unpinned (not in this
 * image): oracle/merge_oracle.py restates the algorithms. */

/* One point per occupied voxel of edge voxel_size, grid origin min - voxel_size/2:
 * the mean of its points (summed in ascending index, f64) and of its colours
 * (as c/255, written back as round(clamp(mean)*255)).  Output in ascending
 * voxel key (ix, iy, iz) (Open3D: hash order); out arrays hold n points.
 * SL_EINVAL for voxel_size <= 0, "voxel_size is too small." (Open3D's check),
 * or a grid over 2e6 voxels per axis. */
int sl_voxel_downsample(sl_ctx* ctx, const double* xyz, const uint8_t* bgr, int64_t n, double voxel_size,
                        double* out_xyz, uint8_t* out_bgr, int64_t* out_n, void* stream);

/* Mean distance to the nb_neighbors (<= 32) nearest points, the point itself
 * included (exact kNN, f64) -> avg_dist[n] (device); keeps
 * 0 < avg < mean + std_ratio * std (Bessel): their indices, ascending, ->
 * out_index (device, capacity n), the count -> *out_n. */
int sl_statistical_outliers(sl_ctx* ctx, const double* xyz, int64_t n, int nb_neighbors, double std_ratio,
                            double* avg_dist, int64_t* out_index, int64_t* out_n, void* stream);

/* select_by_index: out[j] = in[index[j]] (device; bgr optional).  Asynchronous. */
int sl_select_by_index(sl_ctx* ctx, const double* xyz, const uint8_t* bgr, const int64_t* index, int64_t m,
                       double* out_xyz, uint8_t* out_bgr, void* stream);

/* In place p' = M p for a row-major 4x4 pose (device), rows in the order
 * ((m0 x + m1 y) + m2 z) + m3 -- PointCloud::Transform.  Asynchronous. */
int sl_transform_points(sl_ctx* ctx, double* xyz, int64_t n, const double* pose, void* stream);

/* PointCloud::EstimateNormals(KDTreeSearchParamHybrid(radius, max_nn)) on a
 * cloud without normals (processing.py:178: radius = 2 voxel, max_nn = 30):
 * per point, the neighbours with ((dx^2 + dy^2) + dz^2) < radius^2 (itself
 * included) in ascending (distance, index), the first max_nn; covariance from
 * their cumulants (identity below 3 neighbours); normal = Open3D's
 * FastEigen3x3 eigenvector of the smallest eigenvalue, (0, 0, 1) when zero ->
 * normals [n][3] f64 (device).  max_nn <= 32.  Blocking on `stream`. */
int sl_estimate_normals(sl_ctx* ctx, const double* xyz, int64_t n, double radius, int max_nn, double* normals,
                        void* stream);

/* registration_icp(source, target, max_distance, init,
 * TransformationEstimationPointToPlane()) of merge_pro_360 (processing.py:
 * 154-156), Open3D's RegistrationICP loop: every (moved) source point's
 * nearest target point with ((dx^2 + dy^2) + dz^2) < max_distance^2 (least
 * (d^2, index)); the point-to-plane step from those correspondences (JTJ and
 * JTr folded in source order, 64-point blocks left to right; the 6x6 system
 * by a pivoted LDLT as Eigen's (Open3D's A.ldlt().solve(b): zero pivots give
 * zero components, so a rank-deficient system still moves along the
 * directions it constrains); update = [Rz Ry Rx | t] of the solution);
 * transformation = update *
 * transformation; until |d fitness| < relative_fitness and |d rmse| <
 * relative_rmse, or max_iteration steps (Open3D's defaults: 30, 1e-6, 1e-6).
 * source / target / target_normals: device f64 [n][3]; init and the returned
 * transformation: host row-major 4x4; fitness = correspondences / n_src,
 * inlier_rmse = sqrt(sum d^2 / correspondences) of the last evaluation;
 * *iterations = steps taken.  Blocking on `stream`.  Parity vs Open3D is
 * unpinned (oracle/merge_oracle.py restates this arithmetic). */
int sl_icp_point_to_plane(sl_ctx* ctx, const double* source, int64_t n_src, const double* target,
                          const double* target_normals, int64_t n_tgt, double max_distance, const double* init,
                          int max_iteration, double relative_fitness, double relative_rmse, double* transformation,
                          double* fitness, double* inlier_rmse, int* iterations, void* stream);

/* ---- global registration (merge_pro_360's FPFH + RANSAC, processing.py:79-113) ----
 * Open3D's algorithms restated (parity unpinned: no Open3D in this image;
 * oracle/registration_oracle.py is the CPU restatement, bit-identical).
 *
 * KDTreeFlann::SearchHybrid(p, radius, max_nn) of every point of xyz [n][3]
 * (device f64): the points with ((dx^2 + dy^2) + dz^2) < radius^2 (itself
 * included) in ascending (d2, index), the first max_nn -> out_idx /
 * out_d2 [n][max_nn] and out_cnt [n] (device).  max_nn <= 1024.  Blocking.
 * Ties (a documented deviation): equal distances are ordered by index here
 * and in sl_estimate_normals / sl_compute_fpfh; nanoflann leaves them in its
 * KD-tree traversal order (an unstable sort), so with duplicate points Open3D
 * may pick another neighbour set or "self" entry.  No reference fixture covers
 * it; the oracle (oracle/registration_oracle.py) states the same rule, and
 * parity with Open3D stays unpinned. */
int sl_radius_search(sl_ctx* ctx, const double* xyz, int64_t n, double radius, int max_nn, int32_t* out_idx,
                     double* out_d2, int32_t* out_cnt, void* stream);

/* compute_fpfh_feature(pcd, KDTreeSearchParamHybrid(radius, max_nn))
 * (processing.py:91-94: radius 5 voxel, max_nn 100): per point its SPFH (the
 * pair features -- fdlibm acos / atan2 -- of its neighbours, 11 bins each,
 * 100 / (neighbours - 1) per pair) and the FPFH = the 1/d2-weighted sum of the
 * neighbours' SPFH, each third scaled to 100, + its own SPFH (zero for a
 * point without neighbours) -> feature [n][33] f64 (device; Open3D's
 * Feature.data_ transposed).  normals: [n][3] (estimate_normals).  Blocking. */
int sl_compute_fpfh(sl_ctx* ctx, const double* xyz, const double* normals, int64_t n, double radius, int max_nn,
                    double* feature, void* stream);

/* The nearest row of b [nb][dim] for every row of a [na][dim] (device f64;
 * dim == 33): nanoflann's L2 order (four dimensions at a time, then the
 * rest), ties to the lower index (a documented deviation: nanoflann's 1-NN
 * keeps the first candidate its tree traversal meets) -> out [na] (device
 * int32); -1 for a row with no distance below +inf (NaN features never match,
 * as nanoflann's strict compare).  Blocking. */
int sl_feature_nn(sl_ctx* ctx, const double* a, int64_t na, const double* b, int64_t nb, int dim, int32_t* out,
                  void* stream);

/* registration_ransac_based_on_feature_matching(source, target, source_feature,
 * target_feature, mutual_filter, max_distance,
 * TransformationEstimationPointToPoint(False), 3,
 * [CorrespondenceCheckerBasedOnEdgeLength(edge_similarity),
 *  CorrespondenceCheckerBasedOnDistance(max_distance)],
 * RANSACConvergenceCriteria(max_iteration, confidence)) (processing.py:98-111):
 * correspondences = feature nearest neighbours (mutual: both ways agree; fewer
 * than 0.1f * n_src mutual pairs: the one-way set; a source row without a
 * neighbour makes no pair); then Open3D's RANSAC loop
 * as one thread runs it -- iteration i draws correspondences
 * splitmix64(seed + (3 i + k + 1) * 0x9E3779B97F4A7C15) (k = 0..2; Open3D's
 * std::mt19937 draw is unseeded, so no run of it is reproducible), checks edge
 * lengths, fits Umeyama (Eigen's 3x3 JacobiSVD), checks distances, and
 * validates (fitness = source points with a target within max_distance / n,
 * inlier RMSE); the best by (fitness, then lower RMSE) updates the estimated
 * iteration count log(1 - confidence) / log(1 - inlier_ratio^3) -- evaluated
 * on the GPU in batches of hypotheses, walked in iteration order.
 * source / target [n][3], features [n][33]: device f64.  Host outputs: the
 * row-major 4x4 transformation (identity if nothing validated), fitness,
 * inlier_rmse, iterations run, validations (hypotheses that passed both
 * checkers) and the correspondence count (any output pointer but
 * transformation may be NULL).  Blocking on `stream`. */
int sl_ransac_feature_matching(sl_ctx* ctx, const double* source, int64_t n_src, const double* target, int64_t n_tgt,
                               const double* source_feature, const double* target_feature, int mutual_filter,
                               double max_distance, double edge_similarity, int max_iteration, double confidence,
                               uint64_t seed, double* transformation, double* fitness, double* inlier_rmse,
                               int* iterations, int* validations, int64_t* n_corres, void* stream);

/* Release the scratch buffers the merge entry points keep pooled for `device`
 * (kept otherwise for the process's lifetime, at most 16 GiB per device);
 * the bytes released -> *released_bytes (may be NULL). */
int sl_merge_pool_trim(int device, int64_t* released_bytes);

/* ---- multi-GPU gather ----
 * The merge's one exchange: every rank's cloud to `root` in rank order over
 * RCCL (opened with dlopen by soname, so a process that already holds
 * PyTorch's RCCL shares that copy).  One context per rank (GPU):
 *   sl_gather_unique_id  one rank makes the 128-byte id, shared out of band
 *                        (the Python side uses torch.distributed.broadcast_object_list);
 *   sl_gather_init       ncclCommInitRank on the context's device;
 *   sl_gather_counts     blocking: an ncclAllGather of one int64 per rank ->
 *                        counts_out[nranks] (host) on every rank, so the root
 *                        can size its buffers;
 *   sl_gather            grouped ncclSend / ncclRecv of xyz (f32 or f64, 3 per
 *                        point) and bgr (3 B per point) into the root's
 *                        xyz_out / bgr_out at exclusive-scan offsets of
 *                        `counts`; asynchronous on `stream`.
 * Replaces the sequential per-file merge of processing.py:116-140. */
int sl_gather_unique_id(uint8_t* id_out /* 128 bytes */);
int sl_gather_init(sl_ctx* ctx, int nranks, int rank, const uint8_t* id /* 128 bytes */);
int sl_gather_counts(sl_ctx* ctx, int64_t n_local, int64_t* counts_out, void* stream);
int sl_gather(sl_ctx* ctx, const void* xyz, int xyz_dtype, const uint8_t* bgr, const int64_t* counts, int root,
              void* xyz_out, uint8_t* bgr_out, void* stream);

/* The names of SURVEY.md §8(b): sl_decode_triangulate is already batched (V
 * views per call); sl_last_error is sl_ctx_last_error. */
int sl_decode_triangulate_batch(sl_ctx* ctx, const uint8_t* stack, int64_t stack_view_stride, int n_views,
                                int n_img, int H, int W, int n_cols, int n_rows, const uint8_t* tex_bgr,
                                int64_t tex_view_stride, int mask_mode, const double* poses, int32_t* col_out,
                                int32_t* row_out, uint8_t* mask_out, void* xyz_out, int xyz_dtype,
                                uint8_t* bgr_out, int64_t out_capacity, int64_t* view_offsets, void* stream);
const char* sl_last_error(const sl_ctx* ctx);

/* ---- calibration products (csrc/slcalib.hip) ----
 * Replaces the NumPy tail of SLSystem.calibrate_final (server/sl_system.py:348-403):
 * from the stereo parameters OpenCV estimated (cam_K = K1, proj_K = K2, R, T;
 * row-major 3x3 / 3) it derives, on the device,
 *   nc_out        [3][cam_h*cam_w]  unit camera rays, pixel v*cam_w + u (Nc, :353-365)
 *   plane_col_out [4][proj_w]       column planes (n0, n1, n2, d) (wPlaneCol as saved, :397-398, :408)
 *   plane_row_out [4][proj_h]       row planes (wPlaneRow, :401-402, :409)
 * (any output may be NULL; proj_w x proj_h = SCREEN_WIDTH x SCREEN_HEIGHT of
 * config.py).  Bit-identical to the reference's NumPy 2.2 / OpenBLAS 0.3.29
 * evaluation (3-term dots as left-to-right FMA chains).  Asynchronous. */
int sl_calib_products(sl_ctx* ctx, const double* cam_K, const double* proj_K, const double* R, const double* T,
                      int cam_w, int cam_h, int proj_w, int proj_h, double* nc_out, double* plane_col_out,
                      double* plane_row_out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SLGPU_H */
