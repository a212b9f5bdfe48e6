/*
 * dsplat_hip.h — C ABI of libdsplat_hip.so, the MI355X (gfx950) hot path of
 * yuehuarulian/my_depthsplat: the differentiable 3D-Gaussian tile rasterizer behind
 * src/model/decoder/cuda_splatting.py and the plane-sweep cost volume behind
 * src/model/encoder/unimatch/matching.py + mv_unimatch.py.
 *
 * Conventions (every entry point):
 *   - all array arguments are DEVICE pointers (HBM), fp32 unless typed otherwise,
 *     C-contiguous in the layout written next to them;
 *   - the library never allocates or frees: the caller owns every buffer
 *     (the Python layer allocates from the PyTorch-ROCm caching allocator);
 *   - all work is enqueued on `stream` (hipStream_t passed as void*); no host sync,
 *     no hipMalloc, so every call is hipGraph-capturable;
 *   - return 0 on success, non-zero on a bad argument or HIP error; the message is
 *     in dsplat_last_error() (thread-local). No exception crosses the ABI.
 *
 * Reference interfaces replaced (file:line in yuehuarulian/my_depthsplat):
 *   rasterizer  : diff_gaussian_rasterization.GaussianRasterizer.forward/backward,
 *                 called at src/model/decoder/cuda_splatting.py:112-123 (one call per
 *                 view there; here one call sequence renders a whole batch of views)
 *   cost volume : warp_with_pose_depth_candidates  src/model/encoder/unimatch/matching.py:24-90
 *                 fused with the correlation at   src/model/encoder/unimatch/mv_unimatch.py:494-505
 */
#ifndef DSPLAT_HIP_H
#define DSPLAT_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DSR_TILE 16          /* 16x16 pixel screen tiles (upstream BLOCK_X/BLOCK_Y) */
#define DSR_GEOM_STRIDE 12   /* floats per (view, gaussian) geometry record        */

/* One camera/view. Mirrors GaussianRasterizationSettings (cuda_splatting.py:98-111):
 * viewmatrix/projmatrix are the row-major storage of the TRANSPOSED torch matrices
 * (i.e. column-major world->camera and world->clip), campos = c2w[:3, 3]. `scene`
 * selects which Gaussian set [S] this view renders, replacing the per-view
 * `repeat(...)` of decoder_splatting_cuda.py:53-56; viewmatrix/projmatrix/campos are
 * those of the RESCALED camera when scale != 1. 176 bytes, device-resident. */
typedef struct dsr_camera {
    float viewmatrix[16];
    float projmatrix[16];
    float campos[3];
    float tanfovx;
    float tanfovy;
    float bg[3];
    int32_t scene;
    float scale;            /* scale-invariant rescale 1/near (cuda_splatting.py:63-70): the
                               kernel uses means*scale and cov*(scale*scale); 1 = off */
    int32_t _pad[2];
} dsr_camera;

/* Geometry record per (view, gaussian), DSR_GEOM_STRIDE floats:
 *   [0..1] pixel-space mean xy   [2..4] conic (a, b, c)   [5] opacity
 *   [6..8] rgb                   [9] view-space depth     [10] radius (int32 bits)
 *   [11] SH clamp mask (uint32 bits 0..2). radius == 0 <=> culled / not rendered. */

/* Build the camera array on the device from the reference's render_cuda inputs
 * (cuda_splatting.py:62-86 + projection.py:233-247 get_fov + :16-43 projection matrix):
 *   extrinsics [V,4,4] c2w, intrinsics [V,3,3] normalised, near/far [V], bg [V,3],
 *   view_scene [V] int32; scale_invariant != 0 applies the 1/near rescale.
 * Computed in double per view (torch does it in float32: agreement ~1e-7 relative). */
int dsr_build_cameras(int V, const float* extrinsics, const float* intrinsics, const float* near,
                      const float* far, const float* bg, const int32_t* view_scene,
                      int scale_invariant, dsr_camera* cams, uint32_t* zero_counts,
                      uint32_t n_zero, void* stream);
/* zero_counts / n_zero (optional): also zero n_zero words there — the seg_count array of the
 * dsr_project_bin / dsr_preprocess_fwd call that follows, which then gets
 * DSR_LAYOUT_COUNTS_ZEROED and skips its own zeroing launch. */

/* ---- rasterizer forward ------------------------------------------------------------
 * Replaces preprocessCUDA + tiles_touched (upstream K1). Per view v and gaussian g of
 * scene cams[v].scene: cull, EWA projection, conic, radius, SH->RGB (or colors), and
 * the per-(view, tile) entry count seg_count[v*T + t] (T = tiles per view).
 *   means [S,G,3]  shs [S,G,M,3] (M >= (sh_degree+1)^2) xor colors [S,G,3]
 *   opacities [S,G]  cov6 [S,G,6] (xx,xy,xz,yy,yz,zz = cuda_splatting.py:114,122)
 *   layout: DSR_LAYOUT_* bits for the shs / covariance arrays (0 = as above)
 *   out: geom [V,G,12], radii [V,G] int32, seg_count [V*T] (zeroed by this call).  */
#define DSR_LAYOUT_SH_CHANNEL_MAJOR 1  /* shs given as [S,G,3,M] (Gaussians.harmonics)      */
#define DSR_LAYOUT_COV_FULL 2          /* covariance given as [S,G,3,3]; grads: upper triangle */
#define DSR_LAYOUT_COUNTS_ZEROED 4     /* seg_count already zeroed (dsr_build_cameras)       */
#define DSR_LAYOUT_RECT_BINNING 8      /* dsr_project_bin_cameras only: keep the reference's 3-sigma
                                          tile rects instead of the exact alpha >= 1/255 test       */
#define DSR_LAYOUT_EXACT_BINNING 16    /* dsr_project_bin / dsr_preprocess_fwd / dsr_bin_scatter:
                                          exact alpha >= 1/255 tile test (as dsr_project_bin_cameras;
                                          the count and scatter calls of one forward must agree)    */
#define DSR_LAYOUT_VIEWS_PER_SCENE(k) ((k) << 16)  /* dsr_project_bin_cameras: views grouped by
                                          scene in order, k (< 256) per scene: whole scenes are placed
                                          on one XCD (0 = no grouping: blocks x views)              */
#define DSR_LAYOUT_DEFER_GEOM 32       /* dsr_preprocess_cut only: radii, counts, histogram and
                                          cut_rec, but no geometry record and no colour (see
                                          dsr_project_survivors); needs cut_rec, no dgeom_zero      */
int dsr_preprocess_fwd(int S, int G, int V, int H, int W, int sh_degree, int M,
                       const float* means, const float* shs, const float* colors,
                       const float* opacities, const float* cov6, const dsr_camera* cams,
                       float* geom, int32_t* radii, int64_t* dgeom_zero, uint32_t* seg_count,
                       int layout, void* stream);
/* dgeom_zero (every forward entry point that writes geom; optional, NULL = none): the
 * backward's fixed-point gradient accumulator [V, G, DSR_DGEOM_WORDS] int64. The row of every
 * rendered (view, gaussian) (radius > 0) is zeroed in the same pass that writes its geometry
 * record, so a forward with a backward coming needs no separate fill of the accumulator
 * (dsr_render_bwd / dsr_preprocess_bwd never touch the rows of culled gaussians). */

/* Fused alternative to dsr_preprocess_fwd + dsr_bin_scan + dsr_bin_scatter (K1 + K3) for
 * problems whose fixed-capacity key buffer fits: the same projection, plus the keys of every
 * (gaussian, touched tile) written straight into segment (v, t) = keys[(v*T + t) * G ...]
 * (a gaussian touches a tile at most once). One workgroup per (256 gaussians, view); the
 * workgroups of one gaussian block for all views of its scene are placed on one XCD, back
 * to back, so the scene inputs come from HBM once and from that XCD's L2 for the other
 * views. keys must hold V*T*G entries (only V*T segments' prefixes are written);
 * seg_count [V*T] receives the entry counts (zeroed by this call). Consumers take
 * seg_stride = G. Requires T <= 32768 and V*T*G < 2^32. */
int dsr_project_bin(int S, int G, int V, int H, int W, int sh_degree, int M,
                    const float* means, const float* shs, const float* colors,
                    const float* opacities, const float* cov6, const dsr_camera* cams,
                    float* geom, int32_t* radii, int64_t* dgeom_zero, uint32_t* seg_count, uint64_t* keys,
                    int layout, void* stream);

/* dsr_build_cameras + dsr_project_bin in one launch (the inference fast path): every
 * workgroup sets up its view's camera from the render_cuda inputs (as dsr_build_cameras, in
 * float) and the first block of each view stores it to cams [V] for the later calls.
 * seg_count must come zeroed (DSR_LAYOUT_COUNTS_ZEROED in layout; e.g. by dsr_sort_render's
 * clear_counts). Binning: a (gaussian, tile) pair is kept only when the gaussian's
 * alpha >= 1/255 ellipse reaches the tile (exact conic minimum over the tile box), so each
 * segment is an order-preserving subsequence of the reference's 3-sigma list holding every
 * entry that can blend at a pixel of the tile; images are identical, n_contrib counts
 * positions in the shorter list. DSR_LAYOUT_RECT_BINNING keeps the reference's lists. */
int dsr_project_bin_cameras(int S, int G, int V, int H, int W, int sh_degree, int M,
                            const float* means, const float* shs, const float* colors,
                            const float* opacities, const float* cov6, const float* extrinsics,
                            const float* intrinsics, const float* near, const float* far,
                            const float* bg, const int32_t* view_scene, int scale_invariant,
                            dsr_camera* cams, float* geom, int32_t* radii, int64_t* dgeom_zero,
                            uint32_t* seg_count, uint64_t* keys, uint32_t seg_capacity, int layout,
                            void* stream);
/* seg_capacity (bounded key memory; 0 = G): segment (v, t) = keys[(v*T + t) * seg_capacity ...],
 * keys / scratch hold V*T*seg_capacity entries. A tile that receives more entries keeps the
 * first seg_capacity of them while seg_count goes on counting; dsr_sort_render (seg_stride =
 * seg_capacity) recognises such a segment (count > stride) and rebuilds its list from the
 * geometry records (the binning test is a function of one record), so images are identical
 * for every capacity — a capacity above the largest tile list only saves the rebuild.
 * extrinsics == NULL (camera-block mode): cams [V] is an INPUT holding the caller's camera
 * blocks (dsr_build_cameras, or the reference wrapper's GaussianRasterizationSettings packed
 * as dsr_camera); the other camera inputs are ignored and the same projection / binning
 * kernel runs without its in-kernel camera set-up (exact binning unless
 * DSR_LAYOUT_RECT_BINNING). With the wrapper's own matrices the tile lists equal the
 * reference's bit for bit. */

/* Exclusive scan of seg_count[V*T] -> seg_start[V*T+1], seg_cursor[V*T] (= seg_start),
 * totals[0] = N (num_rendered over all views), totals[1] = max entries in one tile,
 * totals[2] = 1 if N reached 2^31 (offsets invalid: render fewer views per call). */
int dsr_bin_scan(int V, int H, int W, const uint32_t* seg_count, uint32_t* seg_start,
                 uint32_t* seg_cursor, uint32_t* totals, void* stream);

/* Emit one 64-bit key per (gaussian, touched tile): key = float_bits(depth) << 32 | id,
 * grouped by segment (v, t) at seg_start; order inside a segment is arbitrary here and
 * fixed by dsr_bin_sort. keys must hold N entries. Replaces duplicateWithKeys (K3). */
int dsr_bin_scatter(int G, int V, int H, int W, const float* geom, uint32_t* seg_cursor,
                    uint64_t* keys, int layout, void* stream);
/* layout: DSR_LAYOUT_EXACT_BINNING when the dsr_preprocess_fwd call that counted the entries
 * had it (other bits ignored). */

/* Segment layout used by the sort and compositing calls:
 *   seg_stride == 0: prefix layout, segment s = keys[seg_start[s] .. seg_start[s+1])
 *                    (dsr_bin_scan / dsr_bin_scatter; seg_count may be NULL)
 *   seg_stride  > 0: fixed capacity, segment s = keys[s*stride .. s*stride + seg_count[s])
 *                    (dsr_project_bin with stride = G; seg_start may be NULL)
 *   seg_stride == DSR_SEG_ENDS: segment s = keys[seg_start[s] .. seg_count[s]), seg_count
 *                    holding absolute END offsets (the cursors after dsr_bin_scatter_cut:
 *                    only the near part of each prefix-layout segment is written) */
#define DSR_SEG_ENDS 0xFFFFFFFFu

/* ---- depth-cut binning (large problems: 6-view 448x768 and up) -----------------------
 * At 6x448x768 a tile's list holds ~31K entries while the compositor consumes at most ~1.1K
 * (every pixel saturates): writing, sorting and reading the other 30K is the dominant cost.
 * These calls write only each tile's nearest entries, chosen with a depth histogram:
 *   1. dsr_preprocess_cut = dsr_preprocess_fwd + a per-(view, super-block) histogram of
 *      depth buckets (DSR_CUT_BUCKETS log-spaced buckets, 16 per octave of view depth from
 *      0.25 near-units, each Gaussian counted once per touched tile);
 *   2. dsr_bin_cutoff picks per (view, super-block) the depth at which the cumulative count
 *      reaches `prefix` entries per tile;
 *   3. dsr_bin_scatter_cut (tail = 0) emits only the entries at or before that depth into the
 *      prefix layout of dsr_bin_scan (full counts): seg_cursor ends at each segment's written
 *      end -> DSR_SEG_ENDS layout for dsr_bin_sort / dsr_render_fwd / dsr_render_bwd.
 * Every emitted entry is nearer than every omitted one (a depth threshold), so the
 * sorted written part IS the head of the full sorted list. dsr_render_fwd flags a tile whose
 * pixels are not all saturated at the end of its written part (seg_overflow[s] = 1 and
 * seg_overflow[V*T] = 1); dsr_bin_scatter_cut with tail = 1 then appends the omitted entries
 * of flagged tiles only (returns at once when seg_overflow[V*T] == 0), after which those
 * tiles are sorted in full and rendered again (seg_filter = seg_overflow). */
#define DSR_CUT_BUCKETS 128
/* Super-block edge in tiles for a W x H image (0: the image is too large for this path). */
int dsr_cut_superblock(int H, int W);
/* depth_hist [V, nsb, DSR_CUT_BUCKETS] uint32 (zeroed by this call), nsb = ceil(tiles_x/sb)
 * * ceil(tiles_y/sb); other arguments and outputs as dsr_preprocess_fwd.
 * cut_rec (optional, [V, G, 2] uint32): per (view, Gaussian) its tile rect (x0 | x1 << 8 |
 * y0 << 16 | y1 << 24, 0 when culled) and its depth bits: 8 bytes the scatter reads instead of
 * the 48-byte geometry record (requires at most 255 tiles per axis; NULL skips it). */
int dsr_preprocess_cut(int S, int G, int V, int H, int W, int sh_degree, int M,
                       const float* means, const float* shs, const float* colors,
                       const float* opacities, const float* cov6, const dsr_camera* cams,
                       float* geom, int32_t* radii, int64_t* dgeom_zero, uint32_t* seg_count,
                       uint32_t* depth_hist, uint32_t* cut_rec, int layout, void* stream);
/* cut [V, nsb] uint32: per super-block, the largest depth (float bits) emitted: inside the
 * bucket where the count reaches `prefix` per tile, interpolated by the fraction still
 * needed (0xffffffff = all). */
int dsr_bin_cutoff(int V, int H, int W, const uint32_t* depth_hist, uint32_t prefix, uint32_t* cut,
                   void* stream);
/* As dsr_bin_scatter, restricted by cut: tail = 0 -> entries with depth bits <= cut; tail = 1 ->
 * the deeper entries of the segments with seg_overflow[s] != 0. seg_overflow here has
 * V*T + 1 + V*nsb words: tile flags, the any-flag, then per-(view, super-block) flags, all
 * written by dsr_render_fwd in the DSR_SEG_ENDS layout. seg_cursor advances past what is
 * written. */
int dsr_bin_scatter_cut(int G, int V, int H, int W, const float* geom, uint32_t* seg_cursor,
                        uint64_t* keys, const uint32_t* cut, int tail, const uint32_t* seg_overflow,
                        const uint32_t* cut_rec, uint32_t* survivors, uint32_t* survivor_count,
                        const uint32_t* totals, uint64_t keys_capacity, void* stream);
/* totals (dsr_bin_scan's, or NULL) and keys_capacity (entries `keys` holds): with totals given,
 * the launch does nothing when totals[0] > keys_capacity (or totals[2] flags an offset overflow) —
 * so the pass can be queued before the
 * host has read N, into a buffer sized from an earlier call, and re-run if it was too small. */
/* cut_rec: dsr_preprocess_cut's compact records (or NULL: the pre-test reads geom).
 * survivors / survivor_count (sizes from dsr_survivor_layout; the counters zeroed by the
 * caller; both NULL: none): the Gaussians that may emit in this pass are listed, per view and
 * per scatter workgroup (for dsr_project_survivors after a DSR_LAYOUT_DEFER_GEOM preprocess;
 * requires cut_rec). */
/* Sizes of the survivor lists for (G, V): *slots uint32 entries, *counters uint32 counters. */
int dsr_survivor_layout(int G, int V, int64_t* slots, int* counters);

/* Deferred geometry: after dsr_preprocess_cut with DSR_LAYOUT_DEFER_GEOM and a scatter pass
 * that listed its survivors, project the listed Gaussians of every view in full (colour
 * included) and write their geometry records (bit-identical to dsr_preprocess_fwd's). At
 * 12x512x960 the scatter keeps ~3 % of the (view, Gaussian) pairs: the preprocess skips the SH
 * reads, the colour and the 48-byte record of the others. Arguments as dsr_preprocess_fwd. */
int dsr_project_survivors(int S, int G, int V, int H, int W, int sh_degree, int M,
                          const float* means, const float* shs, const float* colors,
                          const float* opacities, const float* cov6, const dsr_camera* cams,
                          const uint32_t* survivors, const uint32_t* survivor_count, float* geom,
                          int32_t* radii, int64_t* dgeom_zero, uint8_t* row_live, int layout,
                          void* stream);
/* dgeom_zero / row_live (training with deferred geometry; both NULL for inference): the
 * backward's accumulator rows of the projected (view, gaussian) pairs are zeroed here and
 * row_live[v*G + g] (uint8, zeroed by the caller) set to 1 for them: the only rows
 * dsr_render_bwd adds to and dsr_preprocess_bwd then reads (pass row_live to it). The
 * count pass (dsr_preprocess_cut with DSR_LAYOUT_DEFER_GEOM) touches none of them. */

/* Sort every segment by (depth, id) ascending — identical to upstream's stable radix
 * sort of (tile << 32 | depth) with emission-order ties (K4/K5). max_count sizes the LDS
 * sort (0 = unknown): segments that fit sort in LDS, larger ones sort through HBM using
 * `scratch` (same size as keys). scratch may be NULL only when max_count is an exact
 * bound <= dsr_sort_lds_capacity(). When max_count exceeds the LDS capacity, segments
 * above 4096 entries are split by depth into LDS-sized groups (one MSD pass through
 * scratch), which needs `workspace` of dsr_bin_sort_workspace_size(V, H, W, max_count)
 * bytes (NULL allowed when that is 0). (In the fixed-capacity layout N and the largest
 * segment are sum / max of seg_count: no same-address atomics from every workgroup.)
 * Offsets must stay below 2^31.
 *
 * Prefix mode (prefix > 0, needs seg_sorted [nseg]): in that split path, a segment longer
 * than `prefix` only has its nearest entries sorted — keys[0, P) hold the P >= prefix
 * smallest keys in order, keys[P, n) the rest, unordered — and seg_sorted[s] = P
 * (= n for fully sorted segments; always written when seg_sorted is given). The
 * compositor needs little more than a few hundred entries per tile, so the rest of a
 * 30-40K entry list is never put in order; dsr_render_fwd checks the tail and flags the
 * rare tile that does need it. seg_filter (non-NULL, needs scratch): sort in full only
 * the segments with seg_filter[s] != 0 (the flagged tiles), leaving the others as they are;
 * seg_filter[nseg] is the any-flag word (as dsr_render_fwd / dsr_sort_render write it: 0 =
 * nothing flagged, the launch does nothing).
 * The reference sorts every key (cuda_rasterizer/rasterizer_impl.cu, SortPairs). */
int dsr_bin_sort(int G, int V, int H, int W, const uint32_t* seg_start, const uint32_t* seg_count,
                 uint32_t seg_stride, uint64_t* keys, uint64_t* scratch, uint32_t max_count,
                 void* workspace, uint32_t prefix, uint32_t* seg_sorted, const uint32_t* seg_filter,
                 void* stream);
size_t dsr_bin_sort_workspace_size(int V, int H, int W, uint32_t max_count);
uint32_t dsr_sort_lds_capacity(void);

/* Front-to-back compositing per 16x16 tile (K6). out_color [V,3,H,W], final_T [V,H,W],
 * n_contrib [V,H,W] (uint32). Background from cams[v].bg.
 * seg_sorted (NULL = every segment fully sorted): entries past seg_sorted[s] are an
 * unordered tail (dsr_bin_sort prefix mode); they are only checked, and if one of them
 * passes the alpha test at a pixel that is still live, seg_overflow[s] is set to 1 (caller
 * zeroes it) and that tile's outputs are void: sort the flagged segments in full
 * (dsr_bin_sort with seg_filter = seg_overflow) and call again with seg_filter =
 * seg_overflow and seg_sorted = NULL, which renders only those tiles. In the DSR_SEG_ENDS
 * layout (depth-cut binning) with seg_overflow given, a segment whose written end is below
 * seg_start[s+1] is flagged when any of its pixels is still live at that end. seg_overflow
 * has V*T + 1 words, word V*T set to 1 whenever any tile is flagged; in the DSR_SEG_ENDS
 * layout V*T + 1 + V*nsb words, the last V*nsb flagging the super-blocks of flagged tiles
 * (dsr_preprocess_cut). */
int dsr_render_fwd(int G, int V, int H, int W, const dsr_camera* cams, const float* geom,
                   const uint32_t* seg_start, const uint32_t* seg_count, uint32_t seg_stride,
                   const uint64_t* keys, const uint32_t* seg_sorted, uint32_t* seg_overflow,
                   const uint32_t* seg_filter, float* out_color, float* final_T, uint32_t* n_contrib,
                   void* stream);

/* dsr_bin_sort + dsr_render_fwd in one launch (no prefix / cut modes): each workgroup sorts its
 * tile's keys in LDS and composites from that copy; segments above the LDS class (below) are
 * sorted through `scratch` (same size as keys) by the same workgroup. The sorted keys are
 * written back to `keys` only when write_keys != 0 (dsr_render_bwd needs them). Outputs as
 * dsr_render_fwd; n_contrib may be NULL (an inference call with no backward: the compositor
 * then does not track the last blended position).
 * max_count_hint: the caller's estimate of the largest segment (e.g. the max of an earlier
 * call's counts; 0 = unknown). It picks the LDS class — 2048, 3072 or 4096 keys per tile
 * (smaller classes keep 4 workgroups per CU resident instead of 3) — and affects speed only:
 * results are identical for any hint. */
int dsr_sort_render(int G, int V, int H, int W, const dsr_camera* cams, const float* geom,
                    const uint32_t* seg_start, uint32_t* seg_count, uint32_t seg_stride, uint64_t* keys,
                    uint64_t* scratch, uint64_t* spill_keys, int write_keys, int clear_counts,
                    uint32_t max_count_hint, int binning_layout, float* out_color, float* final_T,
                    uint32_t* n_contrib, uint32_t* seg_overflow, void* stream);
/* seg_overflow (NULL: none; DSR_SEG_ENDS layout only): the depth cut's flags, written exactly
 * as dsr_render_fwd writes them (tile, any-flag, super-block), so this launch can replace
 * dsr_bin_sort + dsr_render_fwd for the written heads when no backward needs sorted keys. */
/* clear_counts != 0 (fixed-capacity layout only): seg_count is zeroed as it is consumed, so
 * the buffer can serve the next dsr_project_bin_cameras call as already-zeroed counters.
 * Bounded capacity (dsr_project_bin_cameras seg_capacity < G, seg_stride = that capacity): a
 * segment with seg_count[s] > seg_stride is rebuilt by its workgroup from the view's geometry
 * records with the binning test of `binning_layout` (the layout bits of the binning call:
 * DSR_LAYOUT_RECT_BINNING = 3-sigma rects, else the exact test) and composited in depth
 * windows of the LDS capacity (slow, exact). With write_keys, the sorted keys of a segment
 * with seg_count[s] <= seg_stride go back to `keys`; those of a rebuilt segment go to
 * spill_keys [V*T, G] (its slots s*G + position, written up to the window in which every pixel
 * of the tile stopped — all that dsr_render_bwd reads). spill_keys (NULL: not stored) needs
 * write_keys and the fixed-capacity layout; pass the same pointer to dsr_render_bwd, which
 * reads a segment with seg_count[s] > seg_stride from there. (round 5: bounded segments for
 * forwards with a backward, no host check between forward and backward) */

/* ---- rasterizer backward -----------------------------------------------------------
 * Deterministic: every per-Gaussian gradient is a sum over (tile, sub-tile wave) partials,
 * accumulated as 64-bit FIXED-POINT integers (integer addition is associative, so the
 * result does not depend on the order the partials arrive in: bit-identical run to run).
 * The fixed-point unit follows the size of the incoming gradient so that a mean loss's tiny
 * dL/dpix keeps full precision: with m = max |dL_dpix| rounded up to 2^k, one unit is
 * 2^(k-32) (DSR_GRAD_FRAC_BITS), i.e. partials are stored as round(x * 2^(32-k)).
 *
 * dsr_grad_scale: per-block maxima of |dL_dpix [V,3,H,W]| into
 * grad_scale [DSR_GRAD_SCALE_BLOCKS] floats (both kernels below derive m from them). */
#define DSR_GRAD_SCALE_BLOCKS 512
#define DSR_GRAD_FRAC_BITS 32
#define DSR_DGEOM_WORDS 9    /* int64 words per (view, gaussian) gradient row          */
int dsr_grad_scale(int V, int H, int W, const float* dL_dpix, float* grad_scale, void* stream);

/* Back-to-front per tile (K7). dL_dpix [V,3,H,W]. Accumulates into dgeom_fx
 * [V,G,DSR_DGEOM_WORDS] int64 fixed point (rows of rendered gaussians zeroed beforehand: by
 * the forward's dgeom_zero or by the caller): [0..1] dL/dxy (ndc scale, as
 * upstream dL_dmean2D), [2..4] dL/dconic, [5] dL/dopacity, [6..8] dL/drgb. */
int dsr_render_bwd(int G, int V, int H, int W, const dsr_camera* cams, const float* geom,
                   const uint32_t* seg_start, const uint32_t* seg_count, uint32_t seg_stride,
                   const uint64_t* keys, const uint64_t* spill_keys, const float* final_T,
                   const uint32_t* n_contrib, const float* dL_dpix, const float* grad_scale, int64_t* dgeom_fx,
                   void* stream);

/* dgeom_fx -> float dgeom [V,G,DSR_GEOM_STRIDE] (words 9..11 zero, rows of culled Gaussians
 * zero, and rows not marked in row_live when it is given): the values the preprocess backward
 * consumes, for callers that want them (tests, diagnostics). */
int dsr_dgeom_to_float(int G, int V, const float* geom, const int64_t* dgeom_fx, const float* grad_scale,
                       const uint8_t* row_live, float* dgeom, void* stream);

/* Preprocess backward (K8 + K9), reduced over all views of each scene without atomics.
 * dgeom_fx / grad_scale: as written by dsr_render_bwd / dsr_grad_scale.
 * scene_view_start [S+1], scene_views [V] list the views of each scene.
 * row_live [V,G] uint8 or NULL: after a deferred-geometry forward (dsr_project_survivors with
 * row_live), only the rows marked 1 are read (the others have no record and no zeroed
 * accumulator); NULL: every row with radius > 0.
 * out (overwritten): dmeans [S,G,3], dshs [S,G,M,3] or NULL, dcolors [S,G,3] or NULL,
 * dopac [S,G], dcov6 [S,G,6]; dmean2D [V,G,3] optional (NULL to skip). `layout` as in
 * the forward; dshs / dcov6 are written in that layout (full covariance: upper triangle,
 * zeros below, as the reference's triu-gather backward produces). */
int dsr_preprocess_bwd(int S, int G, int V, int H, int W, int sh_degree, int M,
                       const float* means, const float* shs, const float* cov6,
                       const dsr_camera* cams, const float* geom, const int64_t* dgeom_fx,
                       const float* grad_scale, const int32_t* scene_view_start, const int32_t* scene_views,
                       const uint8_t* row_live, float* dmeans, float* dshs, float* dcolors, float* dopac,
                       float* dcov6, float* dmean2D, int layout, void* stream);

/* Fused head backward (round 6): dsr_preprocess_bwd + dga_adapter_bwd in one pass for
 * Gaussians made by dga_adapter_fwd from head rows (the training step). Arguments: those of
 * dga_adapter_bwd for the head side (head [B,V,H*W,C], depths [B,V,H*W], images [B,V,3,H,W]
 * (the adapter's forward is re-evaluated), adapter_cams [B*V,104], scale range, sh_mask [d_sh]) and those of dsr_preprocess_bwd for the raster side
 * (target size Ht x Wt, cams, geom, dgeom_fx, grad_scale, scene_view_start / scene_views,
 * row_live; the Gaussians of scene b are rows [b G, (b + 1) G), G = V H W, and the SH degree is
 * sqrt(d_sh) - 1). Writes dhead [B,V,H*W,C] (channels past 10 + 3 d_sh: 0) and, when
 * non-NULL, ddepths [B,V,H*W]: bit-identical to dsr_preprocess_bwd followed by
 * dga_adapter_bwd, without the Gaussian gradients' round trip through HBM. Needs H*W % 256 == 0. */
int dsr_head_bwd(int B, int V, int H, int W, int d_sh, int C, const float* head, const float* depths,
                 const float* images, const float* adapter_cams, float scale_min, float scale_max, const float* sh_mask, int Ht, int Wt,
                 const dsr_camera* cams, const float* geom, const int64_t* dgeom_fx, const float* grad_scale,
                 const int32_t* scene_view_start, const int32_t* scene_views, const uint8_t* row_live, float* dhead,
                 float* ddepths, void* stream);

/* ---- plane-sweep cost volume -------------------------------------------------------
 * Fused warp_with_pose_depth_candidates (matching.py:24-90) + correlation
 * (mv_unimatch.py:494-505):
 *   cost[b,d,y,x] = mean_j ( sum_c ref[b,c,y,x] * warp_j[b,c,d,y,x] ) / sqrt(C)
 * where warp_j bilinearly samples tgt[b,j] (zeros padding, align_corners=True) at the
 * projection of pixel (x,y) at depth[b,d,y,x] through K[b,j] and pose[b,j].
 *   ref [B,C,H,W]  tgt [B,J,C,H,W]  intr [B,J,3,3] (pixel units)  pose [B,J,4,4]
 *   depth [B,D,H,W] when depth_per_pixel else [B,D]   ->   cost [B,D,H,W]
 * C in {16, 32, 64, 128} (matrix cores): small grids (B*H*W <= 32768, e.g. 2x64^2) run one
 * band kernel: 16 reference pixels of a row x 64 depths per workgroup, correlated with the
 * bounding box of their taps as one exact-f32 GEMM (v_mfma_f32_16x16x4_f32) straight from the
 * [B,C,H,W] maps. Larger grids group the reference pixels by the epipolar line they lie on
 * w.r.t. each source view (16 pixels of one line tap a thin band around ONE target line);
 * each group's correlations with its band's distinct target pixels are one GEMM, finished by
 * the 4-tap bilinear gather; the band's bitmap and list cover only the bounding box of the
 * group's taps. Views are summed in launch order (deterministic). Other C: a direct
 * channel-last kernel.
 * path: dcv_cost_volume_path(...) for this shape (0 band, 1 epipolar groups, 2 direct; env
 * DSPLAT_CV_PATH=band / epi overrides it there, for timing tools only). The caller passes the
 * SAME value to the forward and to the backward (which must know what the forward left in the
 * workspace); a path the shape cannot take is an error.
 * workspace: dcv_cost_volume_workspace_size bytes (channel-last copies of tgt and ref with a
 * zero padding row per image, and the epipolar groups), filled here (or, after a band-kernel
 * forward, by dcv_cost_volume_bwd itself) and read by dcv_cost_volume_bwd. */
#define DCV_PATH_BAND 0
#define DCV_PATH_EPI 1
#define DCV_PATH_DIRECT 2
int dcv_cost_volume_path(int B, int J, int C, int H, int W);
size_t dcv_cost_volume_workspace_size(int B, int J, int C, int H, int W);
int dcv_cost_volume_fwd(int B, int J, int C, int H, int W, int D, int depth_per_pixel, int path,
                        const float* ref, const float* tgt, const float* intr, const float* pose,
                        const float* depth, float clamp_min_depth, void* workspace, float* cost,
                        void* stream);

/* Backward of dcv_cost_volume_fwd w.r.t. both feature maps (geometry gets no grad,
 * matching.py:46). dcost [B,D,H,W] -> dref [B,C,H,W] (overwritten), dtgt [B,J,C,H,W]
 * (overwritten). fwd_path: the forward's path argument; ref / tgt: the forward's inputs;
 * workspace: the forward's (completed here when the forward ran the band kernel);
 * dcv_cost_volume_bwd_workspace_size bytes of scratch (channel-last gradient accumulators).
 * On the matrix-core paths both gradients are bit-identical run to run at every image size
 * (the epipolar grouping is a function of the inputs, never of atomic arrival): reference
 * gradients are summed in a fixed order, the shared sums in integer fixed point — the gradient
 * weights in LDS with a unit per reference pixel and depth chunk (from that pixel's largest
 * |dcost|), the target gradients in HBM with the finest unit the int64 range allows for the
 * shape (from the largest |dcost| and |ref| and the number of partial sums per element). A
 * non-finite dcost or ref makes dtgt NaN. The direct kernel (C not a multiple of 16) adds target
 * gradients with float atomics. */
size_t dcv_cost_volume_bwd_workspace_size(int B, int J, int C, int H, int W);
/* The matrix-core backward's workgroup shape for these sizes (what dcv_cost_volume_bwd
 * launches when C is a multiple of 16): 2^pxb reference pixels per workgroup (4: 16, 5: 32,
 * 6: 64 — consecutive epipolar groups sharing one union band) and spt samples per thread
 * (depth chunk (256 >> pxb) * spt). Returns 1 (no matrix-core backward) otherwise. */
int dcv_cost_volume_bwd_shape(int B, int C, int H, int W, int D, int depth_per_pixel, int* pxb, int* spt);
int dcv_cost_volume_bwd(int B, int J, int C, int H, int W, int D, int depth_per_pixel, int fwd_path,
                        const float* ref, const float* tgt, void* workspace, const float* intr,
                        const float* pose, const float* depth, float clamp_min_depth,
                        const float* dcost, float* dref, float* dtgt, void* bwd_workspace,
                        void* stream);

/* Views mode: the same cost volume from per-view features and a neighbour index instead of
 * the stacked tgt the reference builds with batch_features_camera_parameters
 * (mv_transformer.py:653-747, a gather copying every feature map J more times):
 *   features [BV,C,H,W]; nn [BV,J] int32 view indices in [0, BV) (tgt[b, j] = features[nn[b J
 *   + j]]; out-of-range indices are clamped); intr / pose / depth as dcv_cost_volume_fwd.
 * ONE channel-last copy of the features serves every role. Matrix-core shapes only (C a
 * multiple of 16, dcv_cost_volume_path(...) == DCV_PATH_EPI sizes); else status 1.
 * The backward writes dfeatures [BV,C,H,W] = the gradient through both roles (reference and
 * target), bit-identical run to run; max_fanin: an upper bound on how many (b, j) pairs name one
 * view (<= 0: BV J), which sets the int64 fixed-point unit of the target sums. */
size_t dcv_cost_volume_views_workspace_size(int BV, int J, int C, int H, int W);
size_t dcv_cost_volume_views_bwd_workspace_size(int BV, int J, int C, int H, int W);
int dcv_cost_volume_views_fwd(int BV, int J, int C, int H, int W, int D, int depth_per_pixel,
                              const float* features, const int32_t* nn, const float* intr,
                              const float* pose, const float* depth, float clamp_min_depth,
                              void* workspace, float* cost, void* stream);
int dcv_cost_volume_views_bwd(int BV, int J, int C, int H, int W, int D, int depth_per_pixel,
                              int max_fanin, const float* features, const int32_t* nn,
                              void* workspace, const float* intr, const float* pose,
                              const float* depth, float clamp_min_depth, const float* dcost,
                              float* dfeatures, void* bwd_workspace, void* stream);

/* Materialising warp with the exact matching.py:24-90 signature semantics:
 * feature [B,C,H,W], intr [B,3,3], pose [B,4,4], depth [B,D,H,W] -> out [B,C,D,H,W]. */
int dcv_warp_fwd(int B, int C, int H, int W, int D, const float* feature, const float* intr,
                 const float* pose, const float* depth, float clamp_min_depth, float* out,
                 void* stream);

/* Gradient of dcv_warp_fwd w.r.t. `feature`: dout [B,C,D,H,W] -> dfeature [B,C,H,W]
 * (overwritten). Geometry receives no gradient (matching.py:46, torch.no_grad). */
int dcv_warp_bwd(int B, int C, int H, int W, int D, const float* dout, const float* intr,
                 const float* pose, const float* depth, float clamp_min_depth, float* dfeature,
                 void* stream);

/* ---- Gaussian adapter ----------------------------------------------------------------
 * Fused encoder glue + GaussianAdapter + rotate_sh (encoder_depthsplat.py:224-346,
 * gaussian_adapter.py:49-102, gaussians.py:8-44, sh_rotation.py:10-30), one thread per
 * (scene, context view, pixel). head [B,V,H*W,C] (C >= 10 + 3*d_sh: opacity logit, 2 offset
 * logits, 3 scales, 4 quaternion xyzw, 3*d_sh SH channel-major), depths [B,V,H*W],
 * images [B,V,3,H,W], cams [B*V,104] per-view blocks (R c2w [9], t [3], K^-1 [9],
 * Wigner-D of R for degrees 1..3 [9, 25, 49]), sh_mask [d_sh].
 * out: means [B,G,3], covariances [B,G,3,3], harmonics [B,G,3,d_sh], opacities [B,G],
 * G = V*H*W view-major (the decoder's Gaussians). d_sh in {1, 4, 9, 16}. */
/* Per-view blocks for dga_adapter_fwd/bwd from c2w extrinsics [BV,4,4] and normalised
 * intrinsics [BV,3,3]: R, t, K^-1 and the Wigner-D blocks of R up to sh_degree (zeros
 * above). `probes`: for l = 1..3, the probe directions [4(2l+1)+8, 3] then pinv of their
 * real SH [2l+1, 4(2l+1)+8], float64, concatenated (sh_rotation.py builds them). */
int dga_adapter_cameras(int BV, const float* extrinsics, const float* intrinsics, int sh_degree,
                        const double* probes, float* cams, void* stream);

int dga_adapter_fwd(int B, int V, int H, int W, int d_sh, int C, const float* head,
                    const float* depths, const float* images, const float* cams, float scale_min,
                    float scale_max, const float* sh_mask, float* means, float* covariances,
                    float* harmonics, float* opacities, void* stream);

/* Backward of dga_adapter_fwd: any of the output gradients may be NULL (zero). dhead
 * [B,V,H*W,C] overwritten (channels past 10 + 3*d_sh get 0); ddepths [B,V,H*W] overwritten
 * when non-NULL. Images and cameras get no gradient. */
int dga_adapter_bwd(int B, int V, int H, int W, int d_sh, int C, const float* head,
                    const float* depths, const float* cams, float scale_min, float scale_max,
                    const float* sh_mask, const float* dmeans, const float* dcovariances,
                    const float* dharmonics, const float* dopacities, float* dhead, float* ddepths,
                    void* stream);

/* The reference operator itself: GaussianAdapter.forward(extrinsics, intrinsics, coordinates,
 * depths, opacities, raw_gaussians, image_shape, eps, point_cloud, input_images)
 * (gaussian_adapter.py:49-102; called at encoder_depthsplat.py:300-314). Rows n = ((bv * H*W
 * + pixel) * S + s) for BV = b*v views and S Gaussians per pixel (surfaces x spp):
 *   raw [N, C] (C >= 7 + 3*d_sh: scales 3, rotation 4, sh 3*d_sh channel-major),
 *   coordinates [N, 2] normalised image xy, depths [N], images [BV,3,H,W],
 *   cams [BV,104] (dga_adapter_cameras), eps: the quaternion normaliser's epsilon.
 * out: means [N,3], covariances [N,3,3], harmonics [N,3,d_sh], and, when non-NULL, the
 * activated scales [N,3] and normalised rotations [N,4] (AdapterGaussians.scales /
 * .rotations). Opacities pass through unchanged (no kernel work). */
int dga_adapter_forward(int BV, int H, int W, int S, int d_sh, int C, const float* raw,
                        const float* coordinates, const float* depths, const float* images,
                        const float* cams, float scale_min, float scale_max, const float* sh_mask,
                        float eps, float* means, float* covariances, float* harmonics, float* scales,
                        float* rotations, void* stream);
/* Backward of dga_adapter_forward: output gradients may be NULL (zero). draw [N, C]
 * overwritten (unused channels 0); dcoordinates [N, 2] and ddepths [N] when non-NULL.
 * Cameras and images get no gradient. */
int dga_adapter_backward(int BV, int H, int W, int S, int d_sh, int C, const float* raw,
                         const float* coordinates, const float* depths, const float* cams,
                         float scale_min, float scale_max, const float* sh_mask, float eps,
                         const float* dmeans, const float* dcovariances, const float* dharmonics,
                         const float* dscales, const float* drotations, float* draw,
                         float* dcoordinates, float* ddepths, void* stream);

/* Head glue: the conv head's output x [BV, C*r*r, h, w] (C channels per pixel at r x r
 * sub-pixels, pixel-shuffled) to per-pixel rows [BV, (h*r)*(w*r), C] — the layout
 * dga_adapter_fwd reads — in one LDS-tiled pass:
 *   rows[bv][(hh*r + i)*(w*r) + ww*r + j][c] = x[bv][c*r*r + i*r + j][hh][ww]
 * (torch: x.view(BV, C, r, r, h, w).permute(0, 4, 2, 5, 3, 1); with r = 1 the einops
 * rearrange of the head output, encoder_depthsplat.py:224-233). dga_head_rows_bwd writes the
 * inverse (dx from drows). Requires 16 * r * (C + 1) * 4 <= 64 KiB (32-column tiles when
 * 32 * r * (C + 1) * 4 fits). */
int dga_head_rows(int BV, int C, int r, int h, int w, const float* x, float* rows, void* stream);
int dga_head_rows_bwd(int BV, int C, int r, int h, int w, const float* drows, float* dx, void* stream);

/* ---- loss / metric (the step after the rasterizer) ------------------------------------
 * One pass over n_images images of n_per_image floats: loss[0] = w_l1 mean|p - t| +
 * w_mse mean (p - t)^2 (loss_mse.py:33-44), grad (optional) = dloss/dp, psnr (optional)
 * [n_images] = -10 log10 mean (clip01(p) - clip01(t))^2 (metrics.py:12-19). Deterministic
 * (fixed-order fold of per-block partials in `workspace`, dls_loss_workspace_size bytes). */
size_t dls_loss_workspace_size(int n_images, int64_t n_per_image);
int dls_l1_mse_psnr(int n_images, int64_t n_per_image, const float* pred, const float* target,
                    float w_l1, float w_mse, float* loss, float* grad, float* psnr, void* workspace,
                    void* stream);

/* ---- buffer sizing -------------------------------------------------------------------
 * Bytes of every caller-owned buffer of one rasterizer call sequence over V views of
 * W x H pixels and G gaussians per scene (T = ceil(W/16) * ceil(H/16) tiles per view), so a
 * host that is not the Python layer can allocate them (the library never allocates).
 * key_budget: largest key buffer the caller accepts for the sync-free fixed-capacity layout
 * (the Python layer: min(48 GiB, 40 % of the device, free memory minus a reserve)). fixed_capacity = 1: dsr_project_bin(_cameras) applies and
 * keys / scratch are sized V*T*G; 0: the two-phase layout (dsr_preprocess_fwd / _cut, scan,
 * scatter), whose keys / scratch hold N = totals[0] of dsr_bin_scan entries (known only
 * after the scan: keys_bytes is then 0 here). Forward outputs: color [V,3,H,W], final_T
 * [V,H,W], n_contrib [V,H,W]; backward: dgeom_fx [V,G,DSR_DGEOM_WORDS] int64. */
typedef struct dsr_workspace {
    uint64_t cams_bytes;        /* dsr_camera [V]                                   */
    uint64_t geom_bytes;        /* [V,G,12] f32                                     */
    uint64_t radii_bytes;       /* [V,G] i32                                        */
    uint64_t seg_count_bytes;   /* [V*T] u32                                        */
    uint64_t seg_start_bytes;   /* [V*T+1] u32 (two-phase layout)                   */
    uint64_t keys_bytes;        /* u64 keys (fixed capacity: V*T*G)                 */
    uint64_t scratch_bytes;     /* same size as keys: segments above the LDS sort   */
    uint64_t sort_ws_bytes;     /* dsr_bin_sort_workspace_size at the worst case    */
    uint64_t color_bytes, final_T_bytes, n_contrib_bytes, dgeom_bytes;
    uint64_t total_bytes;       /* sum of the above                                 */
    int32_t tiles;              /* T                                                */
    int32_t fixed_capacity;     /* 1: fixed-capacity layout under key_budget        */
} dsr_workspace;
int dsr_workspace_size(int G, int H, int W, int n_views, uint64_t key_budget, dsr_workspace* out);

/* ---- misc ------------------------------------------------------------------------- */
const char* dsplat_last_error(void);
int dsplat_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* DSPLAT_HIP_H */
