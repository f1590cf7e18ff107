/*
 * gr_hip.h — C ABI of the MI355X (gfx950) differentiable Gaussian rasterizer.
 *
 * This is the drop-in boundary for the render op of Kirkice/3DGaussian:
 *
 *   reference surface (file:line)                          replaced by
 *   ------------------------------------------------------ ------------------------------------
 *   python/torch_renderer.py:109-203 render_gaussians_torch gr_fwd_prepare + gr_fwd_render (fwd)
 *     (autograd backward at fit_multiview_stub.py:310)      gr_bwd                         (bwd)
 *   include/gr/renderer.h:33-39 gr::render_gaussians        gr_render_u8
 *   include/gr/renderer.h:10-30 render_gaussians_{cpu,cuda} gr_render_u8 (HIP only)
 *   src/renderer_dispatch.cpp:5-21 (force_cpu / CUDA)       gr_render_u8 (HIP-only dispatch)
 *   src/bindings.cpp:27-100 (pybind11 module)               3dgaussian_amd/gaussian_renderer.py
 *   include/gr/cuda_utils.cuh:10-18 GR_CUDA_CHECK throw     gr_status codes + gr_last_error()
 *   include/gr/gaussian_types.h:24-46 RenderParams          gr_render_params (same field order)
 *
 * Conventions
 *   - Plain C: no C++ or torch types in any signature.  All matrices are 4x4 row-major float32,
 *     exactly as RenderParams::view/proj (gaussian_types.h:28-30).
 *   - The differentiable entry points (gr_fwd_*, gr_bwd) take DEVICE pointers owned by the caller
 *     and a hipStream_t passed as void*.  They allocate nothing and keep no render state between
 *     calls, so they are reentrant and stream-ordered (unlike renderer.cu:349's function-static
 *     buffers).  The only process-global state is the optional diagnostic profiler
 *     (gr_profile_begin/end, off by default: one atomic load per launch when off).
 *     Workspace sizes come from the *_bytes() queries.
 *   - gr_fwd_prepare is the one call that synchronises its stream: it returns the number of
 *     (Gaussian, tile) pairs, which sizes the binning workspace.  gr_fwd_prepare_async enqueues
 *     the same work plus a copy of the plan into caller memory (pinned, for a truly asynchronous
 *     copy) and returns at once, so the preparation of the next views overlaps the current one.
 *   - gr_render_u8 takes HOST pointers (as gr::render_gaussians does) and is synchronous.
 *   - Every function returns GR_OK or an error code; gr_last_error() gives a thread-local message.
 */
#ifndef GR_HIP_H_
#define GR_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GR_TILE 16 /* screen tile edge in pixels (16x16 = 256 pixels per tile) */

typedef enum gr_status {
  GR_OK = 0,
  GR_ERR_INVALID_ARGUMENT = 1, /* shapes / sizes / null pointers (python: ValueError/RuntimeError) */
  GR_ERR_HIP = 2,              /* a HIP runtime call failed (reference: GR_CUDA_CHECK throw)      */
  GR_ERR_WORKSPACE = 3,        /* caller-provided workspace too small                              */
  GR_ERR_OVERFLOW = 4          /* pair count does not fit int32                                    */
} gr_status;

/* Mirrors gr::RenderParams (include/gr/gaussian_types.h:24-46), same field order and defaults
 * (width 800, height 600, zero matrices, black background, enable_depth_sort 0, depth_slices 16,
 * force_cpu 0).  Used by the legacy uint8 surface. */
typedef struct gr_render_params {
  int width;
  int height;
  float view[16];
  float proj[16];
  float background[3];
  int enable_depth_sort; /* 0: OIT weighted average, 1: exact depth-sorted "over" compositing */
  int depth_slices;      /* accepted for ABI compatibility; the HIP path sorts exactly       */
  int force_cpu;         /* 1: the CPU renderer's contract (renderer_dispatch.cpp:12-13); the HIP */
                         /* path already has its semantics, except n <= 0: background, A = 255  */
                         /* (renderer_cpu.cpp:219-240) instead of renderer.cu's all-zero RGBA   */
} gr_render_params;

/* One camera view for the differentiable path (torch_renderer.py:109-121 arguments). */
typedef struct gr_view {
  int width;
  int height;
  float view[16];      /* Camera.view, row-major                                          */
  float proj[16];      /* Camera.proj, row-major                                          */
  float background[3]; /* background colour (torch_renderer.py:128-130)                    */
  float cam_pos[3];    /* inv(view)[:3,3] (torch_renderer.py:81-83); used by SH colours    */
  float cutoff;        /* footprint: tiles where max weight >= o*exp(-cutoff^2/2) (def. 7) */
  float core_cutoff;   /* two-zone footprint: kept tiles whose max weight is  */
                       /* below o*exp(-core_cutoff^2/2) are "tail" tiles that carry only W and */
                       /* D forward and the depth-coupled terms backward; <= 0 or >= cutoff  */
                       /* means one zone (def. 5.5)                                            */
  int no_depth_grad;   /* 0 (default): W and D are accumulated f32-grade, as an upstream depth   */
                       /* gradient needs (d depth/d w cancels on thin pixels); a backward that  */
                       /* gets no depth gradient runs the two-piece splat (nothing cancels).  1: the caller   */
                       /* will not pass a depth gradient to gr_bwd for this view; W and D are   */
                       /* then accumulated within 2^-16 relative (as the colours), and gr_bwd   */
                       /* rejects a non-NULL g_depth (GR_ERR_INVALID_ARGUMENT).  2: no depth    */
                       /* gradient (as 1) but every splat at the default mode's f32 grade       */
                       /* (three-piece splits): the fit path's precision reference              */
  const float* background_dev; /* optional DEVICE pointer to 3 floats: when non-NULL the kernels read */
                       /* the background colour from it (stream-ordered) instead of background[]: */
                       /* a caller holding the background in a device tensor (the reference fit   */
                       /* loop, fit_multiview_stub.py:287) needs no device-to-host read per view  */
  int binned;          /* 1: gr_fwd_bin has already built this view's bins (same plan, geom, bins   */
                       /* and scratch, ordered before the render); gr_fwd_render(_l1) then launches */
                       /* only the splat.  0 (default): the render bins the view itself            */
  int tile;            /* screen tile edge: 0 or 16 (default, GR_TILE) or 32.  32-pixel tiles halve the   */
                       /* (Gaussian, tile) pairs of a ~3-pixel-sigma scene and with them the binning and  */
                       /* the per-pair gradient rows; supported on the fused fit path only (preparation,  */
                       /* gr_fwd_bin, gr_fwd_render_l1 with no_depth_grad = 1, gr_bwd_splat,               */
                       /* gr_gather_view, gr_reduce_sums); the other entry points reject it.              */
  int device_counts;   /* 1: the view was prepared by gr_fwd_prepare_views_sized, and every gr_plan passed  */
                       /* with it holds CAPACITIES (buffer sizes and grids), not the view's counts: the     */
                       /* kernels read the true pair counts from the device (the preparation's device plan), */
                       /* so no host read of the counts sits between the preparation and the render (the   */
                       /* fit step can be captured as one HIP graph).  0 (default): plans are the counts.   */
  int chunk;           /* work-item length in pairs (a multiple of 64, <= 8192).  0 (default): the largest  */
                       /* power of two <= num_pairs / 1024 within [512, 2048] (at least ~4 items per CU).    */
                       /* Each item is one workgroup of the splats; the split tiles' partial sums are added */
                       /* in item order, so the value changes float rounding, deterministically.            */
  int row0;            /* rows > 0: only the band of tile rows [row0, row0 + rows) is rendered: Gaussians are  */
  int rows;            /* binned to its tiles only and the fit loss and its gradient cover its pixels only    */
                       /* (normalised by the whole image's pixel count), so the bands of a view add up to    */
                       /* the view.  The fused fit path only (gr_fwd_render_l1, gr_bwd_splat, gather, reduce, */
                       /* gr_fit_views_batched without depth): a multi-GPU fit splits views across ranks.     */
} gr_view;

/* ------------------------------------------------------------------------------------------ */
/* Differentiable path (device pointers).                                                     */
/*   means (N,3), scales (N,3), colors (N,3) [color_dim 3] or SH deg-1 (N,4,3) [color_dim 12]   */
/*   (extension: degree-3 coefficients (N,16,3) [color_dim 48], basis in DESIGN.md §2),           */
/*   opacities (N,), all float32 contiguous.                                                   */
/*   Views rendered with no_depth_grad and no depth output (the fit path) take f16 operand      */
/*   pieces scaled by 2^4; a view whose largest opacity reaches 2^11 gets a smaller power-of-two */
/*   scale (computed on the device by the preparation), so any opacity gives finite results.     */
/* ------------------------------------------------------------------------------------------ */

/* Sizes produced by gr_fwd_prepare for one view. */
typedef struct gr_plan {
  int64_t num_pairs;      /* kept (Gaussian, tile) pairs: the splat work                     */
  int64_t num_slots;      /* backward partial-sum slots: one per tile of each Gaussian's rectangle */
  int64_t num_core_pairs; /* of num_pairs, the core pairs (two-zone footprint, gr_view)       */
} gr_plan;

/* Per-Gaussian projection records, tile rectangles, pair counts and offsets. */
size_t gr_geom_bytes(int n);

/* Project + cull + count tiles + prefix-scan.  Fills *plan (synchronises `stream`). */
gr_status gr_fwd_prepare(const gr_view* v, int n, const float* means, const float* scales,
                         const float* colors, int color_dim, const float* opacities, void* geom,
                         size_t geom_bytes, gr_plan* plan, void* stream);

/* Same work, stream-ordered: *plan is written on `stream` (by the device itself when it is pinned
 * host memory, else by a device-to-host copy) and is valid once the stream (or an event recorded
 * after this call) has completed.  A pair count that
 * does not fit int32 reads back as num_pairs = -1, which gr_fwd_render reports as
 * GR_ERR_OVERFLOW.  *plan should be pinned host memory (hipHostMalloc / torch pin_memory);
 * pageable memory works but makes the copy synchronous. */
gr_status gr_fwd_prepare_async(const gr_view* v, int n, const float* means, const float* scales,
                               const float* colors, int color_dim, const float* opacities,
                               void* geom, size_t geom_bytes, gr_plan* plan, void* stream);

/* gr_fwd_prepare_async for up to GR_PREPARE_MAX_VIEWS views of the same Gaussians in one pass: the
 * parameters are read once per Gaussian, each view's geom (geom_bytes each) and plan are exactly what
 * gr_fwd_prepare_async writes for that view.  All plans are valid once the stream has completed. */
#define GR_PREPARE_MAX_VIEWS 8
gr_status gr_fwd_prepare_views_async(int num_views, const gr_view* views, int n, const float* means,
                                     const float* scales, const float* colors, int color_dim,
                                     const float* opacities, void* const* geoms, size_t geom_bytes,
                                     gr_plan* const* plans, void* stream);

/* Device-side sizing: gr_fwd_prepare_views_async against per-view CAPACITIES caps[k] (num_pairs: all pairs,
 * num_core_pairs: core pairs; the tail capacity is their difference), for views with device_counts = 1.  The true
 * counts go to the device plan (read by the binning and the splats) and, when observed[k] is non-NULL (pinned host
 * memory), to observed[k] (the caller's next capacities).  A view whose core or tail pairs exceed its capacity is
 * rendered as a view without pairs (background, zero gradients: no kernel reads or writes past a capacity) and sets
 * *overflow (device int) to 1: a caller redoes such a step with larger capacities (gr_fit_param_steps_sched skips
 * its update).  The downstream calls (gr_fwd_bin, gr_fwd_render(_l1), gr_bwd*, gr_gather_view, ...) take caps[k]
 * as their plan.  Needs the counting-sort binning (at most 8,192 screen tiles). */
gr_status gr_fwd_prepare_views_sized(int num_views, const gr_view* views, int n, const float* means,
                                     const float* scales, const float* colors, int color_dim,
                                     const float* opacities, void* const* geoms, size_t geom_bytes,
                                     const gr_plan* caps, gr_plan* const* observed, int* overflow, void* stream);

/* Tile-sorted (tile, Gaussian) pair lists, per-tile ranges and work items. */
size_t gr_bins_bytes(const gr_view* v, int n, const gr_plan* plan);

/* Forward-only scratch (unsorted pairs, sort temporaries, split-tile partials); may be released
 * as soon as gr_fwd_render has been enqueued (stream order keeps it alive for the kernels). */
size_t gr_fwd_scratch_bytes(const gr_view* v, int n, const gr_plan* plan);

/* Per-pixel state saved for the backward pass: 5 floats per pixel. */
size_t gr_saved_floats(const gr_view* v);

/* Emit pairs + sort by tile + tile ranges + forward splat.  Outputs:
 *   out_rgb (H,W,3) clamp((bg+C)/(1+W),0,1) (may be NULL: a caller that only needs the backward, as
 *   the fit loop); out_alpha (H,W) (may be NULL); out_depth (H,W) (may be NULL); saved (5*H*W floats)
 *   accumulators kept for gr_bwd (required).  A view with no_depth_grad
 *   and out_depth NULL skips the depth channel altogether (its saved depth sums are 0). */
gr_status gr_fwd_render(const gr_view* v, int n, const gr_plan* plan, const void* geom, void* bins,
                        size_t bins_bytes, void* scratch, size_t scratch_bytes, float* out_rgb,
                        float* out_alpha, float* out_depth, float* saved, void* stream);

/* gr_fwd_render without output images but with every saved sum (the depth channel's too): the splat of a view
 * whose background is not known yet (the drop-in op renders the next camera ahead of its call); gr_fwd_compose then
 * writes the outputs from `saved` with the view's background (gr_view.background / background_dev), exactly as
 * gr_fwd_render would have written them. */
gr_status gr_fwd_render_saved(const gr_view* v, int n, const gr_plan* plan, const void* geom, void* bins,
                              size_t bins_bytes, void* scratch, size_t scratch_bytes, float* saved, void* stream);
gr_status gr_fwd_compose(const gr_view* v, const float* saved, float* out_rgb, float* out_alpha, float* out_depth,
                         void* stream);

/* The binning half of gr_fwd_render (pair emission, tile sort, work items) on its own, so a caller can
 * run it on another stream (e.g. a high-priority one) and then render with gr_view.binned = 1 on the
 * same plan, geom, bins and scratch. */
gr_status gr_fwd_bin(const gr_view* v, int n, const gr_plan* plan, const void* geom, void* bins, size_t bins_bytes,
                     void* scratch, size_t scratch_bytes, void* stream);

/* Backward workspace: per-pair gradient partials + per-pixel upstream vectors. */
size_t gr_bwd_bytes(const gr_view* v, int n, const gr_plan* plan);

/* Backward of gr_fwd_render.  g_rgb (H,W,3) required; g_alpha, g_depth may be NULL (zero).
 * Writes (overwrites) d_means (N,3), d_scales (N,3) (column 2 is always 0),
 * d_colors (N,3), (N,4,3) or (N,16,3), d_opacities (N,). */
gr_status gr_bwd(const gr_view* v, int n, const gr_plan* plan, const float* means,
                 const float* scales, const float* colors, int color_dim, const float* opacities,
                 const void* geom, const void* bins, const float* saved, const float* g_rgb,
                 const float* g_alpha, const float* g_depth, float* d_means, float* d_scales,
                 float* d_colors, float* d_opacities, void* ws, size_t ws_bytes, void* stream);

/* gr_bwd for a caller that rendered a spatially re-ordered copy of its Gaussians (the drop-in op's Morton layout,
 * 3dgaussian_amd/torch_renderer.py): geom / bins / saved are the copy's render, means .. opacities and d_* are in the
 * CALLER's order, and index[r] (device int[n], a permutation) is the rendered position of the caller's row r.  The
 * chain rule runs in the caller's order (coalesced parameter reads and gradient writes; one gathered 32-byte sums
 * row per Gaussian), so the gradients come back in the caller's order without a separate pass. */
gr_status gr_bwd_indexed(const gr_view* v, int n, const gr_plan* plan, const float* means, const float* scales,
                         const float* colors, int color_dim, const float* opacities, const void* geom, const void* bins,
                         const float* saved, const float* g_rgb, const float* g_alpha, const float* g_depth,
                         const int* index, float* d_means, float* d_scales, float* d_colors, float* d_opacities, void* ws,
                         size_t ws_bytes, void* stream);

/* Camera gradient of a view after gr_bwd (its workspace ws still holds the per-Gaussian sums gr_bwd formed).
 * Replaces the autograd path of the reference's camera operands: python/torch_renderer.py:140-150 moves
 * camera.view / camera.proj into _project (:57-78), the SH view direction (cam = inv(view)[:3,3], :81-83) and the
 * sigma rule (fx = |proj[0,0]|, fy = |proj[1,1]|), so a caller whose camera tensors require grad gets their
 * gradients.  d_camera (device, 35 floats) receives d view (16, row-major), d proj (16) and d cam_pos (3; zero for
 * RGB colours: the caller adds its chain through inv(view)).  depth != 0: gr_bwd was given g_depth (its depth sums
 * enter too).  Deterministic (fixed-order double sums). */
#define GR_CAMERA_GRADS 35
gr_status gr_bwd_camera(const gr_view* v, int n, const gr_plan* plan, const float* means, const float* scales,
                        const float* colors, int color_dim, const float* opacities, void* ws, size_t ws_bytes, int depth,
                        float* d_camera, void* stream);

/* Backward of gr_fwd_render fused with the fit loop's view loss (fit_multiview_stub.py:292-299):
 *   loss = mean|out - target_rgb| + w_sil * mean|alpha - target_mask|   (target_mask may be NULL)
 * The upstream gradients are those of g_scale * loss (torch's abs' = sign, sign(0) = 0), computed
 * per pixel from the saved sums (the outputs recomputed bit-exactly); *loss_out (device float)
 * receives the unscaled view loss.  accumulate != 0 adds the gradients to d_* (a fit's gradient
 * accumulators, one per stream: deterministic in view order) instead of writing them.
 * Replaces, for the fit loop, the autograd chain L1 loss -> gr_bwd -> gradient accumulation across
 * views (fit_multiview_stub.py:299-310).  Same workspace as gr_bwd.  n == 0: no-op. */
gr_status gr_bwd_l1(const gr_view* v, int n, const gr_plan* plan, const float* means,
                    const float* scales, const float* colors, int color_dim, const float* opacities,
                    const void* geom, const void* bins, const float* saved, const float* target_rgb,
                    const float* target_mask, float w_sil, float g_scale, float* loss_out,
                    float* d_means, float* d_scales, float* d_colors, float* d_opacities,
                    int accumulate, void* ws, size_t ws_bytes, void* stream);

/* gr_bwd_l1 with the fit loop's depth term as well (fit_multiview_stub.py:301-305):
 *   loss = mean|out - target_rgb| + w_sil mean|alpha - target_mask|
 *          + w_depth mean|depth / (max(depth) + 1e-6) - target_depth|   (target_depth may be NULL)
 * with torch's gradients of that expression (abs' = sign, max's gradient shared evenly among the
 * arg-max pixels); the view must be rendered with no_depth_grad = 0 and its depth output.
 * gr_bwd_l1 = gr_bwd_fit with target_depth = NULL.  Same workspace as gr_bwd. */
gr_status gr_bwd_fit(const gr_view* v, int n, const gr_plan* plan, const float* means,
                     const float* scales, const float* colors, int color_dim, const float* opacities,
                     const void* geom, const void* bins, const float* saved, const float* target_rgb,
                     const float* target_mask, float w_sil, const float* target_depth, float w_depth,
                     float g_scale, float* loss_out, float* d_means, float* d_scales, float* d_colors,
                     float* d_opacities, int accumulate, void* ws, size_t ws_bytes, void* stream);

/* The fused fit path in three calls (fit_multiview.py; views rendered with no_depth_grad = 1):
 *   gr_fwd_render_l1  gr_fwd_render without depth output, whose epilogue also evaluates the fit
 *                     loop's view loss (as gr_bwd_l1) from the pixel sums: the view loss goes to
 *                     *loss_out, its upstream gradients (pre-split backward operands) to ws (the
 *                     gr_bwd_bytes workspace).  out_rgb / out_alpha may be NULL (no image written);
 *                     no saved sums are kept.
 *   gr_bwd_splat      the backward splat of that view: per-pair gradient partials into ws.
 *   gr_reduce_views   sums the partials of up to GR_REDUCE_MAX_VIEWS such views per Gaussian, applies
 *                     each view's chain rule and writes (accumulate = 0) or adds (accumulate != 0)
 *                     the summed gradient once: the parameters are read and the gradient buffers
 *                     written once per batch instead of once per view.
 * Together: gr_fwd_render + gr_bwd_l1 per view, up to float summation order.  Each view's geom,
 * bins and ws must stay untouched until gr_reduce_views has run on the stream.  Deterministic for a
 * given batch composition.  Replaces, for the fit loop, fit_multiview_stub.py:277-310 (render,
 * L1 + silhouette loss, autograd backward and its gradient sums over the views). */
#define GR_REDUCE_MAX_VIEWS 16
typedef struct gr_reduce_view {
  gr_view view;     /* the view as rendered (same camera, size and cutoffs)     */
  gr_plan plan;     /* its plan                                                */
  const void* geom; /* its gr_fwd_prepare(_async) workspace                    */
  const void* bins; /* its gr_fwd_render_l1 bins                               */
  const void* ws;   /* its gr_fwd_render_l1 / gr_bwd_splat workspace           */
} gr_reduce_view;

gr_status gr_fwd_render_l1(const gr_view* v, int n, const gr_plan* plan, const void* geom, void* bins,
                           size_t bins_bytes, void* scratch, size_t scratch_bytes,
                           const float* target_rgb, const float* target_mask, float w_sil,
                           float g_scale, float* loss_out, float* out_rgb, float* out_alpha,
                           void* ws, size_t ws_bytes, void* stream);

gr_status gr_bwd_splat(const gr_view* v, int n, const gr_plan* plan, const void* geom,
                       const void* bins, void* ws, size_t ws_bytes, void* stream);

gr_status gr_reduce_views(int num_views, const gr_reduce_view* views, int n, const float* means,
                          const float* scales, const float* colors, int color_dim,
                          const float* opacities, float* d_means, float* d_scales, float* d_colors,
                          float* d_opacities, int accumulate, void* stream);

/* gr_reduce_views in two stages, so that a fit can release each view's workspaces right after its
 * backward and the gathers run beside other views' splat kernels (what fit_multiview.py uses):
 *   gr_gather_view   right after gr_bwd_splat of a view: sums its per-pair partials per Gaussian into
 *                    `sums` (gr_view_sums_floats(n) device floats, 8 per Gaussian); the view's geom, bins
 *                    and ws may be released once this has run on the stream.
 *   gr_reduce_sums   the chain rule of up to GR_REDUCE_MAX_VIEWS gathered views: writes (accumulate = 0)
 *                    or adds (accumulate != 0) their summed gradient once.
 * gr_gather_view per view + gr_reduce_sums = gr_reduce_views, up to float summation order (the gathers
 * sum in f32, gr_reduce_views in f64).  Deterministic.  Replaces the same reference code as
 * gr_reduce_views (fit_multiview_stub.py:310, the autograd sums over the views). */
typedef struct gr_sums_view {
  gr_view view;       /* the view as rendered (its camera: the chain rule)                        */
  const float* sums;  /* its gr_gather_view / gr_bwd_fit_gather output                           */
  const float* sums3; /* its per-Gaussian depth sums (gr_bwd_fit_gather; n floats), or NULL (none) */
} gr_sums_view;
size_t gr_view_sums_floats(int n);
gr_status gr_gather_view(const gr_view* v, int n, const gr_plan* plan, const void* geom, const void* bins,
                         const void* ws, float* sums, void* stream);
/* gr_bwd_fit up to the reduction (its depth-loss kernels, the backward splat with the depth-coupled tail pairs and
 * the gather), the per-Gaussian sums going to `sums` (gr_view_sums_floats(n)) and the depth sums to `sums3` (n
 * floats): a depth-loss fit reduces a batch of such views with one gr_reduce_sums (their sums3 set), as the fit path
 * without a depth term does.  The view's geom, bins, saved sums and ws may be released once this has run. */
gr_status gr_bwd_fit_gather(const gr_view* v, int n, const gr_plan* plan, const void* geom, const void* bins,
                            const float* saved, const float* target_rgb, const float* target_mask, float w_sil,
                            const float* target_depth, float w_depth, float g_scale, float* loss_out, void* ws,
                            size_t ws_bytes, float* sums, float* sums3, void* stream);
gr_status gr_reduce_sums(int num_views, const gr_sums_view* views, int n, const float* means,
                         const float* scales, const float* colors, int color_dim,
                         const float* opacities, float* d_means, float* d_scales, float* d_colors,
                         float* d_opacities, int accumulate, void* stream);

/* The fit step's views in one call: the per-view schedule of 3dgaussian_amd/fit_multiview.py
 * (fit_multiview_stub.py:277-310 across several HIP streams) as native host code
 * (3dgaussian_amd/csrc/gr_fit_exec.cpp).  Per view: its preparation ahead on the executor's preparation
 * stream (groups of prep_group views, the first of prep_first), then on render stream j % num_streams
 * (stream 0 = `stream`, the caller's) without a depth target gr_fwd_render_l1 + gr_bwd_splat +
 * gr_gather_view, every batch of a stream's views (reduce_batch at most, its last reduce_tail views)
 * gr_reduce_sums into that stream's accumulators; with depth targets gr_fwd_render + gr_bwd_fit_gather per view and the
 * same batched gr_reduce_sums (with the depth sums).
 * losses[j] (device) receives view j's loss; acc[4k + 0..3] are stream k's d_means, d_scales, d_colors,
 * d_opacities accumulators (written by its first batch, then added to), for k < min(num_streams,
 * num_views): the caller sums them in stream order.  Workspaces are the executor's own, reused in
 * stream order (gr_fit_exec.cpp).  Everything is ordered after `stream` and `stream` is ordered after everything when this
 * returns.  Deterministic; bit-identical to fit_multiview.py's Python schedule with the same settings.
 * The executor holds the streams, events and pinned plan buffer across steps (one per device). */
typedef struct gr_executor gr_executor;
typedef struct gr_fit_target {
  gr_view view;               /* the view (no_depth_grad 1 or 2 without a depth target, 0 with one) */
  const float* target_rgb;    /* (H,W,3) float32 device                                           */
  const float* target_mask;   /* (H,W) or NULL (no silhouette term)                                */
  const float* target_depth;  /* (H,W) or NULL; all views of a call have one, or none              */
} gr_fit_target;
typedef struct gr_fit_config {
  int num_streams;  /* render streams (the caller's + num_streams - 1 of the executor's)      */
  int prep_ahead;   /* views prepared ahead of the one rendering                               */
  int prep_group;   /* views per preparation (<= GR_PREPARE_MAX_VIEWS)                          */
  int prep_first;   /* views of the first preparation                                           */
  int reduce_batch; /* views per gr_reduce_sums (<= GR_REDUCE_MAX_VIEWS)                        */
  int reduce_tail;  /* views in each stream's last batch (0: near-equal batches only)           */
  /* Optional caller-owned streams (hipStream_t): render streams 1..num_streams-1 and the preparation
   * stream.  NULL: the executor's own.  HIP maps streams to GPU_MAX_HW_QUEUES hardware queues in creation
   * order; two render streams on one queue run one after the other, so a caller that already holds
   * streams on distinct queues passes them here.  A change of streams between calls drains the previous
   * ones first. */
  void* const* render_streams;
  void* prep_stream;
  /* Device-side sizing (optional; NULL: the host reads each view's plan before sizing its render): per view its
   * capacities (gr_fwd_prepare_views_sized; the views must have device_counts = 1), the pinned rows receiving the
   * true counts (may be NULL) and the device int raised when a view exceeds its capacities.  No host wait in the
   * call then: the host enqueues the whole step while the device runs it. */
  const gr_plan* caps;
  gr_plan* observed;
  int* overflow;
} gr_fit_config;
gr_status gr_executor_create(int device, gr_executor** executor);
void gr_executor_destroy(gr_executor* executor);
gr_status gr_fit_views(gr_executor* executor, const gr_fit_config* config, int num_views,
                       const gr_fit_target* views, int n, const float* means, const float* scales,
                       const float* colors, int color_dim, const float* opacities, float w_sil,
                       float w_depth, float g_scale, float* losses, float* const* acc, void* stream);

/* ------------------------------------------------------------------------------------------ */
/* Legacy uint8 surface (host pointers), replaces gr::render_gaussians (renderer.h:33-39).    */
/* Semantics of renderer_cpu.cpp: 3-sigma box, w < 1e-5 skip, uint8 round-half-up, A = 255.  */
/* enable_depth_sort = 1 gives exact per-pixel front-to-back compositing in camera-z order.   */
/* rgba must hold width*height*4 bytes.                                                       */
/* ------------------------------------------------------------------------------------------ */
gr_status gr_render_u8(const gr_render_params* p, int n, const float* means, const float* scales,
                       const float* colors, const float* opacities, uint8_t* rgba);

/* ------------------------------------------------------------------------------------------ */
/* Fit-loop loss, the caller's side of the render op (fit_multiview_stub.py:292-299):         */
/*   loss = mean|a - b| + w2 * mean|c - d|   (photometric L1 + weighted silhouette L1)        */
/* Device pointers, float32, stream-ordered, deterministic.  c, d may be NULL with n2 = 0.     */
/* The backward writes g_a = g sign(a-b)/n1 and g_c = (w2 g) sign(c-d)/n2, g = *g_loss.        */
/* ------------------------------------------------------------------------------------------ */
size_t gr_l1_loss_ws_bytes(void);
gr_status gr_l1_loss_fwd(const float* a, const float* b, int64_t n1, const float* c, const float* d,
                         int64_t n2, float w2, float* loss, void* ws, size_t ws_bytes, void* stream);
gr_status gr_l1_loss_bwd(const float* a, const float* b, int64_t n1, const float* c, const float* d,
                         int64_t n2, float w2, const float* g_loss, float* g_a, float* g_c,
                         void* stream);

/* ------------------------------------------------------------------------------------------ */
/* Fit-loop parameter update, the caller's side of the render op (fit_multiview_stub.py:268-275   */
/* activations, :307-308 regulariser, :311 torch.optim.Adam), one pass per parameter tensor:    */
/*   grad = act'(param) * (((accs[0] + accs[1]) + ...) + reg)  (up to GR_FIT_MAX_ACC device arrays  */
/*          of count floats, summed in order; act 0 identity,                                     */
/*          1 softplus(x) + 1e-3, 2 sigmoid: torch's backward formulas);                          */
/*   adam != 0: exp_avg / exp_avg_sq / param updated as Adam's foreach step with                 */
/*   neg_step_size = -lr / (1 - beta1^t), bias_correction2_sqrt = sqrt(1 - beta2^t); the betas are */
/*   doubles so 1 - beta rounds to float as torch's Python-float scalars do.                     */
/* gr_adam_step: the Adam update alone on an assembled gradient (after an all-reduce).           */
/* ------------------------------------------------------------------------------------------ */
#define GR_FIT_MAX_ACC 8
gr_status gr_fit_param_step(int64_t count, int act, float* param, float* grad, const float* const* accs,
                            int num_accs, float reg, int adam, float* exp_avg, float* exp_avg_sq,
                            float neg_step_size, float bias_correction2_sqrt, double beta1, double beta2,
                            float eps, void* stream);
gr_status gr_adam_step(int64_t count, float* param, const float* grad, float* exp_avg,
                       float* exp_avg_sq, float neg_step_size, float bias_correction2_sqrt,
                       double beta1, double beta2, float eps, void* stream);
/* gr_fit_param_steps: gr_fit_param_step (adam != 0) for up to GR_FIT_MAX_PARAMS parameter tensors in one launch
 * (world size 1: no all-reduce between the gradient and the update), each with its own count, activation, arrays,
 * regulariser weight and bias corrections; the same results as one gr_fit_param_step per tensor. */
#define GR_FIT_MAX_PARAMS 8
typedef struct gr_param_step {
  int64_t count;
  int act;
  int num_accs;
  float* param;
  float* grad;                           /* may be NULL: the gradient is not stored */
  const float* accs[GR_FIT_MAX_ACC];
  float* exp_avg;
  float* exp_avg_sq;
  float reg;
  float neg_step_size;
  float bias_correction2_sqrt;
} gr_param_step;
gr_status gr_fit_param_steps(int num, const gr_param_step* steps, double beta1, double beta2, float eps, void* stream);
/* gr_fit_param_steps with the step's Adam scalars and its validity on the device, so that a step captured once (HIP
 * graph) can be replayed: each entry's neg_step_size / bias_correction2_sqrt are replaced by sched[2t], sched[2t+1]
 * with t = *step_dev (the updates applied so far; sched holds them for every step the caller may run), and nothing is
 * updated when *overflow != 0 (a view of the step exceeded its capacity: gr_fwd_prepare_views_sized).  After the
 * update one thread advances *step_dev (no overflow) or raises host_flags[0] (overflow, sticky: the caller clears
 * it), mirrors *step_dev to host_flags[1] and clears *overflow for the next step.  host_flags: pinned host int[2]. */
gr_status gr_fit_param_steps_sched(int num, const gr_param_step* steps, double beta1, double beta2, float eps,
                                   const float* sched, int* step_dev, int* overflow, int* host_flags, void* stream);
/* gr_fit_activations: the fit loop's activations (fit_multiview_stub.py:268-275) in one launch, torch's float formulas:
 * scales = softplus(scales_raw) + 1e-3 (3n floats; x > 20: x), opacities = sigmoid(opacities_raw) (n), and with
 * colors_raw colors = sigmoid(colors_raw) (color_count floats; NULL for SH coefficients, used as they are).  With
 * reg_out, also the regulariser of :307-308, reg_opacity * mean(opacities) + reg_scale * mean(scales), as a device
 * float (the means in double over a fixed block order, then rounded): ws of gr_fit_activations_ws_bytes(n), whose
 * counter must be zero on the first call and is left zero. */
size_t gr_fit_activations_ws_bytes(int64_t n);
gr_status gr_fit_activations(int64_t n, const float* scales_raw, const float* opacities_raw, const float* colors_raw,
                             int64_t color_count, float* scales, float* opacities, float* colors, float reg_scale,
                             float reg_opacity, float* reg_out, void* ws, size_t ws_bytes, void* stream);

/* The fused fit path for up to GR_BATCH_MAX_VIEWS views of one image size in one launch per kernel: per view what
 * gr_fwd_render_l1 + gr_bwd_splat + gr_gather_view do (no_depth_grad = 1; 16- or 32-pixel tiles), or with
 * target_depth what gr_fwd_render (saved sums) + gr_bwd_fit_gather do (no_depth_grad = 0, 16-pixel tiles), each
 * kernel's blocks of every view in one grid.  For small views (C2, C3: a few hundred work items per splat) one view
 * per launch leaves most of the 256 CUs idle; the views of a batch fill them.  The views were prepared (geom, plan)
 * and may be device-sized (device_counts = 1, plan = capacities); bins / scratch / ws (/ saved: 5 floats per
 * pixel, depth path) are the single-view calls' workspaces, sums (n x 8) and sums3 (n, depth path) receive what
 * gr_gather_view / gr_bwd_fit_gather write, loss the view loss.  Then gr_reduce_sums as usual.  Same results as the
 * single-view calls, bit for bit (every block computes what it computes in its own view's launch). */
#define GR_BATCH_MAX_VIEWS 8
typedef struct gr_batch_view {
  gr_view view;
  gr_plan plan;
  const void* geom;
  void* bins;
  size_t bins_bytes;
  void* scratch;
  size_t scratch_bytes;
  void* ws;
  size_t ws_bytes;
  float* saved;
  const float* target_rgb;
  const float* target_mask;
  const float* target_depth;
  float* sums;
  float* sums3;
  float* loss;
} gr_batch_view;
gr_status gr_fit_views_batched(int num_views, const gr_batch_view* views, int n, float w_sil, float w_depth,
                               float g_scale, void* stream);

/* ------------------------------------------------------------------------------------------ */
/* Introspection (host-only, no GPU needed).                                                  */
/* ------------------------------------------------------------------------------------------ */

/* Byte offsets of the sub-buffers inside geom / bins, for debugging and bit-exact tests.
 *   geom: [0] records float4[n+1][2], 32 bytes per Gaussian (record n: padding, o = 0):
 *             A = (px, py, qx, qy), B = (o, r, g, b); then float z_abs[n+1] (entry n: 0)
 *         [1] rect int4[n] (tx0,ty0,tx1,ty1) [2] counts u64[n+1] [3] offsets u64[n+1]
 *         [4] device copy of the plan (gr_plan) and the exact pair total [5] end of the fixed part
 *         (counts/offsets packed: core tiles / first core pair in the low word, tail tiles / first
 *         tail pair after the num_core_pairs core pairs in the high word)
 *   bins: [0] keys (radix-sort fallback only, > 8192 tiles) [1] int[K] Gaussian id of each sorted pair
 *         [2] ranges int2[2 * tiles]: per virtual tile (2t: core list of tile t, 2t+1: its tail list)
 *         [3] pos_of int[K]: sorted position of each pair by emission index (= backward partial-sum
 *         slot order: Gaussian-major, tiles in raster order, core zone first) */
#define GR_GEOM_PARTS 6
void gr_geom_layout(int n, size_t offsets_out[GR_GEOM_PARTS]);
void gr_bins_layout(const gr_view* v, int n, const gr_plan* plan, size_t offsets_out[4]);

/* Live kernel timing with HIP events on the launch stream (bench.py).  Between begin and end,
 * the timed stages are bracketed by two events each; end() synchronises them and returns the
 * summed device time and count of [0] the forward splat kernel, [1] the backward splat kernel,
 * [2] the backward reduction kernel, [3] the binning stage (emit + sort + ranges + work items). */
void gr_profile_begin(void);
gr_status gr_profile_end(double total_ms[4], int launches[4]);

const char* gr_last_error(void);
const char* gr_version(void);

#ifdef __cplusplus
}
#endif

#endif /* GR_HIP_H_ */
