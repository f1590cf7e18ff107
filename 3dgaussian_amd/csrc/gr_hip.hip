// gr_hip.hip — MI355X (gfx950, CDNA4) differentiable Gaussian rasterizer: HIP kernels + C ABI.
//
// Replaces src/renderer.cu (4 CUDA kernels, forward only, uint8, static buffers) and the math of
// python/torch_renderer.py:109-203 (+ its autograd backward) with a tile-binned forward/backward
// (DESIGN.md §5 has the costs; gr_fwd_prepare(_async) / gr_fwd_render / gr_bwd run them in order):
//
//   k_preprocess     per Gaussian: project (torch_renderer.py:57-78), colour (:81-106,:144), sigma
//                    (:146-150), 7-sigma tile rectangle, tile culling into core (5.5 sigma) and tail
//                    tiles, pair counts, 32-byte raster record.
//   k_plan/k_offsets pair offsets (exclusive scan: blocks, then Gaussians); pair totals (overflow-checked) for the host.
//   k_emit_zones     (tile, Gaussian) pairs in Gaussian order: core pairs, then tail pairs.
//   k_tile_count / k_tile_colscan / k_tile_place
//                    stable counting sort of each zone by tile (per-tile lists in Gaussian order) and
//                    pos_of (sorted position of each pair, by emission index).
//   k_work_items_zones  per-(virtual) tile ranges, work items of <= CH pairs.
//   k_raster_fwd_mfma   per work item: records staged through LDS by LDS-DMA, the separable splat as
//                    a contraction on bf16 MFMA with split operands;
//                    a tile split over several items is finished by its last item (arrival ticket);
//                    out/alpha/depth + saved, with the fit loss its upstream fragments and the view loss.
//   k_pixel_grads    per pixel upstream vector U = (dC, dW, dD), pre-split into MFMA fragments.
//   k_raster_bwd_bf16   per work item: the two K = 16 contractions (over x, over y) of U with the
//                    Gaussians' exponentials; 8- or 9-float partial rows at the pairs' sorted positions.
//   k_reduce_bwd     per Gaussian: its rows (through pos_of) summed in a fixed order (deterministic, no
//                    float atomics), then the chain rule back to means/scales/colours/opacity.
//
// The legacy uint8 surface (gr_render_u8, renderer_cpu.cpp semantics) reuses the binning with a
// 3-sigma box, and adds exact depth-sorted front-to-back compositing (enable_depth_sort=1).
//
// Built with -ffp-contract=off: the preprocess float sequence must match oracle/gr_oracle.c
// bit-for-bit (tile rectangles are integers derived from it); hot loops use explicit fmaf.

#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <rocprim/rocprim.hpp>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/gr_hip.h"

// Timing experiments only (tools/ab_variant.sh "-DGR_DEBUG_SKIP=<mask>"): launches left out of a variant
// build to measure their marginal cost in the overlapped fit step - 1 forward splat, 2 backward splat,
// 4 gather, 8 chain-rule reduction, 16 parameter update.  Results of such a build are wrong; the product
// build has 0.  GR_DEBUG_BIN_REPS / GR_DEBUG_PREP_REPS > 1 repeat a view's binning / a group's
// preparation (idempotent: same results) to measure their marginal cost the other way round.
// Tail pairs (the zone between the core and the outer cutoff, where a Gaussian's weight is below
// o * exp(-core^2/2)) carry only W and D.  GR_TAIL2 = 1: their forward and backward contractions use two
// pieces per operand (three products) in every precision mode; their terms are at most e^-15 of the
// Gaussian's peak, so the split's ~2^-16 relative error is far below the f32 grade the core keeps.
#ifndef GR_TAIL2
#define GR_TAIL2 1
#endif
#ifndef GR_DEBUG_PREP_REPS
#define GR_DEBUG_PREP_REPS 1
#endif
#ifndef GR_DEBUG_BIN_REPS
#define GR_DEBUG_BIN_REPS 1
#endif
#ifndef GR_DEBUG_SKIP
#define GR_DEBUG_SKIP 0
#endif

#define GR_VERSION_STR "gr_hip 0.1.0 (gfx950)"

namespace {

thread_local std::string g_last_error;

gr_status set_error(gr_status st, const std::string& msg) {
  g_last_error = msg;
  return st;
}

#define GR_HIP_TRY(expr)                                                                          \
  do {                                                                                            \
    hipError_t e_ = (expr);                                                                       \
    if (e_ != hipSuccess)                                                                         \
      return set_error(GR_ERR_HIP, std::string("HIP error: ") + hipGetErrorString(e_) + " (" +   \
                                       std::to_string((int)e_) + ") at " __FILE__ ":" +           \
                                       std::to_string(__LINE__) + " in " #expr);                  \
  } while (0)

constexpr int T = GR_TILE;        // tile edge
constexpr int TP = GR_TILE * GR_TILE;  // pixels per tile (256)
constexpr float LOG2E = 1.4426950408889634f;

inline size_t align_up(size_t x, size_t a = 256) { return (x + a - 1) / a * a; }

// Tile edge of a view (gr_view.tile): GR_TILE (16) or 32 (the fused fit path's 32-pixel tiles, T32).
constexpr int T32 = 32, TP32 = T32 * T32;
inline int tile_of(const gr_view* v) { return v->tile == T32 ? T32 : T; }
inline int tiles_x_of(int w, int t = T) { return (w + t - 1) / t; }
inline int tiles_y_of(int h, int t = T) { return (h + t - 1) / t; }
inline int tiles_of(const gr_view* v) { return tiles_x_of(v->width, tile_of(v)) * tiles_y_of(v->height, tile_of(v)); }
// Binning unit of the differentiable path: virtual tile 2t holds tile t's core pairs, 2t+1 its tail
// pairs (two-zone footprint), so the pair lists, ranges and work items are per virtual tile.
inline int vtiles_of(const gr_view* v) { return 2 * tiles_of(v); }

int bits_for(uint32_t maxval) {
  int b = 1;
  while (b < 32 && (1u << b) <= maxval) ++b;
  return b;
}

// Kernel parameter block (by value): matrices etc.
struct ViewK {
  int W, H, tiles_x, tiles_y;
  int T, ts;          // tile edge and its log2 (the preparation and binning; the splat kernels are per tile size)
  int ty0, ty1;       // the band of tile rows rendered (gr_view.row0 / rows; the whole view: 0, tiles_y)
  float V[16], P[16];
  float bg[3];
  float cam[3];
  float cutoff;
  float core;         // core radius of the two-zone footprint (= cutoff: one zone)
  const float* bgp;   // gr_view.background_dev: the background read on the device (else bg)
};

// Background channel k of the view (gr_view.background_dev when set: one cached load).
__device__ __forceinline__ float view_bg(const ViewK& v, int k) { return v.bgp ? v.bgp[k] : v.bg[k]; }

ViewK make_viewk(const gr_view* v) {
  ViewK k;
  k.W = v->width;
  k.H = v->height;
  k.T = tile_of(v);
  k.ts = k.T == T32 ? 5 : 4;
  static_assert(T == 16, "ViewK::ts");
  k.tiles_x = tiles_x_of(v->width, k.T);
  k.tiles_y = tiles_y_of(v->height, k.T);
  k.ty0 = v->rows > 0 ? v->row0 : 0;
  k.ty1 = v->rows > 0 ? std::min(v->row0 + v->rows, k.tiles_y) : k.tiles_y;
  std::memcpy(k.V, v->view, sizeof(k.V));
  std::memcpy(k.P, v->proj, sizeof(k.P));
  std::memcpy(k.bg, v->background, sizeof(k.bg));
  std::memcpy(k.cam, v->cam_pos, sizeof(k.cam));
  k.cutoff = v->cutoff > 0.0f ? v->cutoff : 7.0f;
  k.core = (v->core_cutoff > 0.0f && v->core_cutoff < k.cutoff) ? v->core_cutoff : k.cutoff;
  k.bgp = v->background_dev;
  return k;
}

// ------------------------------------------------------------------------------------------------
// Projection (torch_renderer.py:57-78, 146-150).  Same float32 sequence as oracle/gr_oracle.c.
// ------------------------------------------------------------------------------------------------
struct Proj {
  float pc[4], clip[4];
  float ws, px, py, za, sxr, syr, sx, sy;
  bool valid;
};

__device__ __forceinline__ void project(const ViewK& v, float x, float y, float z, float s0, float s1, Proj& o) {
#pragma unroll
  for (int i = 0; i < 4; ++i) o.pc[i] = ((v.V[i * 4 + 0] * x + v.V[i * 4 + 1] * y) + v.V[i * 4 + 2] * z) + v.V[i * 4 + 3];
#pragma unroll
  for (int i = 0; i < 4; ++i)
    o.clip[i] = ((v.P[i * 4 + 0] * o.pc[0] + v.P[i * 4 + 1] * o.pc[1]) + v.P[i * 4 + 2] * o.pc[2]) + v.P[i * 4 + 3] * o.pc[3];
  const float w = o.clip[3];
  o.ws = (fabsf(w) < 1e-8f) ? 1.0f : w;
  const float nx = o.clip[0] / o.ws, ny = o.clip[1] / o.ws, nz = o.clip[2] / o.ws;
  o.px = (nx * 0.5f + 0.5f) * (float)(v.W - 1);
  o.py = (1.0f - (ny * 0.5f + 0.5f)) * (float)(v.H - 1);
  o.valid = (nz >= -1.0f) && (nz <= 1.0f) && (w != 0.0f);
  const float az = fabsf(o.pc[2]);
  o.za = az < 1e-6f ? 1e-6f : az;
  const float fx = fabsf(v.P[0]), fy = fabsf(v.P[5]);
  o.sxr = fabsf(s0) * 0.5f * (float)v.W * fx / o.za;
  o.syr = fabsf(s1) * 0.5f * (float)v.H * fy / o.za;
  o.sx = o.sxr < 1.0f ? 1.0f : o.sxr;
  o.sy = o.syr < 1.0f ? 1.0f : o.syr;
}

// Degree-3 extension of the reference's direction basis (torch_renderer.py:94-106 has degree 1:
// col = k0 + k1 x + k2 y + k3 z with d = (x, y, z) the unit view direction).  The basis is the real
// spherical-harmonic polynomials up to degree 3 without normalisation constants, continuing the
// reference's unnormalised degree-1 terms: 1 | x y z | xy yz 3z^2-1 xz x^2-y^2 | y(3x^2-y^2) xyz
// y(5z^2-1) z(5z^2-3) x(5z^2-1) z(x^2-y^2) x(x^2-3y^2).  With the degree-2/3 coefficients zero it is
// the reference's degree-1 colour (same float operations for the first four terms).
template <typename F>
__host__ __device__ __forceinline__ void sh3_basis(F x, F y, F z, F (&Y)[16]) {
  Y[0] = F(1);
  Y[1] = x;
  Y[2] = y;
  Y[3] = z;
  Y[4] = x * y;
  Y[5] = y * z;
  Y[6] = F(3) * z * z - F(1);
  Y[7] = x * z;
  Y[8] = x * x - y * y;
  Y[9] = y * (F(3) * x * x - y * y);
  Y[10] = x * y * z;
  Y[11] = y * (F(5) * z * z - F(1));
  Y[12] = z * (F(5) * z * z - F(3));
  Y[13] = x * (F(5) * z * z - F(1));
  Y[14] = z * (x * x - y * y);
  Y[15] = x * (x * x - F(3) * y * y);
}
// d Y_i / d(x, y, z)
template <typename F>
__host__ __device__ __forceinline__ void sh3_basis_grad(F x, F y, F z, F (&G)[16][3]) {
  const F xx = x * x, yy = y * y, zz = z * z;
  const F g[16][3] = {{0, 0, 0},
                      {1, 0, 0},
                      {0, 1, 0},
                      {0, 0, 1},
                      {y, x, 0},
                      {0, z, y},
                      {0, 0, F(6) * z},
                      {z, 0, x},
                      {F(2) * x, F(-2) * y, 0},
                      {F(6) * x * y, F(3) * xx - F(3) * yy, 0},
                      {y * z, x * z, x * y},
                      {0, F(5) * zz - F(1), F(10) * y * z},
                      {0, 0, F(15) * zz - F(3)},
                      {F(5) * zz - F(1), 0, F(10) * x * z},
                      {F(2) * x * z, F(-2) * y * z, xx - yy},
                      {F(3) * xx - F(3) * yy, F(-6) * x * y, 0}};
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 3; ++j) G[i][j] = g[i][j];
}

// Colour before clamp (torch_renderer.py:86-106): RGB (CD = 3), the reference's degree-1 basis
// (CD = 12) or its degree-3 extension (CD = 48).
template <int CD>
__device__ __forceinline__ void eval_color(const ViewK& v, float mx, float my, float mz, const float* col, float out[3]) {
  if constexpr (CD == 3) {
    out[0] = col[0];
    out[1] = col[1];
    out[2] = col[2];
  } else {
    float d0 = v.cam[0] - mx, d1 = v.cam[1] - my, d2 = v.cam[2] - mz;
    const float nrm = sqrtf(d0 * d0 + d1 * d1 + d2 * d2) + 1e-8f;
    d0 /= nrm;
    d1 /= nrm;
    d2 /= nrm;
#pragma unroll
    for (int k = 0; k < 3; ++k) out[k] = ((col[k] + col[3 + k] * d0) + col[6 + k] * d1) + col[9 + k] * d2;
    if constexpr (CD == 48) {
      float Y[16];
      sh3_basis(d0, d1, d2, Y);
#pragma unroll
      for (int i = 4; i < 16; ++i)
#pragma unroll
        for (int k = 0; k < 3; ++k) out[k] += col[3 * i + k] * Y[i];
    }
  }
}

__device__ __forceinline__ float clamp01(float x) { return x < 0.0f ? 0.0f : (x > 1.0f ? 1.0f : x); }

// Tile rectangle of the cutoff*sigma box (oracle/gr_oracle.c tile_rect, bit-exact).
__device__ __forceinline__ int tile_rect(const ViewK& v, const Proj& p, float op, int4& r) {
  r = make_int4(0, 0, -1, -1);
  if (!p.valid || !(op >= 0.0f)) return 0;
  const float R = v.cutoff;
  const float rx = R * p.sx, ry = R * p.sy;
  const float lox = p.px - rx, hix = p.px + rx, loy = p.py - ry, hiy = p.py + ry;
  const float wm1 = (float)(v.W - 1), hm1 = (float)(v.H - 1);
  if (!(hix >= 0.0f) || !(lox <= wm1) || !(hiy >= 0.0f) || !(loy <= hm1)) return 0;
  const int x0 = (lox <= 0.0f) ? 0 : (int)floorf(lox);
  const int x1 = (hix >= wm1) ? (v.W - 1) : (int)ceilf(hix);
  const int y0 = (loy <= 0.0f) ? 0 : (int)floorf(loy);
  const int y1 = (hiy >= hm1) ? (v.H - 1) : (int)ceilf(hiy);
  r = make_int4(x0 >> v.ts, y0 >> v.ts, x1 >> v.ts, y1 >> v.ts);  // (x0, y0 >= 0: the oracle's x0 / T)
  r.y = max(r.y, v.ty0);  // a band of tile rows (gr_view.rows): the tiles outside it get no pair
  r.w = min(r.w, v.ty1 - 1);
  if (r.y > r.w) {
    r = make_int4(0, 0, -1, -1);
    return 0;
  }
  return (r.z - r.x + 1) * (r.w - r.y + 1);
}

// Largest weight of a Gaussian over tile (tx,ty)'s pixel centres (clipped to the image), as the exp2
// exponent e = log2(w/o); q = -0.5 log2(e) / sigma^2 as stored in record word A
// (oracle/gr_oracle.c tile_emax, bit-exact).
__device__ __forceinline__ float tile_emax(const ViewK& v, float px, float py, float qx, float qy, int tx, int ty) {
  const int xe = min(tx * v.T + v.T - 1, v.W - 1), ye = min(ty * v.T + v.T - 1, v.H - 1);
  const float lox = (float)(tx * v.T) + 0.5f, hix = (float)xe + 0.5f;
  const float loy = (float)(ty * v.T) + 0.5f, hiy = (float)ye + 0.5f;
  const float cx = px < lox ? lox : (px > hix ? hix : px);
  const float cy = py < loy ? loy : (py > hiy ? hiy : py);
  const float dx = cx - px, dy = cy - py;
  return (dx * dx) * qx + (dy * dy) * qy;
}

__device__ __forceinline__ float radius_thr(float R) { return (-0.5f * LOG2E) * (R * R); }

// tile_emax in its column and row terms, ex(tx) + ey(ty) (the same float operations, so the same value bit for bit):
// the tile loops of the preparation and of the emission evaluate the row term once per row.
__device__ __forceinline__ float tile_ex(const ViewK& v, float px, float qx, int tx) {
  const int xe = min(tx * v.T + v.T - 1, v.W - 1);
  const float lox = (float)(tx * v.T) + 0.5f, hix = (float)xe + 0.5f;
  const float cx = px < lox ? lox : (px > hix ? hix : px);
  const float dx = cx - px;
  return (dx * dx) * qx;
}
__device__ __forceinline__ float tile_ey(const ViewK& v, float py, float qy, int ty) {
  const int ye = min(ty * v.T + v.T - 1, v.H - 1);
  const float loy = (float)(ty * v.T) + 0.5f, hiy = (float)ye + 0.5f;
  const float cy = py < loy ? loy : (py > hiy ? hiy : py);
  const float dy = cy - py;
  return (dy * dy) * qy;
}
// tile_class from the two terms and the view's two thresholds (radius_thr of the cutoff and of the core)
__device__ __forceinline__ int tile_class_e(float e, float thr_cut, float thr_core) {
  return !(e >= thr_cut) ? 0 : (e >= thr_core ? 2 : 1);
}

// Tile culling inside the rectangle: keep tile (tx,ty) iff the Gaussian's largest weight over it is
// >= o * exp(-cutoff^2/2).
__device__ __forceinline__ bool tile_pass(const ViewK& v, float px, float py, float qx, float qy, int tx, int ty) {
  return tile_emax(v, px, py, qx, qy, tx, ty) >= radius_thr(v.cutoff);
}

// Two-zone footprint (oracle/gr_oracle.c tile_class): 0 culled, 1 tail (largest weight below
// o * exp(-core^2/2): W and D forward, depth-coupled terms backward), 2 core (every channel).
__device__ __forceinline__ int tile_class(const ViewK& v, float px, float py, float qx, float qy, int tx, int ty) {
  const float e = tile_emax(v, px, py, qx, qy, tx, ty);
  if (!(e >= radius_thr(v.cutoff))) return 0;
  return e >= radius_thr(v.core) ? 2 : 1;
}

__device__ __forceinline__ float qcoef(float s) { return (-0.5f * LOG2E) / (s * s); }


// ------------------------------------------------------------------------------------------------
// Geometry buffer layout.
// ------------------------------------------------------------------------------------------------
// Per-Gaussian raster record, 32 bytes = one aligned 32-byte sector, so the random per-pair gathers of
// the raster kernels touch one sector per pair and two Morton neighbours share a 64-byte segment:
//   rec[2i+0] = A: px, py, qx, qy  (q = -0.5*log2(e)/sigma^2)
//   rec[2i+1] = B: o, r, g, b (clamped)
// followed (same geom part) by the camera depths z_abs[n+1] (only the forward's D channel and the
// depth-coupled backward read them): zrec_of().
constexpr int REC4 = 2;  // float4 per record

// Per-Gaussian pair counts of the two zones, packed core | tail << 32 into one u64; its exclusive
// scan gives each Gaussian's first core pair (low word, in [0, Kc)) and first tail pair (high word,
// relative to Kc: tail pairs fill [Kc, K)).  A pair's index in this emission order is also its
// backward partial-sum slot, so each Gaussian's partials are contiguous (k_reduce_bwd).  The packed
// words cannot carry into each other as long as K < 2^31, which k_plan checks against an exact
// 64-bit total (Geom::total) before trusting them.
struct Cnt2 {
  unsigned long long v;
  __host__ __device__ unsigned c() const { return (unsigned)(v & 0xffffffffull); }
  __host__ __device__ unsigned t() const { return (unsigned)(v >> 32); }
};

struct Geom {
  float4* rec;   // [n+1][REC4] raster records (record n: padding)
  float* zr;     // [n+1] camera depth z_abs (entry n: padding), right after the records
  int4* rect;    // tile rectangle
  unsigned long long* counts;   // n+1, packed Cnt2
  unsigned long long* offsets;  // n+1, packed Cnt2
  gr_plan* plan;                // device copy of the plan (gr_fwd_prepare_async copies it to the host)
  unsigned long long* total;    // [blocks of k_preprocess] exact per-block totals of kept pairs (overflow check)
  float* omax;                  // [blocks of k_preprocess] largest opacity of the block's kept Gaussians
  int* f16_sa;                  // [1] exponent pre-scale of the f16 forward's A operands (k_plan, f16_sa_of)
  void* scan_tmp;
  size_t scan_tmp_bytes;
};

// off: [0] records, [1] rect, [2] counts, [3] offsets, [4] device copy of the plan + exact per-block
//      totals + per-block opacity maxima + the f16 pre-scale, [5] scan temp (= end of the fixed part)
size_t geom_fixed(int n, size_t off[GR_GEOM_PARTS]) {
  size_t o = 0;
  const size_t nn = (size_t)(n > 0 ? n : 1);
  off[0] = o; o = align_up(o + (nn + 1) * (REC4 * sizeof(float4) + sizeof(float)));  // + pad record rec[n]; z[n+1]
  off[1] = o; o = align_up(o + nn * sizeof(int4));
  off[2] = o; o = align_up(o + (nn + 1) * sizeof(unsigned long long));
  off[3] = o; o = align_up(o + (nn + 1) * sizeof(unsigned long long));
  off[4] = o; o = align_up(o + sizeof(gr_plan) + (nn / 256 + 2) * (sizeof(unsigned long long) + sizeof(float)) + 16);
  off[5] = o;
  return o;
}

template <typename CountT>
size_t scan_tmp_bytes_t(int n) {
  size_t tmp = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, (CountT*)nullptr, (CountT*)nullptr, n + 1, (hipStream_t)0);
  return tmp;
}
size_t scan_tmp_bytes(int n) { return scan_tmp_bytes_t<unsigned long long>(n); }

Geom geom_view(void* base, int n) {
  size_t off[GR_GEOM_PARTS];
  const size_t fixed = geom_fixed(n, off);
  char* b = (char*)base;
  Geom g;
  g.plan = (gr_plan*)(b + off[4]);
  g.rec = (float4*)(b + off[0]);
  g.zr = (float*)(g.rec + (size_t)REC4 * ((size_t)n + 1));
  g.rect = (int4*)(b + off[1]);
  g.counts = (unsigned long long*)(b + off[2]);
  g.offsets = (unsigned long long*)(b + off[3]);
  g.total = (unsigned long long*)(b + off[4] + sizeof(gr_plan));
  g.omax = (float*)(g.total + (size_t)n / 256 + 2);
  g.f16_sa = (int*)(g.omax + (size_t)n / 256 + 2);
  g.scan_tmp = b + fixed;
  g.scan_tmp_bytes = 0;
  return g;
}

// ------------------------------------------------------------------------------------------------
// Bins buffer layout.
// ------------------------------------------------------------------------------------------------
#ifndef GR_CH
#define GR_CH 2048
#endif
constexpr int CH = GR_CH;  // Gaussians per raster work item (one chunk of one tile's list)
// 32-pixel tiles (gr_view.tile = 32): four times the pixels per pair, so a quarter... of the pairs per item would keep
// the item's work; fewer, longer items keep the split tiles' partial sums (4 x 1024 floats per item) small.
#ifndef GR_CH32
#define GR_CH32 2048
#endif
constexpr int CH32 = GR_CH32;
constexpr int NPART = 9;  // backward partial sums per (Gaussian, tile) pair

// Virtual tiles up to which the pairs are grouped by the stable counting sort (16-bit keys; see
// "Pair order by tile" below); past it, a radix sort.
constexpr int TSORT_MAX_TILES = 16384;

inline bool short_keys(int tiles) { return tiles <= TSORT_MAX_TILES; }

// Persistent binning state (kept from forward to backward).
struct Bins {
  uint32_t* keys;      // [K] sorted tile keys (radix-sort path only; the counting sort needs none)
  int* pairs;          // [K] Gaussian id of each sorted pair (its emission index: pos_of's inverse)
  int2* ranges;        // [vtiles] pair range of each virtual tile
  int4* items;         // [cap] work items (tile, k0, k1, chunk)
  int* num_items;      // [2]: all work items, the non-empty ones (listed first; an empty tile's item comes after them)
  int* tile_item0;     // [tiles] first work item of each tile
  int* pos_of;         // [K] sorted position of each pair, by emission index (k_reduce_bwd's map)
  int* ticket;         // [tiles] arrivals of a split tile's items (k_raster_fwd_mfma), then the finished-tile fan-in's
                       // counters (arrive_last_tile); zeroed by the work-item builder, left zero by every user
};

// Forward-only scratch (freed by the caller after gr_fwd_render).
struct Scratch {
  uint32_t* keys_in;   // [K] tile key of each emitted pair (uint16_t when short_keys(tiles))
  int* ids_in;         // [K]
  float* fwd_part;     // [cap][5][256] partial accumulators of tiles split over several items
  int2* pairs_in;      // [K] (radix path) unsorted (id, emission index) pairs
  int2* pairs_sorted;  // [K] (radix path) the same, sorted by virtual tile
  void* sort_tmp;
};

inline int64_t item_cap(int tiles, int64_t K, int ch = CH) { return (K + ch - 1) / ch + tiles; }
// Per tile size: the work-item length, the split-tile partial sums per item (forward channels x pixels) and the
// backward's upstream fragments per tile.
constexpr int UF32_FRAGS = 2 * 4 * 2 * 2 * 64;  // uint4 per 32-pixel tile: (side, channel, K-step, piece) x 64 lanes
constexpr int UF32_STRIDE = UF32_FRAGS + 64;  // + one chunk: the tile's four f16 operand exponents (an int4 at its start)
struct TileCfg {
  int T, ch;
  size_t part_floats, uf_frags;
};
constexpr int UF_FRAGS16 = 2 * 3 * 3 * 64;  // (= UF_FRAGS below)
// Work-item length: gr_view.chunk when set (a view with few tiles gets more, shorter items to fill the CUs: one
// workgroup per item), else the tile size's default; a multiple of 64 in [64, 8192].
// Unset (0), a view with K pairs (host-sized plans) gets the largest power of two <= K / 1024 within [512, default]:
// at least ~1024 items (four per CU) when the pairs allow (C2 / C3: 256 tiles of ~2k pairs each, 0.93 -> 0.89 ms per
// step); large views keep the default.  (A device-sized view's plan holds capacities: its rule reads them, so it
// matches the host-sized view's item length unless the two fall on either side of a power of two.)
static int64_t tune_env(const char* name);
inline int chunk_of(const gr_view* v, int base, int64_t K) {
  static const int64_t force = tune_env("GR_TUNE_CHUNK");
  int64_t c = base;
  if (v->chunk > 0) {
    c = v->chunk;
  } else if (force > 0) {
    c = force;
  } else if (K >= 0) {
    c = 512;
    while (c < base && 2 * c * 1024 <= K) c *= 2;
  }
  return (int)std::min<int64_t>(8192, std::max<int64_t>(64, (c + 63) / 64 * 64));
}
// K: the plan's pair count (the work-item length follows it, chunk_of); -1 where only the tile geometry is needed
inline TileCfg tile_cfg(const gr_view* v, int64_t K = -1) {
  return tile_of(v) == T32 ? TileCfg{T32, chunk_of(v, CH32, K), (size_t)4 * TP32, (size_t)UF32_STRIDE}
                           : TileCfg{T, chunk_of(v, CH, K), (size_t)5 * TP, (size_t)UF_FRAGS16};
}

// `vtiles` = 2 x tiles (core and tail lists of each tile) on the differentiable path.
// The finished-tile fan-in's counters behind the per-tile tickets (arrive_last_tile): eight shards and a top counter,
// each on a 128-byte line of its own.
constexpr int FAN_STRIDE = 32;
__host__ __device__ inline size_t fan_offset(int tiles) { return ((size_t)tiles + 1 + FAN_STRIDE - 1) / FAN_STRIDE * FAN_STRIDE; }

size_t bins_fixed(int vtiles, int64_t K, size_t off[8], int ch = CH) {
  const int tiles = vtiles;
  const size_t kk = (size_t)(K > 0 ? K : 1);
  const size_t cap = (size_t)item_cap(tiles, K, ch);
  size_t o = 0;
  off[0] = o; o = align_up(o + (short_keys(tiles) ? 1 : kk) * sizeof(uint32_t));
  off[1] = o; o = align_up(o + kk * sizeof(int));
  off[2] = o; o = align_up(o + (size_t)tiles * sizeof(int2));
  off[3] = o; o = align_up(o + cap * sizeof(int4));
  off[4] = o; o = align_up(o + 2 * sizeof(int));
  off[5] = o; o = align_up(o + (size_t)tiles * sizeof(int));
  off[6] = o; o = align_up(o + kk * sizeof(int));
  off[7] = o; o = align_up(o + (fan_offset(tiles / 2) + 9 * FAN_STRIDE) * sizeof(int));
  return o;
}

// off: [0] emitted keys, [1] emitted ids, [2] split-tile partials, [3] / [4] (radix path) unsorted /
// sorted pairs
size_t scratch_fixed(int vtiles, int64_t K, size_t off[5], int ch = CH, size_t part_floats = (size_t)5 * TP) {
  const int tiles = vtiles;
  const size_t kk = (size_t)(K > 0 ? K : 1);
  const size_t cap = (size_t)item_cap(tiles, K, ch);
  size_t o = 0;
  off[0] = o; o = align_up(o + kk * sizeof(uint32_t));
  off[1] = o; o = align_up(o + kk * sizeof(int));
  off[2] = o; o = align_up(o + cap * part_floats * sizeof(float));
  off[3] = o; o = align_up(o + (short_keys(tiles) ? 1 : kk) * sizeof(int2));
  off[4] = o; o = align_up(o + (short_keys(tiles) ? 1 : kk) * sizeof(int2));
  return o;
}

// Pair order by tile.  Pairs leave the emission in Gaussian order; the forward and backward need them
// grouped by tile with ascending Gaussian ids inside a tile (a stable sort by tile).  Up to
// TSORT_MAX_TILES tiles this is a stable counting sort over 16-bit tile keys (k_emit_count, k_tile_colscan,
// k_tile_place below): the keys are read twice and the ids once, instead of a radix sort's
// histogram + two scatter passes over keys and values.  Larger images use the hipcub radix sort on
// 32-bit keys.

// Waves per k_tile_place block: the per-wave tile cursors (tiles ints per wave) and the block's static LDS within
// 64 KiB (four waves up to 4,000 tiles: an 800x800 view's 2,500 take 40 KB, so three to four blocks share a CU with
// the other render streams' splat blocks; a block of 8 waves and 80 KB waited behind them up to 3x its standalone
// time, profiles/r04p_*); beyond 16,256 tiles one wave, whose cursors take up to 128 KiB.
// GR_TUNE_PLACE_WAVES / GR_TUNE_COL_TARGET (environment, read once): tuning overrides for tools/bin_bench.py.
static int64_t tune_env(const char* name) {
  const char* e = std::getenv(name);
  return e ? std::atoll(e) : 0;
}
inline int tsort_waves(int tiles) {
  static const int64_t force = tune_env("GR_TUNE_PLACE_WAVES");
  const int64_t per_wave = 4ll * tiles, budget = 65536 - 512;
  const int w = 4 * per_wave <= budget ? 4 : 2 * per_wave <= budget ? 2 : 1;
  if (force == 8 && 8 * per_wave <= 81920 - 512) return 8;
  return force == 1 || force == 2 || force == 4 ? std::min<int>(w, (int)force) : w;
}

#ifndef GR_TS_SEG
#define GR_TS_SEG 24
#endif
constexpr int TS_SEG = GR_TS_SEG;  // 64-pair steps per register-resident segment (1536 pairs per wave;
                                   // 16 and 32 (2048) were slower, two segments per wave much slower)

// Columns of the counting sort: each region's pairs (emission order) cut into columns of cw consecutive pairs, one
// k_tile_place block per column and one register segment (64 TS_SEG pairs) per wave: every block and wave gets the
// same work whatever the scene.  cw doubles (several segments per wave) while the count matrix (tiles x columns
// ints, zeroed, counted into, scanned and read) would outweigh half the keys and columns remain to spare (many
// tiles: 1080p).  The per-column tile counts come from the emission (k_emit_count), not from a pass of their own.
inline int col_width(int64_t K, int tiles) {
  static const int64_t force = tune_env("GR_TUNE_COL_TARGET");
  const int waves = tsort_waves(tiles);
  if (force > 0) return (int)((force + 64 * waves - 1) / (64 * waves) * (64 * waves));
  const int64_t kk = K > 0 ? K : 1;
  int64_t pw = 64ll * TS_SEG;
  auto cols_of = [&](int64_t w) { return (kk + w * waves - 1) / (w * waves); };
  while ((int64_t)tiles * cols_of(pw) > (1ll << 28) || ((int64_t)tiles * cols_of(pw) > kk / 2 && cols_of(2 * pw) >= 1024))
    pw *= 2;
  return (int)(pw * waves);
}
inline int cols_of(int64_t Kz, int cw) { return (int)((Kz + cw - 1) / cw); }

// Scratch behind the fixed part: counting sort = per region its count matrix M, its column scan S and its tile
// totals T (`tiles` = virtual tiles, 2 x screen tiles); radix sort = its temp storage.
size_t tile_sort_tmp_bytes(int n, int64_t K, int tiles) {
  if (short_keys(tiles)) {
    // per region its M, S (columns x tiles) and T (tiles); each region has at most K pairs
    const int st = tiles / 2;
    const size_t cells = (size_t)st * cols_of(K > 0 ? K : 1, col_width(K, st));
    (void)n;
    return 4 * align_up(cells * sizeof(int)) + 2 * align_up((size_t)st * sizeof(int));
  }
  size_t tmp = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, (const uint32_t*)nullptr, (uint32_t*)nullptr, (const int2*)nullptr,
                                           (int2*)nullptr, (int)(K > 0 ? K : 1), 0, bits_for((uint32_t)tiles),
                                           (hipStream_t)0);
  return tmp;
}

template <typename KeyT>
size_t sort_tmp_bytes(int64_t K, int bits) {
  size_t tmp = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, (KeyT*)nullptr, (KeyT*)nullptr, (int*)nullptr, (int*)nullptr,
                                     (int)(K > 0 ? K : 1), 0, bits, (hipStream_t)0);
  return tmp;
}

Bins bins_view(void* base, int tiles, int64_t K, int ch = CH) {
  size_t off[8];
  bins_fixed(tiles, K, off, ch);
  char* b = (char*)base;
  Bins r;
  r.keys = (uint32_t*)(b + off[0]);
  r.pairs = (int*)(b + off[1]);
  r.ranges = (int2*)(b + off[2]);
  r.items = (int4*)(b + off[3]);
  r.num_items = (int*)(b + off[4]);
  r.tile_item0 = (int*)(b + off[5]);
  r.pos_of = (int*)(b + off[6]);
  r.ticket = (int*)(b + off[7]);
  return r;
}

Scratch scratch_view(void* base, int tiles, int64_t K, int ch = CH, size_t part_floats = (size_t)5 * TP) {
  size_t off[5];
  const size_t fixed = scratch_fixed(tiles, K, off, ch, part_floats);
  char* b = (char*)base;
  Scratch r;
  r.keys_in = (uint32_t*)(b + off[0]);
  r.ids_in = (int*)(b + off[1]);
  r.fwd_part = (float*)(b + off[2]);
  r.pairs_in = (int2*)(b + off[3]);
  r.pairs_sorted = (int2*)(b + off[4]);
  r.sort_tmp = b + fixed;
  return r;
}

// ------------------------------------------------------------------------------------------------
// Kernels: binning.
// ------------------------------------------------------------------------------------------------
// Exclusive scan of one value per thread over a block of NW waves (wave shuffles, then the wave totals
// through LDS); `total` = the block's sum.
template <int NW>
__device__ __forceinline__ unsigned long long block_exclusive_scan(unsigned long long x, unsigned long long* sh,
                                                                   unsigned long long& total) {
  const int lane = (int)threadIdx.x & 63, w = (int)threadIdx.x >> 6;
  unsigned long long inc = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long y = __shfl_up(inc, o);
    if (lane >= o) inc += y;
  }
  __syncthreads();  // sh may still be read by a previous call
  if (lane == 63) sh[w] = inc;
  __syncthreads();
  unsigned long long base = 0, all = 0;
#pragma unroll
  for (int u = 0; u < NW; ++u) {
    base += u < w ? sh[u] : 0ull;
    all += sh[u];
  }
  total = all;
  return base + inc - x;
}

template <int CD>
__device__ __forceinline__ unsigned long long preprocess_one(const ViewK& v, int i, const float* __restrict__ means,
                                                             const float* __restrict__ scales,
                                                             const float* __restrict__ colors,
                                                             const float* __restrict__ opac, Geom& g);

template <int CD>
__global__ __launch_bounds__(256) void k_preprocess(ViewK v, int n, const float* __restrict__ means,
                                                    const float* __restrict__ scales, const float* __restrict__ colors,
                                                    const float* __restrict__ opac, Geom g) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == n) {
    g.counts[n] = 0ull;
    float4* pad = g.rec + (size_t)REC4 * n;  // padding record of the raster batches (rec_of)
    pad[0] = make_float4(1e30f, 1e30f, -1.0f, -1.0f);
    pad[1] = make_float4(0.f, 0.f, 0.f, 0.f);
    g.zr[n] = 0.0f;
  }
  unsigned long long kept = 0;
  if (i < n) kept = preprocess_one<CD>(v, i, means, scales, colors, opac, g);
  // the largest opacity of a kept Gaussian (the f16 forward's operand range, f16_sa_of)
  // (times max(1, z): the depth channel's operand o z ex)
  float om = kept != 0 ? g.rec[(size_t)REC4 * i + 1].x * fmaxf(1.0f, g.zr[i]) : 0.0f;
  // the block's packed pair counts (core | tail << 32; a block's counts cannot carry): k_plan scans the
  // blocks, k_offsets the Gaussians inside each block
  __shared__ unsigned long long wsum[4];
  __shared__ float wmax[4];
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) {
    kept += __shfl_xor(kept, m);
    om = fmaxf(om, __shfl_xor(om, m));
  }
  if ((threadIdx.x & 63) == 0) {
    wsum[threadIdx.x >> 6] = kept;
    wmax[threadIdx.x >> 6] = om;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    g.total[blockIdx.x] = (wsum[0] + wsum[1]) + (wsum[2] + wsum[3]);
    g.omax[blockIdx.x] = fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3]));
  }
}

// One Gaussian in one view from its loaded parameters (k_preprocess, k_preprocess_views).
template <int CD>
__device__ __forceinline__ unsigned long long preprocess_vals(const ViewK& v, int i, float mx, float my, float mz, float s0,
                                                              float s1, const float* __restrict__ col, float op,
                                                              const Geom& g) {
  Proj p;
  project(v, mx, my, mz, s0, s1, p);
  float c[3];
  eval_color<CD>(v, mx, my, mz, col, c);
  int4 r;
  const float qx = qcoef(p.sx);
  const float qy = qcoef(p.sy);
  int core = 0, tail = 0;
  const int area = tile_rect(v, p, op, r);
  if (area > 0) {
    const float thr_cut = radius_thr(v.cutoff), thr_core = radius_thr(v.core);
    for (int ty = r.y; ty <= r.w; ++ty) {
      const float ey = tile_ey(v, p.py, qy, ty);
      for (int tx = r.x; tx <= r.z; ++tx) {
        const int cls = tile_class_e(tile_ex(v, p.px, qx, tx) + ey, thr_cut, thr_core);
        core += cls == 2;
        tail += cls == 1;
      }
    }
  }
  float4* rec = g.rec + (size_t)REC4 * i;
  rec[0] = make_float4(p.px, p.py, qx, qy);
  rec[1] = make_float4(op < 0.0f ? 0.0f : op, clamp01(c[0]), clamp01(c[1]), clamp01(c[2]));
  g.zr[i] = p.za;
  g.rect[i] = r;
  g.counts[i] = (unsigned long long)core | ((unsigned long long)tail << 32);
  return (unsigned long long)core | ((unsigned long long)tail << 32);
}

template <int CD>
__device__ __forceinline__ unsigned long long preprocess_one(const ViewK& v, int i, const float* __restrict__ means,
                                                             const float* __restrict__ scales,
                                                             const float* __restrict__ colors,
                                                             const float* __restrict__ opac, Geom& g) {
  return preprocess_vals<CD>(v, i, means[3 * i], means[3 * i + 1], means[3 * i + 2], scales[3 * i], scales[3 * i + 1],
                             colors + (size_t)CD * i, opac[i], g);
}

// Several views of the same Gaussians (gr_fwd_prepare_views_async): each thread loads its Gaussian's
// parameters once and runs the per-view preprocess for every view of the batch (the same float sequence as
// k_preprocess, view by view); per view the block's packed pair counts go to that view's totals.
constexpr int PREP_MAX_VIEWS = GR_PREPARE_MAX_VIEWS;
struct PrepBatch {
  int nv;
  ViewK v[PREP_MAX_VIEWS];
  Geom g[PREP_MAX_VIEWS];
};

template <int CD>
__global__ __launch_bounds__(256) void k_preprocess_views(PrepBatch B, int n, const float* __restrict__ means,
                                                          const float* __restrict__ scales,
                                                          const float* __restrict__ colors,
                                                          const float* __restrict__ opac) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  float mx = 0.f, my = 0.f, mz = 0.f, s0 = 0.f, s1 = 0.f, op = 0.f;
  if (i < n) {
    mx = means[3 * i];
    my = means[3 * i + 1];
    mz = means[3 * i + 2];
    s0 = scales[3 * i];
    s1 = scales[3 * i + 1];
    op = opac[i];
  }
  __shared__ unsigned long long wsum[PREP_MAX_VIEWS][4];
  __shared__ float wmax[PREP_MAX_VIEWS][4];
  // views k = blockIdx.y, blockIdx.y + gridDim.y, ... (a grid of several view rows when few Gaussians fill it)
  for (int k = blockIdx.y; k < B.nv; k += gridDim.y) {
    const Geom& g = B.g[k];
    if (i == n) {
      g.counts[n] = 0ull;
      float4* pad = g.rec + (size_t)REC4 * n;
      pad[0] = make_float4(1e30f, 1e30f, -1.0f, -1.0f);
      pad[1] = make_float4(0.f, 0.f, 0.f, 0.f);
      g.zr[n] = 0.0f;
    }
    unsigned long long kept = 0;
    if (i < n) kept = preprocess_vals<CD>(B.v[k], i, mx, my, mz, s0, s1, colors + (size_t)CD * i, op, g);
    float om = kept != 0 ? fmaxf(op, 0.0f) * fmaxf(1.0f, g.zr[i]) : 0.0f;  // as k_preprocess
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) {
      kept += __shfl_xor(kept, m);
      om = fmaxf(om, __shfl_xor(om, m));
    }
    if ((threadIdx.x & 63) == 0) {
      wsum[k][threadIdx.x >> 6] = kept;
      wmax[k][threadIdx.x >> 6] = om;
    }
  }
  __syncthreads();
  if ((int)threadIdx.x < B.nv && (int)threadIdx.x % (int)gridDim.y == (int)blockIdx.y) {
    const int k = threadIdx.x;
    B.g[k].total[blockIdx.x] = (wsum[k][0] + wsum[k][1]) + (wsum[k][2] + wsum[k][3]);
    B.g[k].omax[blockIdx.x] = fmaxf(fmaxf(wmax[k][0], wmax[k][1]), fmaxf(wmax[k][2], wmax[k][3]));
  }
}

constexpr int EWIN = 4096;  // pairs staged in LDS per emit block

// Pairs of 256 consecutive Gaussians form one contiguous range; they are built in LDS and written
// out with coalesced stores (direct scattered stores only when a block overflows the window).
// Legacy (uint8) path: every tile of the rectangle, one contiguous pair range per Gaussian.
template <typename KeyT, typename OffT>
__global__ __launch_bounds__(256) void k_emit(ViewK v, int n, const int4* __restrict__ rect,
                                              const OffT* __restrict__ counts, const OffT* __restrict__ offsets,
                                              const KeyT* __restrict__ low_keys, KeyT* keys, int* ids) {
  __shared__ KeyT sK[EWIN];
  __shared__ int sI[EWIN];
  const int g0 = blockIdx.x * 256;
  const int i = g0 + (int)threadIdx.x;
  const int gend = min(n, g0 + 256);
  const int k0 = (int)(offsets[g0] & 0xffffffffu), k1 = (int)(offsets[gend] & 0xffffffffu);
  const bool staged = (k1 - k0) <= EWIN;
  if (i < n && counts[i] != 0) {
    const int4 r = rect[i];
    int k = (int)(offsets[i] & 0xffffffffu);  // pair index (low word when packed)
    const KeyT low = low_keys ? low_keys[i] : (KeyT)0;
    for (int ty = r.y; ty <= r.w; ++ty)
      for (int tx = r.x; tx <= r.z; ++tx) {
        const KeyT t = (KeyT)(ty * v.tiles_x + tx);
        KeyT key;
        if constexpr (sizeof(KeyT) == 8)
          key = (t << 32) | low;
        else
          key = t;
        if (staged) {
          sK[k - k0] = key;
          sI[k - k0] = i;
        } else {
          keys[k] = key;
          ids[k] = i;
        }
        ++k;
      }
  }
  if (!staged) return;  // uniform per block
  __syncthreads();
  for (int e = (int)threadIdx.x; e < k1 - k0; e += 256) {
    keys[k0 + e] = sK[e];
    ids[k0 + e] = sI[e];
  }
}

// Differentiable path: pairs of the kept tiles (tile_class), core pairs at [0, Kc) and tail pairs at
// [Kc, K), each in Gaussian order (the index here is the pair's partial-sum slot).  Keys: the tile (VKEY = false: each region is counting-sorted on its own) or the virtual
// tile 2*tile + tail (VKEY = true: one radix sort of the whole array).  The pairs of 256 consecutive
// Gaussians are built in LDS and written out with coalesced stores.
template <typename KeyT, bool VKEY>
__global__ __launch_bounds__(256) void k_emit_zones(ViewK v, int n, const int4* __restrict__ rect,
                                                    const Cnt2* __restrict__ counts, const Cnt2* __restrict__ offsets,
                                                    const float4* __restrict__ rec, KeyT* keys, int* ids) {
  __shared__ KeyT sK[EWIN];
  __shared__ int sI[EWIN];
  const int g0 = blockIdx.x * 256;
  const int i = g0 + (int)threadIdx.x;
  const int gend = min(n, g0 + 256);
  const int Kc = (int)offsets[n].c();
  const int c0 = (int)offsets[g0].c(), c1 = (int)offsets[gend].c();
  const int t0 = (int)offsets[g0].t(), t1 = (int)offsets[gend].t();
  const int nc = c1 - c0;
  const bool staged = nc + (t1 - t0) <= EWIN;
  if (i < n && counts[i].v != 0) {
    const int4 r = rect[i];
    const float4 a = rec[(size_t)REC4 * i];
    int kc = (int)offsets[i].c(), kt = (int)offsets[i].t();
    for (int ty = r.y; ty <= r.w; ++ty)
      for (int tx = r.x; tx <= r.z; ++tx) {
        const int cls = tile_class(v, a.x, a.y, a.z, a.w, tx, ty);
        if (cls == 0) continue;
        const int t = ty * v.tiles_x + tx;
        const KeyT key = (KeyT)(VKEY ? 2 * t + (cls == 1) : t);
        const int e = cls == 2 ? kc++ - c0 : nc + (kt++ - t0);  // index in the block's window
        if (staged) {
          sK[e] = key;
          sI[e] = i;
        } else {
          const int k = e < nc ? c0 + e : Kc + t0 + (e - nc);
          keys[k] = key;
          ids[k] = i;
        }
      }
  }
  if (!staged) return;  // uniform per block
  __syncthreads();
  const int ne = nc + (t1 - t0);
  for (int e = (int)threadIdx.x; e < ne; e += 256) {
    const int k = e < nc ? c0 + e : Kc + t0 + (e - nc);
    keys[k] = sK[e];
    ids[k] = sI[e];
  }
}

// Differentiable path, counting-sort views: one block per 256 consecutive Gaussians (k_preprocess's blocks, one per
// thread).  The block
//   - scans its Gaussians' packed pair counts (core | tail << 32) on top of the block's offset (k_plan's exclusive
//     scan of the block totals) and writes every Gaussian's offsets (the gather and the reductions read them): no
//     separate offsets pass;
//   - emits its pairs, core pairs at [0, Kc) and tail pairs at [Kc, K), each in Gaussian order with the tiles in
//     raster order (a pair's index is its partial-sum slot), staged in an LDS window and written with coalesced
//     stores (direct scattered stores when the block overflows the window: about 8 pairs per Gaussian at C4, 2k per
//     block).
// (Counting the pairs per column here as well, in an LDS histogram flushed with atomics, doubled the kernel's VALU
// work and bank conflicts and cost more than the counting pass it saved: profiles/r04r_pmc_bin.txt.)
// Block 0 also zeroes the finished-tile fan-in's counters (`fan`), which the column scan's fan-in uses first.
// ---- Batched launches (gr_fit_views_batched) -----------------------------------------------------------------------
// A kernel's blocks for several views of the same image size in ONE launch: block b belongs to the view whose block
// range [first[v], first[v + 1]) holds it and runs exactly as block b - first[v] of that view's own launch (a per-view
// grid of gx x (count / gx) blocks), with that view's arguments.  Small views (C2, C3: ~300 work items per splat, a
// few hundred blocks per binning kernel) leave most CUs idle per launch; eight views per launch fill them.  The kernel
// bodies take blockIdx / gridDim as parameters (shadowing the builtins), so the single-view launch is the same code.
constexpr int GR_BATCH_MAX = 8;
struct BI {
  int x, y;
};
template <class A>
struct VBatch {
  int nv;
  int first[GR_BATCH_MAX + 1];
  int gx[GR_BATCH_MAX];
  A a[GR_BATCH_MAX];
};
template <class A>
__device__ __forceinline__ int vbatch_view(const VBatch<A>& B, int b) {
  int v = 0;
  while (v + 1 < B.nv && b >= B.first[v + 1]) ++v;
  return v;
}

constexpr int EWIN_BLK = 4096;  // pairs staged in LDS per block
__device__ __forceinline__ void k_emit_offsets_body(ViewK v, int n, const int4* __restrict__ rect, const Cnt2* __restrict__ counts,
                                                      const unsigned long long* __restrict__ bsum, Cnt2* __restrict__ offsets,
                                                      const float4* __restrict__ rec, uint16_t* __restrict__ keys,
                                                      int* __restrict__ ids, int* __restrict__ fan, const BI blockIdx, const BI gridDim) {
  __shared__ int sI[EWIN_BLK];
  __shared__ uint16_t sK[EWIN_BLK];
  __shared__ unsigned long long wsum[4];
  const int tid = threadIdx.x, b = blockIdx.x, i = b * 256 + tid;
  if (b == 0 && tid < 9) fan[FAN_STRIDE * tid] = 0;
  if (offsets[n].v == 0ull) {  // no pair (a view over its capacity, gr_fwd_prepare_views_sized): every offset is zero
    if (i < n) offsets[i].v = 0ull;
    return;
  }
  const Cnt2 cn{i < n ? counts[i].v : 0ull};
  // every load the block needs issued before the scan's barriers (their latencies overlap instead of adding up)
  const Cnt2 cb{bsum[b]};
  const int Kc = (int)offsets[n].c();
  const int4 rc = i < n ? rect[i] : make_int4(0, 0, -1, -1);
  const float4 a = i < n ? rec[(size_t)REC4 * i] : make_float4(0.f, 0.f, 0.f, 0.f);
  unsigned long long tot;
  const unsigned long long ex = block_exclusive_scan<4>(cn.v, wsum, tot);
  const int c0 = (int)cb.c(), t0 = (int)cb.t();  // the block's first core pair, first tail pair (after Kc)
  const int nc = (int)(tot & 0xffffffffull), nt = (int)(tot >> 32);
  const bool staged = nc + nt <= EWIN_BLK;       // uniform per block
  const unsigned long long run = cb.v + ex;
  if (i < n) offsets[i].v = run;
  if (cn.v != 0) {
    int kc = (int)(run & 0xffffffffull), kt = (int)(run >> 32);
    const float thr_cut = radius_thr(v.cutoff), thr_core = radius_thr(v.core);
    for (int ty = rc.y; ty <= rc.w; ++ty) {
      const float ey = tile_ey(v, a.y, a.w, ty);
      for (int tx = rc.x; tx <= rc.z; ++tx) {
        const int cls = tile_class_e(tile_ex(v, a.x, a.z, tx) + ey, thr_cut, thr_core);
        if (cls == 0) continue;
        const int t = ty * v.tiles_x + tx;
        const int e = cls == 2 ? kc++ - c0 : nc + (kt++ - t0);  // index in the block's window
        if (staged) {
          sK[e] = (uint16_t)t;
          sI[e] = i;
        } else {
          const int k = e < nc ? c0 + e : Kc + t0 + (e - nc);
          keys[k] = (uint16_t)t;
          ids[k] = i;
        }
      }
    }
  }
  if (!staged) return;  // uniform per block
  __syncthreads();
  for (int e = tid; e < nc + nt; e += 256) {
    const int k = e < nc ? c0 + e : Kc + t0 + (e - nc);
    keys[k] = sK[e];
    ids[k] = sI[e];
  }
}
__global__ __launch_bounds__(256) void k_emit_offsets(ViewK v, int n, const int4* __restrict__ rect, const Cnt2* __restrict__ counts,
                                                      const unsigned long long* __restrict__ bsum, Cnt2* __restrict__ offsets,
                                                      const float4* __restrict__ rec, uint16_t* __restrict__ keys,
                                                      int* __restrict__ ids, int* __restrict__ fan) {
  k_emit_offsets_body(v, n, rect, counts, bsum, offsets, rec, keys, ids, fan, BI{(int)blockIdx.x, (int)blockIdx.y}, BI{(int)gridDim.x, (int)gridDim.y});
}
struct k_emit_offsets_args {
  ViewK v;
  int n;
  const int4* rect;
  const Cnt2* counts;
  const unsigned long long* bsum;
  Cnt2* offsets;
  const float4* rec;
  uint16_t* keys;
  int* ids;
  int* fan;
};
__global__ __launch_bounds__(256) void k_emit_offsets_views(VBatch<k_emit_offsets_args> B) {
  const int vb = vbatch_view(B, (int)blockIdx.x);
  const k_emit_offsets_args& a = B.a[vb];
  const int lb = (int)blockIdx.x - B.first[vb], gx = B.gx[vb];
  k_emit_offsets_body(a.v, a.n, a.rect, a.counts, a.bsum, a.offsets, a.rec, a.keys, a.ids, a.fan, BI{lb % gx, lb / gx}, BI{gx, (B.first[vb + 1] - B.first[vb]) / gx});
}


// Radix-sort path: the sorted (id, emission index) values -> the Gaussian ids and the sorted position of
// each pair by emission index (the counting sort writes both in k_tile_place).
__global__ __launch_bounds__(256) void k_pos_of(int64_t K, const int2* __restrict__ sorted, int* __restrict__ ids,
                                                int* __restrict__ pos_of) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K) return;
  const int2 p = sorted[k];
  ids[k] = p.x;
  pos_of[p.y] = (int)k;
}

// Radix-sort path: the sort's values, (gaussian id, emission index).
__global__ __launch_bounds__(256) void k_pair_values(int64_t K, const int* __restrict__ ids, int2* __restrict__ pairs) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < K) pairs[k] = make_int2(ids[k], (int)k);
}

template <typename KeyT>
__global__ __launch_bounds__(256) void k_ranges(int64_t K, const KeyT* __restrict__ keys, int2* ranges) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K) return;
  const int shift = sizeof(KeyT) == 8 ? 32 : 0;
  const int t = (int)(keys[k] >> shift);
  if (k == 0 || (int)(keys[k - 1] >> shift) != t) ranges[t].x = (int)k;
  if (k == K - 1 || (int)(keys[k + 1] >> shift) != t) ranges[t].y = (int)(k + 1);
}

// ------------------------------------------------------------------------------------------------
// MFMA formulation.  With axis-aligned footprints the weight is separable,
//   w_g(x,y) = o_g * ex_g(x) * ey_g(y),  ex_g(x) = 2^(qx (x+.5-px)^2),  ey_g(y) likewise,
// so the per-tile splat is a dense contraction over the tile's Gaussians g:
//   forward   C_k[x][y] = sum_g (o_g v_gk ex_g(x)) * ey_g(y),  v = (1, r, g, b, z)
//   backward  D_k,f[y][g] = sum_x U_k[x][y] * (f(x) ex_g(x)),  f in {1, dx, dx^2}
// evaluated on bf16 MFMA with exactly split operands (k_raster_fwd_mfma, k_raster_bwd_bf16).
// ------------------------------------------------------------------------------------------------
typedef float f32x4 __attribute__((ext_vector_type(4)));

// Work items: each non-empty (virtual) tile's pair list is cut into chunks of CH Gaussians, so every
// workgroup gets about the same amount of work however unevenly Gaussians fall on tiles; a tile with no pair in
// either zone gets one empty item (its pixels are background: the forward writes them, and their loss terms).
// Items are ordered by (virtual tile, chunk), so the core and tail items of a tile are adjacent.  The builders
// also zero the forward's arrival tickets (Bins::ticket).  k_work_items reads existing per-virtual-tile ranges
// (radix-sort path, empty views); the counting sort's k_tile_place cuts them from the tile totals
// (work_items_zones).
// One workgroup of WI_THREADS (256: it fits beside the splat kernels on a partly occupied CU; a
// 1024-thread block waits for a whole CU to drain, which under four render streams took up to 1.6 ms).
#ifndef GR_WI_THREADS
#define GR_WI_THREADS 256
#endif
constexpr int WI_THREADS = GR_WI_THREADS;
__device__ __forceinline__ int chunks_of(int len, int ch) { return (len + ch - 1) / ch; }
__global__ __launch_bounds__(WI_THREADS) void k_work_items(int vtiles, const int2* __restrict__ ranges, int4* __restrict__ items,
                                                     int* __restrict__ num_items, int* __restrict__ tile_item0,
                                                     int* __restrict__ ticket, int ch) {
  typedef hipcub::BlockScan<int, WI_THREADS> Scan;
  __shared__ typename Scan::TempStorage tmp;
  __shared__ int carry;
  const int tiles = vtiles / 2;
  // pass 0: the non-empty tiles' items, in tile order; pass 1: one empty item per empty tile, after all of them
  for (int pass = 0; pass < 2; ++pass) {
    if (threadIdx.x == 0 && pass == 0) carry = 0;
    __syncthreads();
    for (int base = 0; base < tiles; base += WI_THREADS) {
      const int t = base + (int)threadIdx.x;
      const int2 rc = t < tiles ? ranges[2 * t] : make_int2(0, 0), rt = t < tiles ? ranges[2 * t + 1] : make_int2(0, 0);
      const int chc = chunks_of(rc.y - rc.x, ch), cht = chunks_of(rt.y - rt.x, ch);
      const int nch = t >= tiles ? 0 : pass == 0 ? chc + cht : (chc + cht == 0 ? 1 : 0);
      int excl, total;
      Scan(tmp).ExclusiveSum(nch, excl, total);
      const int first = carry + excl;
      if (t < tiles && pass == 0) {
        ticket[t] = 0;
        tile_item0[2 * t] = first;
        tile_item0[2 * t + 1] = first + chc;
        for (int c = 0; c < chc; ++c) items[first + c] = make_int4(2 * t, rc.x + c * ch, min(rc.y, rc.x + (c + 1) * ch), c);
        for (int c = 0; c < cht; ++c)
          items[first + chc + c] = make_int4(2 * t + 1, rt.x + c * ch, min(rt.y, rt.x + (c + 1) * ch), c);
      } else if (nch) {
        tile_item0[2 * t] = tile_item0[2 * t + 1] = first;
        items[first] = make_int4(2 * t, 0, 0, 0);
      }
      __syncthreads();
      if (threadIdx.x == 0) carry += total;
      __syncthreads();
    }
    if (threadIdx.x == 0) num_items[1 - pass] = carry;  // (pass 0: the non-empty count; pass 1: all)
  }
  if (threadIdx.x < 9) ticket[fan_offset(tiles) + FAN_STRIDE * threadIdx.x] = 0;
}

// Staging pipeline for the 256-wide Gaussian batches of a work item: the records of batch b+1 are
// copied global -> LDS by LDS-DMA (global_load_lds, no VGPR destination) while batch b is computed,
// and the Gaussian ids of batch b+2 are in flight in a register, so neither the id load nor the
// dependent record gathers sit on the critical path.  The __syncthreads() at the top of each batch
// waits for this wave's DMA (vmcnt(0)) and, as a barrier, for every other wave's.
// Unconditional load (index clamped into the item, k1 > k0); the padding select (k >= k1) is made
// only when the pair is consumed, a batch later (stage_pair): selecting here lets the compiler turn
// the load into a predicated one, and the join after it waits for every outstanding memory
// operation, the in-flight DMA included.
__device__ __forceinline__ int stage_id(int k, int k1, const int* __restrict__ pairs) { return pairs[min(k, k1 - 1)]; }
__device__ __forceinline__ int stage_pair(int raw, int k, int k1) { return k < k1 ? raw : -1; }

typedef __attribute__((address_space(3))) void* lds_ptr_t;

// One LDS-DMA per lane: 16 (4) bytes from gsrc to wave_base + lane * 16 (4).  Issued from inline asm
// so the compiler does not track it: hipcc would otherwise wait for the DMA (vmcnt(0)) before the
// first LDS read of the batch being computed, serialising the copy with the compute.  Completion is
// awaited explicitly by stage_wait() before the barrier that publishes the buffer.
__device__ __forceinline__ uint32_t lds_addr(void* p) {
  return __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_ptr_t)p);
}
__device__ __forceinline__ void glds16(const void* gsrc, void* wave_base) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_addr(wave_base)) : "memory");
}
__device__ __forceinline__ void glds4(const void* gsrc, void* wave_base) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_addr(wave_base)) : "memory");
}
// This wave's LDS-DMAs (and every other vector memory op) have completed; follow with a barrier.
__device__ __forceinline__ void stage_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// In the splat kernels every wave stages (LDS-DMA) and reads only its own 64-Gaussian slice of a batch,
// so the wave's own vmcnt orders its reads (MI355X_MICROARCH.md item 7) and no barrier is needed
// between batches: a wave never waits for another wave's copy.
#ifdef GR_STAGE_BARRIER
#define GR_STAGE_SYNC() __syncthreads()
#else
#define GR_STAGE_SYNC() ((void)0)
#endif

// Record of Gaussian g; g < 0 (padding) reads the pad record rec[n] written by k_preprocess: o = 0
// and px = +huge, so every weight it produces is exactly 0 (exp2(-inf) = 0) without a select.
__device__ __forceinline__ const float4* rec_of(int g, int n, const float4* __restrict__ rec) {
  return rec + (size_t)REC4 * (g >= 0 ? g : n);
}
// camera depth of Gaussian g (n: padding), stored after the n+1 records
__device__ __forceinline__ const float* zrec_of(int g, int n, const float4* __restrict__ rec) {
  return reinterpret_cast<const float*>(rec + (size_t)REC4 * ((size_t)n + 1)) + (g >= 0 ? g : n);
}

// XCD-aware work-item order: the dispatcher deals workgroups round-robin over the 8 XCDs
// (MI355X_MICROARCH.md §Workgroup dispatch), so block b runs on XCD-group b % 8.  Give each XCD
// group a contiguous run of items (= neighbouring tiles, which share most Gaussians) so their
// records stay in that XCD's L2.  Bijective for any count (cdna_hip_programming.md §5 'XCD swizzle').
// Speed only: any placement gives the same results.
__device__ __forceinline__ int xcd_item(int b, int nwg) {
#if defined(GR_NO_XCD_REMAP)
  return b;
#endif
  const int q = nwg >> 3, r = nwg & 7, xcd = b & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (b >> 3);
}

// Write-through (sc1) stores and loads of data handed from one workgroup to another inside a launch, with an
// arrival ticket (MI355X_MICROARCH.md, Valid forms, first row of the hand-off table: every store and load of the
// handed-off bytes sc1; each storing wave drained, a barrier, then one lane's agent-scope atomic add; the workgroup
// whose add returns count - 1 reads after its add has returned and a barrier).
template <typename V>
__device__ __forceinline__ void st_through(V* p, V x) { __hip_atomic_store(p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
template <typename V>
__device__ __forceinline__ V ld_through(const V* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// The 16-byte form (round 6, the 32-pixel forward's split-tile partials): raw buffer stores / loads with the sc1 cache
// policy (the same write-through as the 4-byte atomics above compile to), through a buffer resource on the hand-off
// buffer; the compiler tracks them (vmcnt) like any load / store.  A quarter of the memory instructions.
constexpr int GR_CPOL_SC1 = 16;  // cache-policy immediate: sc1
__device__ __forceinline__ __amdgpu_buffer_rsrc_t through_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);  // raw, 32-bit data
}
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_through16(__amdgpu_buffer_rsrc_t r, int byte_off, float4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z),
                                                 __float_as_uint(v.w)},
                                         r, byte_off, 0, GR_CPOL_SC1);
}
__device__ __forceinline__ float4 ld_through16(__amdgpu_buffer_rsrc_t r, int byte_off) {
  const u32x4_t u = __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, GR_CPOL_SC1);
  return make_float4(__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w));
}
// Every thread of the block calls this after its write-through stores: true in the block that arrives last of
// `count` (uniform per block).  `flag`: one LDS word.
__device__ __forceinline__ bool arrive_last(int* ticket, int count, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's stores have completed
  __syncthreads();                                   // ... and every wave's
  if (threadIdx.x == 0) *flag = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == count - 1;
  __syncthreads();
  return *flag != 0;
}

// arrive_last for one arrival of each of `count` indices of a launch (a per-tile kernel's block, the block that
// finishes a split tile, a column-scan block): index i arrives on shard i & 7 of `fan` (fan_offset: eight shards and a
// top counter, each on a 128-byte line), the last arrival of each shard on the top counter.  One counter for all of
// them would serialise the ~2,500 returning atomics of an 800^2 view (one word saturates at ~88 per us,
// MI355X_MICROARCH.md fanin / dequeue: ~28 us at the end of the launch).  The counters are left zero.
__device__ __forceinline__ bool arrive_last_of(int* fan, int count, int idx, int* flag) {
  const int sh = idx & 7, nsh = count < 8 ? count : 8;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's stores have completed
  __syncthreads();                                   // ... and every wave's
  if (threadIdx.x == 0) {
    int last = 0;
    if (__hip_atomic_fetch_add(&fan[FAN_STRIDE * sh], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ((count - sh + 7) >> 3) - 1) {
      __hip_atomic_store(&fan[FAN_STRIDE * sh], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = __hip_atomic_fetch_add(&fan[FAN_STRIDE * 8], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nsh - 1;
      if (last) __hip_atomic_store(&fan[FAN_STRIDE * 8], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    *flag = last;
  }
  __syncthreads();
  return *flag != 0;
}

__device__ __forceinline__ bool arrive_last_tile(int* ticket, int tiles, int tile, int* flag) {
  return arrive_last_of(ticket + fan_offset(tiles), tiles, tile, flag);
}

// ---- Stable counting sort of the pairs by tile -------------------------------------------------
// The emitted pairs of each region (zone 0: core pairs [0, Kc), zone 1: tail pairs [Kc, K)) are cut into columns:
// column c = the region's pairs [c cw, c cw + cw) (col_width), a memset of M and three dependent launches:
//   k_emit_count    emits the pairs and counts each column's pairs per tile into M[column][tile] (zeroed before;
//                   it also writes the Gaussians' offsets);
//   k_tile_colscan  scans M over the columns of each tile (S = start of (column, tile) within the tile) and
//                   writes the tile's total T[tile];
//   k_tile_place    one block per (region, column): scans T into the tile starts itself, re-counts per wave,
//                   turns tile starts + S into per-wave cursors and walks each wave's pairs in order, 64 at a
//                   time.  Lanes holding the same tile in one step are ranked by bit-plane ballots (one ballot
//                   per key bit: the lanes agreeing with this lane on every bit), and the highest lane of each
//                   group advances the tile's cursor.  Block 0 of the launch instead cuts the per-virtual-tile
//                   ranges and work items the splats read (work_items_zones), beside the placing blocks.
// Everything is walked in pair order, so the Gaussian ids inside each tile come out ascending:
// exactly the oracle's stable sort (oracle/gr_oracle.c gro_bin), and deterministic.
constexpr int TS_RB = 9, TS_RH = 1 << (TS_RB - 1);  // relative tile keys in ts_place

struct TZone {
  int64_t K;              // pairs of the region
  int cols;               // its columns (0: an empty region)
  int zbase;              // emission index of its first pair
  const uint16_t* keys;   // its keys and ids (emission order)
  const int* ids;
  int* M;                 // its count matrix, column scan and tile totals
  int* S;
  int* T;
};
struct TZones {
  int ch;  // work-item length (pairs): CH, or CH32 for 32-pixel tiles
  TZone z[2];
  int cw;  // pairs per column (col_width)
  // device-side sizing (gr_view.device_counts): the packed true counts (core | tail << 32, the offsets' end) on the
  // device; z[*].K and cols are then the capacities (the grid), and zone_at() gives each zone's true K, first pair and
  // key / id pointers (z[0].keys / ids: the arrays' start)
  const unsigned long long* kdev;
};
__device__ __forceinline__ TZone zone_at(const TZones& Z, int zone) {
  TZone zz = Z.z[zone];
  if (Z.kdev) {
    const unsigned long long e = *Z.kdev;
    const int Kc = (int)(e & 0xffffffffull);
    zz.K = zone ? (int64_t)(e >> 32) : (int64_t)Kc;
    zz.zbase = zone ? Kc : 0;
    zz.keys = Z.z[0].keys + zz.zbase;
    zz.ids = Z.z[0].ids + zz.zbase;
  }
  return zz;
}
// Column block b of the combined grid -> (zone, column), XCD-aware within the grid.
__device__ __forceinline__ int tzone_of(const TZones& Z, int b, int& c) {
  b = xcd_item(b, Z.z[0].cols + Z.z[1].cols);
  const int zone = b < Z.z[0].cols ? 0 : 1;
  c = b - (zone ? Z.z[0].cols : 0);
  return zone;
}
// Pairs [k0, k1) of column c in a region of K pairs, relative to the region's first pair (k1 <= k0: a column past the
// region's true end under device-side sizing).
__device__ __forceinline__ void column_range(const TZones& Z, int64_t K, int c, int64_t& k0, int64_t& k1) {
  k0 = (int64_t)c * Z.cw;
  k1 = min(K, k0 + Z.cw);
}

// Per-column tile counts M[c][t]: one block per (region, column), the column's keys read once (coalesced, eight
// loads in flight per thread) into an LDS histogram.
__device__ __forceinline__ void k_tile_count_body(TZones Z, int tiles, const BI blockIdx, const BI gridDim) {
  extern __shared__ int hist[];
  int c;
  const int zone = tzone_of(Z, (int)blockIdx.x, c);
  const TZone zz = zone_at(Z, zone);
  const uint16_t* __restrict__ keys = zz.keys;
  for (int t = threadIdx.x; t < tiles; t += 256) hist[t] = 0;
  __syncthreads();
  int64_t k0, k1;
  column_range(Z, zz.K, c, k0, k1);
  for (int64_t kb = k0 + threadIdx.x; kb < k1; kb += 256 * 8) {
    int d[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) d[j] = kb + j * 256 < k1 ? (int)keys[kb + j * 256] : -1;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (d[j] >= 0) atomicAdd(&hist[d[j]], 1);
  }
  __syncthreads();
  for (int t = threadIdx.x; t < tiles; t += 256) zz.M[(size_t)c * tiles + t] = hist[t];
}
__global__ __launch_bounds__(256) void k_tile_count(TZones Z, int tiles) {
  k_tile_count_body(Z, tiles, BI{(int)blockIdx.x, (int)blockIdx.y}, BI{(int)gridDim.x, (int)gridDim.y});
}
struct k_tile_count_args {
  TZones Z;
  int tiles;
};
__global__ __launch_bounds__(256) void k_tile_count_views(VBatch<k_tile_count_args> B) {
  const int vb = vbatch_view(B, (int)blockIdx.x);
  const k_tile_count_args& a = B.a[vb];
  const int lb = (int)blockIdx.x - B.first[vb], gx = B.gx[vb];
  k_tile_count_body(a.Z, a.tiles, BI{lb % gx, lb / gx}, BI{gx, (B.first[vb + 1] - B.first[vb]) / gx});
}


// Column scan of M: S[c][t] = sum of M[c'][t] over c' < c, T[t] = the tile's total.  A block takes
// CS_T tiles x CS_G column groups; a thread's column run (up to CS_R of them) is loaded at once and kept
// in registers for the second pass, so the kernel waits on memory about twice instead of once per 8
// columns and never reads M again.
// 256 threads per block (16 tiles x 16 column groups): a 1024-thread block needs a whole CU free and
// waits behind the splat kernels of the other render streams (up to 0.9 ms per launch at C4).
#ifndef GR_CS_T
#define GR_CS_T 16
#endif
#ifndef GR_CS_THREADS
#define GR_CS_THREADS 256
#endif
#ifndef GR_CS_R
#define GR_CS_R 96
#endif
constexpr int CS_T = GR_CS_T, CS_G = GR_CS_THREADS / GR_CS_T, CS_R = GR_CS_R;

__device__ __forceinline__ void tile_colscan_block(const TZone& zz, int tiles, int bx) {
  const int cols = zz.cols;
  const int* __restrict__ M = zz.M;
  int* __restrict__ S = zz.S;
  int* __restrict__ T = zz.T;
  __shared__ int part[CS_G][CS_T + 1];
  const int tl = (int)threadIdx.x % CS_T, g = (int)threadIdx.x / CS_T;
  const int t = bx * CS_T + tl;
  const int per = (cols + CS_G - 1) / CS_G;
  const int c0 = min(cols, g * per), c1 = min(cols, c0 + per);
  const bool regs = per <= CS_R;  // uniform
  int val[CS_R];
  int sum = 0;
  if (t < tiles) {
    if (regs) {
#pragma unroll
      for (int q = 0; q < CS_R; ++q) val[q] = c0 + q < c1 ? M[(size_t)(c0 + q) * tiles + t] : 0;
#pragma unroll
      for (int q = 0; q < CS_R; ++q) sum += val[q];
    } else {
#pragma unroll 8
      for (int c = c0; c < c1; ++c) sum += M[(size_t)c * tiles + t];
    }
  }
  part[g][tl] = sum;
  __syncthreads();
  if (g == 0) {
    int run = 0;
    for (int u = 0; u < CS_G; ++u) {
      const int v = part[u][tl];
      part[u][tl] = run;
      run += v;
    }
    if (t < tiles) st_through(&T[t], run);  // read by this launch's last block (work_items_zones<true>)
  }
  __syncthreads();
  if (t < tiles) {
    int run = part[g][tl];
    if (regs) {
#pragma unroll
      for (int q = 0; q < CS_R; ++q)
        if (c0 + q < c1) {
          S[(size_t)(c0 + q) * tiles + t] = run;
          run += val[q];
        }
    } else {
#pragma unroll 8
      for (int c = c0; c < c1; ++c) {
        const int v = M[(size_t)c * tiles + t];
        S[(size_t)c * tiles + t] = run;
        run += v;
      }
    }
  }
}


template <bool THROUGH, int NT>
__device__ void work_items_zones(int tiles, int Kc, const int* __restrict__ Tc, const int* __restrict__ Tt,
                                 int2* __restrict__ ranges, int4* __restrict__ items, int* __restrict__ num_items,
                                 int* __restrict__ tile_item0, int* __restrict__ ticket, int ch);
// ... and the block that finishes last (arrive_last_of over the grid) scans the tile totals into the per-virtual-tile
// ranges and cuts the work items (work_items_zones): no launch of its own between the scan and the placement.
__device__ __forceinline__ void k_tile_colscan_body(TZones Z, int tiles, int2* __restrict__ ranges,
                                                             int4* __restrict__ items, int* __restrict__ num_items,
                                                             int* __restrict__ tile_item0, int* __restrict__ ticket, const BI blockIdx, const BI gridDim) {
  __shared__ int last;
  const TZone zz = zone_at(Z, (int)blockIdx.y);
  if (zz.K > 0) tile_colscan_block(zz, tiles, (int)blockIdx.x);  // (an empty region: no counts, and the work items get no totals for it)
  const int nb = (int)(gridDim.x * gridDim.y);
  if (!arrive_last_of(ticket + fan_offset(tiles), nb, (int)(blockIdx.y * gridDim.x + blockIdx.x), &last)) return;
  const TZone z0 = zone_at(Z, 0), z1 = zone_at(Z, 1);
  work_items_zones<true, GR_CS_THREADS>(tiles, z1.zbase, z0.K > 0 ? z0.T : nullptr, z1.K > 0 ? z1.T : nullptr,
                                  ranges, items, num_items, tile_item0, ticket, Z.ch);
}
__global__ __launch_bounds__(GR_CS_THREADS) void k_tile_colscan(TZones Z, int tiles, int2* __restrict__ ranges,
                                                             int4* __restrict__ items, int* __restrict__ num_items,
                                                             int* __restrict__ tile_item0, int* __restrict__ ticket) {
  k_tile_colscan_body(Z, tiles, ranges, items, num_items, tile_item0, ticket, BI{(int)blockIdx.x, (int)blockIdx.y}, BI{(int)gridDim.x, (int)gridDim.y});
}
struct k_tile_colscan_args {
  TZones Z;
  int tiles;
  int2* ranges;
  int4* items;
  int* num_items;
  int* tile_item0;
  int* ticket;
};
__global__ __launch_bounds__(GR_CS_THREADS) void k_tile_colscan_views(VBatch<k_tile_colscan_args> B) {
  const int vb = vbatch_view(B, (int)blockIdx.x);
  const k_tile_colscan_args& a = B.a[vb];
  const int lb = (int)blockIdx.x - B.first[vb], gx = B.gx[vb];
  k_tile_colscan_body(a.Z, a.tiles, a.ranges, a.items, a.num_items, a.tile_item0, a.ticket, BI{lb % gx, lb / gx}, BI{gx, (B.first[vb + 1] - B.first[vb]) / gx});
}



__device__ __forceinline__ void ts_load(int64_t kb, int64_t k1, int64_t klast, int lane, const uint16_t* __restrict__ keys,
                                        const int* __restrict__ ids_in, int (&d)[TS_SEG], int (&id)[TS_SEG]) {
  // branch-free: out-of-range lanes load the last pair (K >= 1) and are marked d = -1 (every column but a region's
  // last is whole)
#pragma unroll
  for (int j = 0; j < TS_SEG; ++j) {
    const int64_t k = kb + j * 64 + lane;
    const int64_t kc = k < k1 ? k : klast;
    const int key = (int)keys[kc];
    id[j] = ids_in[kc];
    d[j] = k < k1 ? key : -1;
  }
}

// One register-resident segment of k_tile_place: TS_SEG steps of 64 pairs, in pair order.
// kseg: emission index of the segment's first pair (the slot written next to the Gaussian id).
__device__ __forceinline__ void ts_place(int lane, int bits, int* my, const int (&d)[TS_SEG], const int (&id)[TS_SEG],
                                         int kseg, int* __restrict__ pairs_out, int* __restrict__ pos_of) {
  const uint64_t below = (1ull << lane) - 1ull;
#pragma unroll
  for (int j = 0; j < TS_SEG; ++j) {
    const bool ok = d[j] >= 0;
    const uint64_t live = __ballot(ok);
    if (live == 0) break;  // wave-uniform: the rest of this wave's range is past its end
    // keep the lanes whose key bit b equals this lane's: m &= ~(ballot ^ bit mask), one v_bitop3 per half
    // Usually the step's tiles lie within TS_RH of lane 0's (neighbouring Gaussians): then the keys
    // relative to it take TS_RB bits instead of `bits` (lane 0 is live whenever any lane is).
    const int rel = d[j] - __builtin_amdgcn_readfirstlane(d[j]) + TS_RH;
    const bool near = __ballot(ok && (unsigned)rel >= 2u * TS_RH) == 0;
    const int key = near ? rel : d[j];
    const int nb = near && TS_RB < bits ? TS_RB : bits;
    unsigned mlo = (unsigned)live, mhi = (unsigned)(live >> 32);
    for (int b = 0; b < nb; ++b) {
      const int bm = __builtin_amdgcn_sbfe(key, b, 1);  // 0 or -1
      const uint64_t v = __ballot(bm != 0);
      mlo &= ~((unsigned)v ^ (unsigned)bm);
      mhi &= ~((unsigned)(v >> 32) ^ (unsigned)bm);
    }
    const uint64_t m = ((uint64_t)mhi << 32) | mlo;
    if (ok) {
      const int pos = my[d[j]] + __popcll(m & below);
      pairs_out[pos] = id[j];
      pos_of[kseg + j * 64 + lane] = pos;  // emission order: coalesced
      __builtin_amdgcn_wave_barrier();  // every lane has read the cursor before it moves
      if ((m >> lane) == 1ull) my[d[j]] = pos + 1;  // highest lane of its group
    }
  }
}

// Counting-sort views: the per-tile totals of the core region (Tc) and of the tail region (Tt, starting at Kc)
// scanned into the virtual-tile ranges (2t: core, 2t+1: tail), then cut into work items of <= CH pairs.  Thread i
// owns a contiguous run of tiles: its run's totals are scanned across the block once (three block scans instead of
// three per NT tiles), then the run is walked again with running offsets.  The last block of k_tile_colscan
// (THROUGH: the totals were written in that launch, write-through).  A run's totals are loaded RUNQ at a time,
// together, and kept in registers for the second walk when the run fits (<= RUNQ tiles: 2,560 tiles at NT = 256).
constexpr int RUNQ = 10;
template <bool THROUGH, int NT>
__device__ void work_items_zones(int tiles, int Kc, const int* __restrict__ Tc, const int* __restrict__ Tt,
                                 int2* __restrict__ ranges, int4* __restrict__ items, int* __restrict__ num_items,
                                 int* __restrict__ tile_item0, int* __restrict__ ticket, int ch) {
  __shared__ unsigned long long sh[NT / 64];  // two packed 64-bit block scans
  const int per = (tiles + NT - 1) / NT;
  const int t0 = min(tiles, (int)threadIdx.x * per), t1 = min(tiles, t0 + per);
  int rc_[RUNQ], rt_[RUNQ];
  auto ld = [&](const int* T, int t) { return !T || t >= t1 ? 0 : THROUGH ? ld_through(T + t) : T[t]; };
  auto load_run = [&](int b) {
#pragma unroll
    for (int q = 0; q < RUNQ; ++q) {
      rc_[q] = ld(Tc, b + q);
      rt_[q] = ld(Tt, b + q);
    }
  };
  int sc = 0, st = 0, sch = 0, se = 0;
  for (int b = t0; b < t1; b += RUNQ) {
    load_run(b);
#pragma unroll
    for (int q = 0; q < RUNQ; ++q) {
      const int nc = rc_[q], nt = rt_[q];  // (0 past the run, and for an empty zone)
      sc += nc;
      st += nt;
      const int nch = chunks_of(nc, ch) + chunks_of(nt, ch);
      sch += nch;
      se += nch == 0 && b + q < t1;  // an empty tile: one empty item, after every non-empty one
    }
  }
  // (pair counts < 2^31 and item counts: no carry between the packed halves)
  unsigned long long t1v, t2v;
  const unsigned long long e1 = block_exclusive_scan<NT / 64>((unsigned long long)sc | ((unsigned long long)st << 32), sh, t1v);
  const unsigned long long e2 = block_exclusive_scan<NT / 64>((unsigned long long)sch | ((unsigned long long)se << 32), sh, t2v);
  sc = (int)(e1 & 0xffffffffull);
  st = (int)(e1 >> 32);
  sch = (int)(e2 & 0xffffffffull);
  se = (int)(e2 >> 32);
  const int total = (int)(t2v & 0xffffffffull), empties = (int)(t2v >> 32);
  se += total;
  for (int b = t0; b < t1; b += RUNQ) {
    if (t1 - t0 > RUNQ) load_run(b);  // (a run of at most RUNQ tiles is still in registers)
#pragma unroll
    for (int q = 0; q < RUNQ; ++q) {
      const int t = b + q;
      if (t < t1) {
        const int nc = rc_[q], nt = rt_[q];
        const int2 rc = nc > 0 ? make_int2(sc, sc + nc) : make_int2(0, 0);
        const int2 rt = nt > 0 ? make_int2(Kc + st, Kc + st + nt) : make_int2(0, 0);
        const int chc = chunks_of(nc, ch), cht = chunks_of(nt, ch);
        ranges[2 * t] = rc;
        ranges[2 * t + 1] = rt;
        tile_item0[2 * t] = sch;
        tile_item0[2 * t + 1] = sch + chc;
        ticket[t] = 0;
        for (int c = 0; c < chc; ++c) items[sch + c] = make_int4(2 * t, rc.x + c * ch, min(rc.y, rc.x + (c + 1) * ch), c);
        for (int c = 0; c < cht; ++c)
          items[sch + chc + c] = make_int4(2 * t + 1, rt.x + c * ch, min(rt.y, rt.x + (c + 1) * ch), c);
        if (chc + cht == 0) {
          tile_item0[2 * t] = tile_item0[2 * t + 1] = se;
          items[se++] = make_int4(2 * t, 0, 0, 0);
        }
        sc += nc;
        st += nt;
        sch += chc + cht;
      }
    }
  }
  if (threadIdx.x == 0) {
    num_items[0] = total + empties;
    num_items[1] = total;
  }
  if (threadIdx.x < 9) ticket[fan_offset(tiles) + FAN_STRIDE * threadIdx.x] = 0;
}

// Grid: the columns of both regions.  LDS: the per-wave cursors [waves][tiles].
#ifndef GR_PLACE_WAVES
#define GR_PLACE_WAVES 3
#endif
constexpr int TS_CQ = 8;  // tiles per thread per round of k_tile_place's cursor pass
template <int WAVES>
__device__ __forceinline__ void k_tile_place_body(TZones Z, int tiles, int bits,
                                                                    const int2* __restrict__ ranges,
                                                                    int* __restrict__ pairs_out, int* __restrict__ pos_of, const BI blockIdx, const BI gridDim) {
  extern __shared__ int cur[];  // [WAVES][tiles]
  constexpr int NT = 64 * WAVES;
  int c;
  const int zone = tzone_of(Z, (int)blockIdx.x, c);
  const TZone zz = zone_at(Z, zone);
  const int64_t K = zz.K;
  const int zbase = zz.zbase;
  const uint16_t* __restrict__ keys = zz.keys;
  const int* __restrict__ ids_in = zz.ids;
  const int* __restrict__ S = zz.S + (size_t)c * tiles;
  const int w = (int)threadIdx.x >> 6, lane = (int)threadIdx.x & 63;
  int* my = cur + (size_t)w * tiles;
  int64_t kc0, kc1;
  column_range(Z, K, c, kc0, kc1);
  if (kc1 <= kc0) return;  // a column past the region's end (device-side sizing; uniform per block)
  // this wave's part of the column: whole 64-pair steps, the parts in wave order
  const int64_t steps = (kc1 - kc0 + 63) / 64, wsteps = (steps + WAVES - 1) / WAVES;
  const int64_t k0 = min(kc1, kc0 + (int64_t)w * wsteps * 64), k1 = min(kc1, k0 + wsteps * 64);
  const int nseg = (int)((wsteps + TS_SEG - 1) / TS_SEG);
  int d[TS_SEG], id[TS_SEG];
  ts_load(k0, k1, K - 1, lane, keys, ids_in, d, id);  // in flight while the counters are cleared
  // tile bases of the cursor pass (the tile's range start + this column's start within the tile), TS_CQ tiles per
  // thread per round, strided over the block (coalesced) and loaded together; the first round under the count pass
  int rx[TS_CQ], sx[TS_CQ];
  auto load_bases = [&](int t0) {
#pragma unroll
    for (int q = 0; q < TS_CQ; ++q) {
      const int t = min(t0 + q * NT, tiles - 1);
      rx[q] = ranges[2 * t + zone].x;
      sx[q] = S[t];
    }
  };
  load_bases((int)threadIdx.x);
  for (int t = lane; t < tiles; t += 64) my[t] = 0;
  __builtin_amdgcn_wave_barrier();
  for (int seg = 0; seg < nseg; ++seg) {  // this wave's count per tile
    if (seg > 0) ts_load(k0 + (int64_t)seg * 64 * TS_SEG, k1, K - 1, lane, keys, ids_in, d, id);
    // ids are >= 0, so the increment is 1; using id[j] here makes the wave wait for the id loads
    // now, before any store: on gfx9 loads and stores share vmcnt, and a load still pending after a
    // store forces a full vmcnt(0) (i.e. waiting for every earlier store) before each later store.
#pragma unroll
    for (int j = 0; j < TS_SEG; ++j) atomicAdd(&my[d[j] < 0 ? 0 : d[j]], (d[j] < 0 ? 0 : 1) + (id[j] >> 31));
  }
  __syncthreads();
  // cursor of (tile, wave) = tile start + column start within the tile + lower waves' counts
  for (int t0 = threadIdx.x; t0 < tiles; t0 += TS_CQ * NT) {
    if (t0 != (int)threadIdx.x) load_bases(t0);
#pragma unroll
    for (int q = 0; q < TS_CQ; ++q) {
      const int t = t0 + q * NT;
      if (t >= tiles) break;
      int r = rx[q] + sx[q];
#pragma unroll
      for (int u = 0; u < WAVES; ++u) {
        const int m = cur[(size_t)u * tiles + t];
        cur[(size_t)u * tiles + t] = r;
        r += m;
      }
    }
  }
  __syncthreads();
  if (nseg == 1) {
    ts_place(lane, bits, my, d, id, zbase + (int)k0, pairs_out, pos_of);  // keys and ids are still in registers
  } else {
    for (int seg = 0; seg < nseg; ++seg) {
      ts_load(k0 + (int64_t)seg * 64 * TS_SEG, k1, K - 1, lane, keys, ids_in, d, id);
      ts_place(lane, bits, my, d, id, zbase + (int)(k0 + (int64_t)seg * 64 * TS_SEG), pairs_out, pos_of);
    }
  }
}
template <int WAVES>
__global__ __launch_bounds__(64 * WAVES, GR_PLACE_WAVES) void k_tile_place(TZones Z, int tiles, int bits,
                                                                    const int2* __restrict__ ranges,
                                                                    int* __restrict__ pairs_out, int* __restrict__ pos_of) {
  k_tile_place_body<WAVES>(Z, tiles, bits, ranges, pairs_out, pos_of, BI{(int)blockIdx.x, (int)blockIdx.y}, BI{(int)gridDim.x, (int)gridDim.y});
}
struct k_tile_place_args {
  TZones Z;
  int tiles;
  int bits;
  const int2* ranges;
  int* pairs_out;
  int* pos_of;
};
template <int WAVES>
__global__ __launch_bounds__(64 * WAVES, GR_PLACE_WAVES) void k_tile_place_views(VBatch<k_tile_place_args> B) {
  const int vb = vbatch_view(B, (int)blockIdx.x);
  const k_tile_place_args& a = B.a[vb];
  const int lb = (int)blockIdx.x - B.first[vb], gx = B.gx[vb];
  k_tile_place_body<WAVES>(a.Z, a.tiles, a.bits, a.ranges, a.pairs_out, a.pos_of, BI{lb % gx, lb / gx}, BI{gx, (B.first[vb + 1] - B.first[vb]) / gx});
}


// Exact three-way bf16 split: x = hi + mid + lo, each a truncated bf16 (hi keeps 8 significant bits,
// the f32 remainders are exact), returned as f32 values whose low 16 bits are zero.
__device__ __forceinline__ void split3(float x, float& hi, float& mid, float& lo) {
  hi = __uint_as_float(__float_as_uint(x) & 0xffff0000u);
  const float r1 = x - hi;
  mid = __uint_as_float(__float_as_uint(r1) & 0xffff0000u);
  lo = r1 - mid;  // <= 8 significant bits: exactly a bf16
}
// two bf16 (high halves of a, b) into one dword: low half = a, high half = b
__device__ __forceinline__ unsigned pack_bf16(float a, float b) {
  return __builtin_amdgcn_perm(__float_as_uint(b), __float_as_uint(a), 0x07060302u);
}

typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ s16x8 as_frag(uint4 u) {
  s16x8 f;
  __builtin_memcpy(&f, &u, sizeof(f));
  return f;
}

// Split-precision forward (k_raster_fwd_mfma<1|2>): the same contraction on v_mfma_f32_16x16x32_bf16
// (K = 32 Gaussians per instruction).  Mode 1: B = ey and the W / D operands (o ex, o z ex) are split
// exactly into three bf16 pieces and multiplied with the six products of weight >= 2^-16 (f32-grade,
// as the backward): the depth gradient d depth / d w = (z - depth) / (W + 1e-6) cancels
// catastrophically on thin pixels, so W and D must carry full f32 accuracy.  The colour operands
// (o c ex) take two round-to-nearest pieces and three products (split2_frag): each colour accumulator
// is a sum of non-negative terms, each within ~2^-16 of exact with unbiased errors, so its relative
// error stays below that (no cancellation) — far inside the 1e-4 parity bar.  Mode 2 (no_depth_grad
// views): W and D take the colours' two pieces too.
// Lane l supplies A[x = l&15][g = 8(l>>4) + j] and B[g][y = l&15], j = 0..7, and receives
// C[x = 4(l>>4) + r][y = l&15] (the f32 kernel's output map).
__device__ __forceinline__ void split3_frag(const float (&v)[8], s16x8 (&f)[3]) {
  float hi[8], mid[8], lo[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) split3(v[j], hi[j], mid[j], lo[j]);
  f[0] = as_frag(make_uint4(pack_bf16(hi[0], hi[1]), pack_bf16(hi[2], hi[3]), pack_bf16(hi[4], hi[5]), pack_bf16(hi[6], hi[7])));
  f[1] = as_frag(make_uint4(pack_bf16(mid[0], mid[1]), pack_bf16(mid[2], mid[3]), pack_bf16(mid[4], mid[5]),
                            pack_bf16(mid[6], mid[7])));
  f[2] = as_frag(make_uint4(pack_bf16(lo[0], lo[1]), pack_bf16(lo[2], lo[3]), pack_bf16(lo[4], lo[5]), pack_bf16(lo[6], lo[7])));
}
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
// two pieces, both rounded to nearest (v_cvt_pk_bf16_f32): hi = bf16(x), lo = bf16(x - hi).  |x - hi|
// <= 2^-9 |x| and |x - hi - lo| <= 2^-17 |x|, so the dropped lo*lo product is <= 2^-18 of the
// product and every error term is unbiased (a truncated hi would leave a residual of up to 2^-7 and
// a one-signed lo*lo of up to 2^-14).
__device__ __forceinline__ void split2_frag(const float (&v)[8], s16x8 (&f)[2]) {
  unsigned h[4], l[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const f32x2_t x = {v[2 * p], v[2 * p + 1]};
    const bf16x2_t hb = __builtin_convertvector(x, bf16x2_t);
    __builtin_memcpy(&h[p], &hb, 4);
    const f32x2_t r = {x.x - __uint_as_float(h[p] << 16), x.y - __uint_as_float(h[p] & 0xffff0000u)};
    const bf16x2_t lb = __builtin_convertvector(r, bf16x2_t);
    __builtin_memcpy(&l[p], &lb, 4);
  }
  f[0] = as_frag(make_uint4(h[0], h[1], h[2], h[3]));
  f[1] = as_frag(make_uint4(l[0], l[1], l[2], l[3]));
}
__device__ __forceinline__ f32x4 mfma16(const s16x8& a, const s16x8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// sum over the six significant piece products, smallest first
__device__ __forceinline__ f32x4 mfma16_split3(const s16x8 (&a)[3], const s16x8 (&b)[3], f32x4 c) {
  c = mfma16(a[2], b[0], c);
  c = mfma16(a[1], b[1], c);
  c = mfma16(a[0], b[2], c);
  c = mfma16(a[1], b[0], c);
  c = mfma16(a[0], b[1], c);
  return mfma16(a[0], b[0], c);
}
// a in two round-to-nearest pieces, b in the first two pieces of a split (two RNE pieces, or the
// truncated hi + mid of an exact three-piece split, whose lo then enters as a third product so that the
// truncation leaves no one-signed error): the products of weight >= 2^-17.
template <bool B3>
__device__ __forceinline__ f32x4 mfma16_split2(const s16x8 (&a)[2], const s16x8 (&b)[3], f32x4 c) {
  c = mfma16(a[1], b[0], c);
  if constexpr (B3) c = mfma16(a[0], b[2], c);
  c = mfma16(a[0], b[1], c);
  return mfma16(a[0], b[0], c);
}

// two-piece split of 8 values held as 4 pairs (split2_frag)
__device__ __forceinline__ void split2_frag2(const f32x2_t (&v)[4], s16x8 (&f)[2]) {
  float u[8];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    u[2 * p] = v[p].x;
    u[2 * p + 1] = v[p].y;
  }
  split2_frag(u, f);
}

__device__ __forceinline__ void split3_frag2(const f32x2_t (&v)[4], s16x8 (&f)[3]) {
  float u[8];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    u[2 * p] = v[p].x;
    u[2 * p + 1] = v[p].y;
  }
  split3_frag(u, f);
}

// f16 two-piece split (forward MODE 3/4 when GR_FWD_F16): the operands are pre-scaled (folded into the
// exponent arguments) so the footprint's smallest weights stay normal in f16: B = ey by 2^GR_F16_SB
// (ey <= 1, so B <= 2^12), A = o c ex by 2^GR_F16_SA (finite for opacities up to 4094; colours are
// clamped to [0, 1]); the accumulators are rescaled by 2^-(SA+SB), exactly.
// hi = f16(x) rounded to nearest (v_cvt_pk_f16_f32), lo = x - hi exact in f32 (one v_fma_mix_f32 per value reads
// hi's f16 half), rounded to nearest f16: |x - hi| <= 2^-11 |x| and |x - hi - lo| <= 2^-22 |x| while both pieces
// are normal, so the three products miss a b by at most 3 * 2^-22 of it (round 6; truncated pieces, as before,
// left 3 * 2^-20; r06e, profiles/r06_ab_bwd32_f16.txt: the forward even either way, the knob removed).  Four
// instructions per pair of values instead of five; the lo pair straight from v_fma_mix{lo,hi}_f16 (three) measured
// slower, forward 160 -> 167 us, backward 202 -> 206 us (profiles/r06_probe_diag.txt).  Same-box A/B at C4 (fit path):
// forward 145/154 -> 140/135 us, step 1369-1380 -> 1403-1408 Mpx/s (A/B at SA = SB = 12); fit-path errors vs the float64 oracle
// out 1e-7, gradients <= 1.2e-5 (profiles/r02p_ab_f16.txt).
#ifndef GR_FWD_F16
#define GR_FWD_F16 1
#endif
#ifndef GR_F16_SA
#define GR_F16_SA 4
#endif
#ifndef GR_F16_SB
#define GR_F16_SB 12
#endif
// The A pre-scale of a view: 2^GR_F16_SA while the largest o max(1, z) of its kept Gaussians is below 2^11,
// lowered by one per binade above, so o * c * ex * 2^sa stays <= 2^15 (the z factor is a margin kept from an f16 depth channel)
// (no inf, whatever the opacities and depths; k_plan computes it from k_preprocess's per-block maxima).  Views with
// o z below 2048 - every fit, whose opacities are sigmoid outputs, at any sane camera distance - get exactly
// GR_F16_SA.  The A operands are o c ex with o = max(op, 0)
// (the record's clamp, torch_renderer.py:177) and c clamped to [0, 1] (:144), so |A| <= 2^sa max(op, 0): a negative
// opacity contributes nothing and needs no range (tests/test_scale_gpu.py, opacities down to -1e5).
__device__ __forceinline__ int f16_sa_of(float omax) {
  if (!(omax <= 3.0e38f)) return GR_F16_SA;  // inf / NaN opacities give inf / NaN outputs in any precision
  int e = 0;
  (void)frexpf(omax, &e);  // omax <= 2^e
  return GR_F16_SA - (e > 11 ? e - 11 : 0);
}
__device__ __forceinline__ float f16_resid_lo(float x, unsigned h) {  // x - f16(h[15:0])
  float r;
  asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(r) : "v"(h), "v"(x));
  return r;
}
__device__ __forceinline__ float f16_resid_hi(float x, unsigned h) {  // x - f16(h[31:16])
  float r;
  asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(r) : "v"(h), "v"(x));
  return r;
}
typedef _Float16 f16x2h_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned pk_f16(float a, float b) {  // two f16, round to nearest even: v_cvt_pk_f16_f32
  return __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2_t{a, b}, f16x2h_t));
}
__device__ __forceinline__ void split2h_frag2(const f32x2_t (&v)[4], s16x8 (&f)[2]) {
  unsigned h[4], l[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    h[p] = pk_f16(v[p].x, v[p].y);
    l[p] = pk_f16(f16_resid_lo(v[p].x, h[p]), f16_resid_hi(v[p].y, h[p]));
  }
  f[0] = as_frag(make_uint4(h[0], h[1], h[2], h[3]));
  f[1] = as_frag(make_uint4(l[0], l[1], l[2], l[3]));
}
// the same split (round to nearest) of 8 values held as a plain array
__device__ __forceinline__ void split2h_frag(const float (&v)[8], s16x8 (&f)[2]) {
  unsigned h[4], l[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    h[p] = pk_f16(v[2 * p], v[2 * p + 1]);
    l[p] = pk_f16(f16_resid_lo(v[2 * p], h[p]), f16_resid_hi(v[2 * p + 1], h[p]));
  }
  f[0] = as_frag(make_uint4(h[0], h[1], h[2], h[3]));
  f[1] = as_frag(make_uint4(l[0], l[1], l[2], l[3]));
}
// The 32-pixel backward's A operands (the per-pixel upstream vectors) in f16 pieces: per channel the values are scaled
// by 2^e with e = 14 - exponent(bound of |u|), so the bound lies in [2^13, 2^14) and values down to 2^-17 of it keep
// both pieces normal (exact power-of-two scaling, undone on the backward's sums)
__device__ __forceinline__ int f16_exp_of(float m) {
  if (!(m > 0.0f) || !(m <= 3.0e38f)) return 0;  // an all-zero channel, or inf / NaN (they propagate either way)
  int e = 0;
  (void)frexpf(m, &e);  // m < 2^e
  return 14 - e;
}
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
__device__ __forceinline__ f32x4 mfma16h(const s16x8& a, const s16x8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, a), __builtin_bit_cast(f16x8_t, b), c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16h_split2(const s16x8 (&a)[2], const s16x8 (&b)[2], f32x4 c) {
  c = mfma16h(a[1], b[0], c);
  c = mfma16h(a[0], b[1], c);
  return mfma16h(a[0], b[0], c);
}

// Staged batch layout of the split-precision forward: nine planes of TP floats (px py qx qy o r g b z),
// one LDS-DMA dword per lane and field.  A lane's eight Gaussians of a step are then consecutive in every
// plane (two ds_read_b128 per field) and the operand arithmetic runs on packed f32 pairs of Gaussians
// (v_pk_add_f32 / v_pk_mul_f32: two lanes' worth per issue, the same IEEE results as the scalar ops).
constexpr int FWD_PLANES = 9;

// The LDS-DMAs of one staged Gaussian: record fields f = 0..7 (0..4 for tail items, which need no
// colour) to plane f, z to plane 8.  One asm block: m0 is saved once, and the fields share the record's
// address register: the instruction offset (4f) is added to the LDS address too, so m0 is set to
// plane f's base minus 4f.
#define GR_GLDS_FIELD(F) "s_add_u32 m0, %3, " #F "*1020\n\ts_nop 0\n\tglobal_load_lds_dword %1, off offset:" #F "*4\n\t"
#define GR_GLDS_FIELD2(F) "s_add_u32 m0, %2, " #F "*1020\n\ts_nop 0\n\tglobal_load_lds_dword %1, off offset:" #F "*4\n\t"
template <bool TAIL, bool ZCH = true>
__device__ __forceinline__ void glds4_planes(const float4* rec, const float* z, float* wave_base) {
  static_assert(TP == 256, "plane stride 1024 B is written into the asm below");
  unsigned keep;
  if constexpr (!ZCH) {  // no depth channel: px py qx qy o (tail: W only) or all eight record fields
    if constexpr (TAIL)
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\t"
                   GR_GLDS_FIELD2(1) GR_GLDS_FIELD2(2) GR_GLDS_FIELD2(3) GR_GLDS_FIELD2(4) "s_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(rec), "s"(lds_addr(wave_base)) : "memory", "scc");
    else
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\t"
                   GR_GLDS_FIELD2(1) GR_GLDS_FIELD2(2) GR_GLDS_FIELD2(3) GR_GLDS_FIELD2(4)
                   GR_GLDS_FIELD2(5) GR_GLDS_FIELD2(6) GR_GLDS_FIELD2(7) "s_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(rec), "s"(lds_addr(wave_base)) : "memory", "scc");
    (void)z;
  } else if constexpr (TAIL) {
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\t"
                 GR_GLDS_FIELD(1) GR_GLDS_FIELD(2) GR_GLDS_FIELD(3) GR_GLDS_FIELD(4)
                 "s_add_u32 m0, %3, 8192\n\ts_nop 0\n\tglobal_load_lds_dword %2, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(rec), "v"(z), "s"(lds_addr(wave_base)) : "memory", "scc");
  } else {
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\t"
                 GR_GLDS_FIELD(1) GR_GLDS_FIELD(2) GR_GLDS_FIELD(3) GR_GLDS_FIELD(4)
                 GR_GLDS_FIELD(5) GR_GLDS_FIELD(6) GR_GLDS_FIELD(7)
                 "s_add_u32 m0, %3, 8192\n\ts_nop 0\n\tglobal_load_lds_dword %2, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(rec), "v"(z), "s"(lds_addr(wave_base)) : "memory", "scc");
  }
}
#undef GR_GLDS_FIELD
#undef GR_GLDS_FIELD2

// ZCH = false (views rendered for the fused fit path: no depth output, no depth gradient): the depth
// channel is not accumulated (no z staging, no D products).
template <bool TAIL, bool PRECISE, bool ZCH = true>
__device__ __forceinline__ void fwd_accumulate_bf16(float* smem, int n, int k0, int k1, int tid, int wave, float xc, float yc,
                                                    int gq, const int* __restrict__ pairs, const float4* __restrict__ rec,
                                                    f32x4& cW, f32x4& cR, f32x4& cG, f32x4& cB, f32x4& cD, float sa) {
  constexpr int BUF = FWD_PLANES * TP;  // floats per buffer
  auto stage = [&](int g, int b) {
    glds4_planes<TAIL, ZCH>(rec_of(g, n, rec), zrec_of(g, n, rec), smem + b * BUF + 64 * wave);
  };
  stage(stage_pair(stage_id(k0 + tid, k1, pairs), k0 + tid, k1), 0);
  int idn = stage_id(k0 + TP + tid, k1, pairs);
  int buf = 0;
  const f32x2_t X = {xc, xc}, Y = {yc, yc};
  // core items of renders without a depth output take f16 pieces (W and the colours).  A depth output
  // D / (W + 1e-6) divides by W: where W is small the pieces of its smallest terms are f16 subnormals
  // (relL2 1.8e-3 on the drop-in's 65k-Gaussian view, tests/test_chain_gpu.py), so W and D stay on bf16
  // pieces, whose exponent range is f32's; tail items (small weights) too
  constexpr bool F16 = GR_FWD_F16 && !PRECISE && !TAIL && !ZCH;
  const f32x2_t SA = {sa, sa}, SB = {(float)GR_F16_SB, (float)GR_F16_SB};
  (void)SA;
  (void)SB;
  for (int base = k0; base < k1; base += TP, buf ^= 1) {
    stage_wait();
    GR_STAGE_SYNC();
    if (base + TP < k1) stage(stage_pair(idn, base + TP + tid, k1), buf ^ 1);
    idn = stage_id(base + 2 * TP + tid, k1, pairs);
    const int cnt = min(TP, k1 - base) - wave * 64;           // Gaussians of this batch for this wave
    const int nst = cnt <= 0 ? 0 : min(2, (cnt + 31) >> 5);  // steps of 32 (padding records are zero)
    for (int st = 0; st < nst; ++st) {
      const float* s = smem + buf * BUF + wave * 64 + st * 32 + 8 * gq;
      // the eight Gaussians of field f as four pairs
      auto ld = [&](int f, f32x2_t (&v)[4]) {
        const float4 u0 = *reinterpret_cast<const float4*>(s + f * TP);
        const float4 u1 = *reinterpret_cast<const float4*>(s + f * TP + 4);
        v[0] = f32x2_t{u0.x, u0.y};
        v[1] = f32x2_t{u0.z, u0.w};
        v[2] = f32x2_t{u1.x, u1.y};
        v[3] = f32x2_t{u1.z, u1.w};
      };
      f32x2_t px[4], py[4], qx[4], qy[4], o[4], z[4];
      ld(0, px);
      ld(1, py);
      ld(2, qx);
      ld(3, qy);
      ld(4, o);
      if constexpr (ZCH) ld(8, z);
      f32x2_t aW[4], aD[4], bv[4], oe[4];
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const f32x2_t dx = X - px[p], dy = Y - py[p];
#if GR_FWD_F16
        const f32x2_t tx = F16 ? __builtin_elementwise_fma(dx * qx[p], dx, SA) : (dx * qx[p]) * dx;
        const f32x2_t ty = F16 ? __builtin_elementwise_fma(dy * qy[p], dy, SB) : (dy * qy[p]) * dy;
#else
        const f32x2_t tx = (dx * qx[p]) * dx, ty = (dy * qy[p]) * dy;
#endif
        const f32x2_t ex = {__builtin_amdgcn_exp2f(tx.x), __builtin_amdgcn_exp2f(tx.y)};
        bv[p] = f32x2_t{__builtin_amdgcn_exp2f(ty.x), __builtin_amdgcn_exp2f(ty.y)};
        oe[p] = o[p] * ex;
        aW[p] = oe[p];
        if constexpr (ZCH) aD[p] = oe[p] * z[p];
      }
      s16x8 fb[3], f3[3], fb2h[2];
      if constexpr (PRECISE) {
        split3_frag2(bv, fb);
        split3_frag2(aW, f3);
        cW = mfma16_split3(f3, fb, cW);
        if constexpr (ZCH) {
          split3_frag2(aD, f3);
          cD = mfma16_split3(f3, fb, cD);
        }
      } else if (F16) {  // f16 pieces of the pre-scaled operands
        s16x8 f2[2];
        split2h_frag2(bv, fb2h);
        split2h_frag2(aW, f2);
        cW = mfma16h_split2(f2, fb2h, cW);
      } else {  // no depth gradient will follow: W and D need only what the colours need
        s16x8 f2b[2], f2[2];
        split2_frag2(bv, f2b);
        fb[0] = f2b[0];
        fb[1] = f2b[1];
        split2_frag2(aW, f2);
        cW = mfma16_split2<false>(f2, fb, cW);
        if constexpr (ZCH) {
          split2_frag2(aD, f2);
          cD = mfma16_split2<false>(f2, fb, cD);
        }
      }
      if constexpr (!TAIL) {
        f32x2_t c[4], a[4];
        s16x8 f2[2];
        if constexpr (F16) {
          ld(5, c);
#pragma unroll
          for (int p = 0; p < 4; ++p) a[p] = oe[p] * c[p];
          split2h_frag2(a, f2);
          cR = mfma16h_split2(f2, fb2h, cR);
          ld(6, c);
#pragma unroll
          for (int p = 0; p < 4; ++p) a[p] = oe[p] * c[p];
          split2h_frag2(a, f2);
          cG = mfma16h_split2(f2, fb2h, cG);
          ld(7, c);
#pragma unroll
          for (int p = 0; p < 4; ++p) a[p] = oe[p] * c[p];
          split2h_frag2(a, f2);
          cB = mfma16h_split2(f2, fb2h, cB);
        } else {
        ld(5, c);
#pragma unroll
        for (int p = 0; p < 4; ++p) a[p] = oe[p] * c[p];
        split2_frag2(a, f2);
        cR = mfma16_split2<PRECISE>(f2, fb, cR);
        ld(6, c);
#pragma unroll
        for (int p = 0; p < 4; ++p) a[p] = oe[p] * c[p];
        split2_frag2(a, f2);
        cG = mfma16_split2<PRECISE>(f2, fb, cG);
        ld(7, c);
#pragma unroll
        for (int p = 0; p < 4; ++p) a[p] = oe[p] * c[p];
        split2_frag2(a, f2);
        cB = mfma16_split2<PRECISE>(f2, fb, cB);
        }
      }
    }
  }
}

// Items of a tile (virtual tiles 2t: core, 2t+1: tail; contiguous in the item list).
__device__ __forceinline__ int tile_chunks(int2 r, int ch = CH) { return (r.y - r.x + ch - 1) / ch; }

__device__ __forceinline__ void write_pixel(const ViewK& v, int p, const float* acc, float* __restrict__ out_rgb,
                                            float* __restrict__ out_alpha, float* __restrict__ out_depth,
                                            float4* __restrict__ saved4, float* __restrict__ savedD) {
  const float aW = acc[0], den = 1.0f + aW;
  if (out_rgb) {  // (gr_fwd_render_l1 may render no image: its loss gradients come from the sums)
    out_rgb[3 * p + 0] = clamp01((view_bg(v, 0) + acc[1]) / den);
    out_rgb[3 * p + 1] = clamp01((view_bg(v, 1) + acc[2]) / den);
    out_rgb[3 * p + 2] = clamp01((view_bg(v, 2) + acc[3]) / den);
  }
  if (out_alpha) out_alpha[p] = clamp01(aW / den);
  if (out_depth) {
    const float d = acc[4] / (aW + 1e-6f);
    out_depth[p] = d < 0.0f ? 0.0f : d;
  }
  if (saved4) {
    saved4[p] = make_float4(aW, acc[1], acc[2], acc[3]);
    savedD[p] = acc[4];
  }
}

// gr_fwd_compose: a view's outputs from its saved pixel sums (write_pixel), with the view's background.
__global__ __launch_bounds__(256) void k_compose(ViewK v, int hw, const float4* __restrict__ saved4,
                                                 const float* __restrict__ savedD, float* __restrict__ out_rgb,
                                                 float* __restrict__ out_alpha, float* __restrict__ out_depth) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= hw) return;
  const float4 a = saved4[p];
  const float acc[5] = {a.x, a.y, a.z, a.w, savedD[p]};
  write_pixel(v, p, acc, out_rgb, out_alpha, out_depth, nullptr, nullptr);
}

// bf16 split-precision backward (k_raster_bwd_bf16): per tile, A fragments of v_mfma_f32_32x32x16_bf16
// for 2 sides (T: contraction over x, R: over y) x 3 channel pairs x 3 bf16 pieces x 64 lanes, 16 B each.
constexpr int UF_FRAGS = 2 * 3 * 3 * 64;  // uint4 per tile
static_assert(UF_FRAGS == UF_FRAGS16, "TileCfg");
// channel pairs on the 32 MFMA rows (16 per channel): (dC_r, dC_g), (dC_b, -), (dW, dD); tail items
// (depth-coupled terms only) need just the last pair
// Without an upstream depth gradient dD is identically zero, so the four live channels fill two pairs:
// (dC_r, dC_g), (dC_b, dW) and the third pair is never contracted (two thirds of the MFMA work).
__device__ __forceinline__ int pair_channel(int pr, int c, bool depth) {
  if (!depth) return pr == 0 ? c : (pr == 1 ? 2 + c : -1);
  return pr == 0 ? c : (pr == 1 ? (c == 0 ? 2 : -1) : 3 + c);
}
// contracted coordinate of k-slot 8h + j of the 32x32x16 operands: the 8 pixels a lane half h owns,
// {4h..4h+3, 8+4h..8+4h+3}, which are also the output rows that lane half holds (C map, row =
// (reg&3) + 8 (reg>>2) + 4h): one set of exponentials per lane serves both contractions.
__device__ __forceinline__ int kslot_pixel(int h, int j) { return (j < 4) ? 4 * h + j : 8 + 4 * h + (j - 4); }

// Per-pixel upstream vector U = (dC_r, dC_g, dC_b, dW, dD) of the OIT finalize
// (torch_renderer.py:192-203), laid out as pre-split MFMA fragments [tile][UF_FRAGS] for the backward
// work items.  Fused fit loss (L1Args.t_rgb != nullptr, gr_bwd_l1 / gr_fwd_render_l1): the upstream
// gradients are those of the fit loop's view loss mean|out - t| + w_sil mean|alpha - m|
// (fit_multiview_stub.py:292-299) scaled by g_scale, evaluated from the pixel's sums exactly as
// write_pixel turns them into outputs, with torch's abs' = sign (sign(0) = 0); per-tile sums of
// |out - t| and |alpha - m| go to tile_loss.
struct L1Args {
  const float* t_rgb;   // (H,W,3) target image
  const float* t_mask;  // (H,W) silhouette target or nullptr
  float w_sil, g_scale;
  float* tile_loss;     // [tiles][4]: sums of |out - t|, |alpha - m|, |d_pred - t_d|, and the depth-max term
  // depth loss (gr_bwd_fit, fit_multiview_stub.py:301-305): w_depth mean|depth / (max(depth) + 1e-6) - t_depth|
  const float* t_depth = nullptr;  // (H,W) depth target or nullptr (no depth term)
  float w_depth = 0.0f;
  const float* dscal = nullptr;    // device scalars: [0] max(depth), [1] the max's gradient per arg-max pixel
  int pieces = 2;                  // bf16 pieces of the upstream fragments (gr_fwd_render_l1: 3 at f32 grade)
  // gr_fwd_render_l1: the view loss, written by the forward's last finished tile (photometric / silhouette element
  // counts n1 / n2, tile_loss_total)
  float* loss_out = nullptr;
  int64_t n1 = 0, n2 = 0;
};

// The view loss from the per-tile L1 sums (one block of 256 threads; double sums in a fixed order):
// mean |out - t| + w_sil mean |alpha - m| (+ w_depth mean |d_pred - t_d| with n3 > 0).  THROUGH: the sums were
// written in the same launch (write-through, arrive_last).
template <bool THROUGH>
__device__ __forceinline__ void tile_loss_total(const float* __restrict__ tile_loss, int tiles, int64_t n1, int64_t n2,
                                                float w_sil, int64_t n3, float w_depth, float* __restrict__ loss,
                                                double (*r)[256]) {
  const int t = threadIdx.x;
  auto ld = [&](int i) { return THROUGH ? ld_through(tile_loss + i) : tile_loss[i]; };
  double s1 = 0.0, s2 = 0.0, s3 = 0.0;
  for (int i = t; i < tiles; i += 256) {
    s1 += (double)ld(4 * i);
    s2 += (double)ld(4 * i + 1);
    if (n3 > 0) s3 += (double)ld(4 * i + 2);
  }
  r[0][t] = s1;
  r[1][t] = s2;
  r[2][t] = s3;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w) {
      r[0][t] += r[0][t + w];
      r[1][t] += r[1][t + w];
      r[2][t] += r[2][t + w];
    }
    __syncthreads();
  }
  if (t != 0) return;
  float l = (float)(r[0][0] / (double)n1);
  if (n2 > 0) l = l + w_sil * (float)(r[1][0] / (double)n2);
  if (n3 > 0) l = l + w_depth * (float)(r[2][0] / (double)n3);
  *loss = l;
}

__device__ __forceinline__ float sign0(float t) { return t > 0.0f ? 1.0f : (t < 0.0f ? -1.0f : 0.0f); }

// U of pixel p from its sums s = (W, C_r, C_g, C_b) and D; l_rgb / l_sil get the pixel's L1 terms.
__device__ __forceinline__ void pixel_upstream(const ViewK& v, int p, float4 s, float Dp, const float* __restrict__ g_rgb,
                                               const float* __restrict__ g_alpha, const float* __restrict__ g_depth,
                                               const L1Args& l1, float (&u)[5], float& l_rgb, float& l_sil) {
  const float den = 1.0f + s.x, dden = s.x + 1e-6f;
  // one correctly rounded reciprocal of the finalize's denominator instead of ten divisions (each ~10 VALU): the
  // quotients below are products with it, within 1 ulp of the divisions (round 6, the L1 epilogue of the fit forwards)
  const float inv = 1.0f / den;
  float gW = 0.f;
  const float C[3] = {s.y, s.z, s.w};
  const float HWf = (float)v.W * (float)v.H;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float r = (view_bg(v, k) + C[k]) * inv;
    float gk;
    if (l1.t_rgb) {
      const float t = clamp01(r) - l1.t_rgb[3 * p + k];
      l_rgb += fabsf(t);
      gk = sign0(t) * (l1.g_scale / (3.0f * HWf));
    } else {
      gk = g_rgb[3 * p + k];
    }
    const float go = (r >= 0.0f && r <= 1.0f) ? gk : 0.0f;
    u[k] = go * inv;
    gW -= (go * r) * inv;
  }
  const float al = s.x * inv;
  float ga = 0.0f;
  bool has_a = g_alpha != nullptr;
  if (l1.t_rgb && l1.t_mask) {
    const float t = clamp01(al) - l1.t_mask[p];
    l_sil = fabsf(t);
    ga = sign0(t) * ((l1.w_sil * l1.g_scale) / HWf);
    has_a = true;
  } else if (g_alpha) {
    ga = g_alpha[p];
  }
  if (has_a && al >= 0.0f && al <= 1.0f) gW += ga * (inv * inv);
  const bool dfit = l1.t_rgb && l1.t_depth;
  if (g_depth || dfit) {
    const float d = Dp / dden;
    if (d >= 0.0f) {  // depth = clamp_min(D / (W + 1e-6), 0): the gradient passes where d >= 0
      float gd;
      if (dfit) {  // d (w_depth mean|d / (M + 1e-6) - t|) / d depth, plus the max's share on arg-max pixels
        const float M = l1.dscal[0], dm = M + 1e-6f;
        const float t = d / dm - l1.t_depth[p];
        gd = (sign0(t) * ((l1.w_depth * l1.g_scale) / HWf)) / dm;
        if (d == M) gd += l1.dscal[1];
      } else {
        gd = g_depth[p];
      }
      gW -= gd * Dp / (dden * dden);
      u[4] = gd / dden;
    }
  }
  u[3] = gW;
}

// Depth loss of the fused fit backward (gr_bwd_fit): the depth image's maximum M (per tile, then one
// block: exact, order-free), then per tile the sums of |d / (M + 1e-6) - t|, of the max's chain term
// sign(.) (d / (M + 1e-6)) / (M + 1e-6) (torch's div backward w.r.t. the denominator, up to its factor) and
// the count of arg-max pixels; one block turns them into the max's gradient per arg-max pixel
// (torch's max backward shares it evenly among ties).  Depth = max(D / (W + 1e-6), 0) from the saved sums,
// exactly as write_pixel made it.
__device__ __forceinline__ float saved_depth(const float4* __restrict__ saved4, const float* __restrict__ savedD, int p) {
  const float d = savedD[p] / (saved4[p].x + 1e-6f);
  return d < 0.0f ? 0.0f : d;
}

// Per tile the depth maximum; the last tile to finish (arrive_last_tile) takes the image's.
__device__ __forceinline__ void k_depth_tile_max_body(ViewK v, const float4* __restrict__ saved4,
                                                        const float* __restrict__ savedD, float* __restrict__ tile_aux,
                                                        float* __restrict__ dscal, int* __restrict__ ticket, const BI blockIdx, const BI gridDim) {
  const int tile = blockIdx.x, tid = threadIdx.x, tiles = v.tiles_x * v.tiles_y;
  const int tx = tile % v.tiles_x, ty = tile / v.tiles_x;
  const int x = tx * T + (tid & (T - 1)), y = ty * T + (tid >> 4);
  float m = (x < v.W && y < v.H) ? saved_depth(saved4, savedD, y * v.W + x) : 0.0f;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  __shared__ float sm[4];
  __shared__ int last;
  if ((tid & 63) == 0) sm[tid >> 6] = m;
  __syncthreads();
  if (tid == 0) st_through(&tile_aux[2 * tile], fmaxf(fmaxf(sm[0], sm[1]), fmaxf(sm[2], sm[3])));
  if (!arrive_last_tile(ticket, tiles, tile, &last)) return;
  m = 0.0f;
  for (int t = tid; t < tiles; t += 256) m = fmaxf(m, ld_through(&tile_aux[2 * t]));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if ((tid & 63) == 0) sm[tid >> 6] = m;
  __syncthreads();
  if (tid == 0) dscal[0] = fmaxf(fmaxf(sm[0], sm[1]), fmaxf(sm[2], sm[3]));
}
__global__ __launch_bounds__(256) void k_depth_tile_max(ViewK v, const float4* __restrict__ saved4,
                                                        const float* __restrict__ savedD, float* __restrict__ tile_aux,
                                                        float* __restrict__ dscal, int* __restrict__ ticket) {
  k_depth_tile_max_body(v, saved4, savedD, tile_aux, dscal, ticket, BI{(int)blockIdx.x, (int)blockIdx.y}, BI{(int)gridDim.x, (int)gridDim.y});
}
struct k_depth_tile_max_args {
  ViewK v;
  const float4* saved4;
  const float* savedD;
  float* tile_aux;
  float* dscal;
  int* ticket;
};
__global__ __launch_bounds__(256) void k_depth_tile_max_views(VBatch<k_depth_tile_max_args> B) {
  const int vb = vbatch_view(B, (int)blockIdx.x);
  const k_depth_tile_max_args& a = B.a[vb];
  const int lb = (int)blockIdx.x - B.first[vb], gx = B.gx[vb];
  k_depth_tile_max_body(a.v, a.saved4, a.savedD, a.tile_aux, a.dscal, a.ticket, BI{lb % gx, lb / gx}, BI{gx, (B.first[vb + 1] - B.first[vb]) / gx});
}


__device__ void depth_final(const float* __restrict__ tile_loss, const float* __restrict__ tile_aux, int tiles, int64_t HW,
                            float w_depth, float g_scale, float* __restrict__ dscal, double (*r)[256]);
// Per tile the depth loss's sums; the last tile to finish (arrive_last_tile) turns them into the max's
// gradient per arg-max pixel (depth_final).
__device__ __forceinline__ void k_depth_tile_sums_body(ViewK v, const float4* __restrict__ saved4,
                                                         const float* __restrict__ savedD, const float* __restrict__ t_depth,
                                                         float* __restrict__ dscal, float* __restrict__ tile_loss,
                                                         float* __restrict__ tile_aux, int64_t HW, float w_depth,
                                                         float g_scale, int* __restrict__ ticket, const BI blockIdx, const BI gridDim) {
  const int tile = blockIdx.x, tid = threadIdx.x;
  const int tx = tile % v.tiles_x, ty = tile / v.tiles_x;
  const int x = tx * T + (tid & (T - 1)), y = ty * T + (tid >> 4);
  float l = 0.f, sd = 0.f, cnt = 0.f;
  if (x < v.W && y < v.H) {
    const int p = y * v.W + x;
    const float d = saved_depth(saved4, savedD, p), M = dscal[0], dm = M + 1e-6f;
    const float t = d / dm - t_depth[p];
    l = fabsf(t);
    sd = sign0(t) * ((d / dm) / dm);
    cnt = d == M ? 1.0f : 0.0f;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    l += __shfl_xor(l, o);
    sd += __shfl_xor(sd, o);
    cnt += __shfl_xor(cnt, o);
  }
  __shared__ float sm[3][4];
  if ((tid & 63) == 0) {
    sm[0][tid >> 6] = l;
    sm[1][tid >> 6] = sd;
    sm[2][tid >> 6] = cnt;
  }
  __syncthreads();
  if (tid == 0) {
    st_through(&tile_loss[4 * tile + 2], ((sm[0][0] + sm[0][1]) + sm[0][2]) + sm[0][3]);
    st_through(&tile_loss[4 * tile + 3], ((sm[1][0] + sm[1][1]) + sm[1][2]) + sm[1][3]);
    st_through(&tile_aux[2 * tile + 1], ((sm[2][0] + sm[2][1]) + sm[2][2]) + sm[2][3]);
  }
  __shared__ int last;
  __shared__ double r[3][256];
  const int tiles = v.tiles_x * v.tiles_y;
  if (!arrive_last_tile(ticket, tiles, tile, &last)) return;
  depth_final(tile_loss, tile_aux, tiles, HW, w_depth, g_scale, dscal, r);
}
__global__ __launch_bounds__(256) void k_depth_tile_sums(ViewK v, const float4* __restrict__ saved4,
                                                         const float* __restrict__ savedD, const float* __restrict__ t_depth,
                                                         float* __restrict__ dscal, float* __restrict__ tile_loss,
                                                         float* __restrict__ tile_aux, int64_t HW, float w_depth,
                                                         float g_scale, int* __restrict__ ticket) {
  k_depth_tile_sums_body(v, saved4, savedD, t_depth, dscal, tile_loss, tile_aux, HW, w_depth, g_scale, ticket, BI{(int)blockIdx.x, (int)blockIdx.y}, BI{(int)gridDim.x, (int)gridDim.y});
}
struct k_depth_tile_sums_args {
  ViewK v;
  const float4* saved4;
  const float* savedD;
  const float* t_depth;
  float* dscal;
  float* tile_loss;
  float* tile_aux;
  int64_t HW;
  float w_depth;
  float g_scale;
  int* ticket;
};
__global__ __launch_bounds__(256) void k_depth_tile_sums_views(VBatch<k_depth_tile_sums_args> B) {
  const int vb = vbatch_view(B, (int)blockIdx.x);
  const k_depth_tile_sums_args& a = B.a[vb];
  const int lb = (int)blockIdx.x - B.first[vb], gx = B.gx[vb];
  k_depth_tile_sums_body(a.v, a.saved4, a.savedD, a.t_depth, a.dscal, a.tile_loss, a.tile_aux, a.HW, a.w_depth, a.g_scale, a.ticket, BI{lb % gx, lb / gx}, BI{gx, (B.first[vb + 1] - B.first[vb]) / gx});
}


// dscal[1] = -(w_depth g_scale / HW) sum_p sign(.) (d_p / dm) / dm / (number of arg-max pixels), from the tiles'
// write-through sums (the last tile of k_depth_tile_sums)
__device__ void depth_final(const float* __restrict__ tile_loss, const float* __restrict__ tile_aux, int tiles, int64_t HW,
                            float w_depth, float g_scale, float* __restrict__ dscal, double (*r)[256]) {
  const int t = threadIdx.x;
  double s1 = 0.0, s2 = 0.0;
  for (int i = t; i < tiles; i += 256) {
    s1 += (double)ld_through(&tile_loss[4 * i + 3]);
    s2 += (double)ld_through(&tile_aux[2 * i + 1]);
  }
  r[0][t] = s1;
  r[1][t] = s2;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w) {
      r[0][t] += r[0][t + w];
      r[1][t] += r[1][t + w];
    }
    __syncthreads();
  }
  if (t != 0) return;
  const float gM = -((w_depth * g_scale) / (float)HW) * (float)r[0][0];
  dscal[1] = r[1][0] > 0.0 ? gM / (float)r[1][0] : 0.0f;
}

// The tile's L1 sums (block of 256 threads, one pixel each): waves, then the 4 wave sums in a fixed order.
__device__ __forceinline__ void tile_loss_sums(int tile, int tid, float l_rgb, float l_sil, float* tile_loss) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    l_rgb += __shfl_xor(l_rgb, o);
    l_sil += __shfl_xor(l_sil, o);
  }
  __shared__ float sL[2][4];
  if ((tid & 63) == 0) {
    sL[0][tid >> 6] = l_rgb;
    sL[1][tid >> 6] = l_sil;
  }
  __syncthreads();
  if (tid == 0) {
    // write-through: the forward's last finished tile reads them in the same launch (arrive_last)
    st_through(&tile_loss[4 * tile], ((sL[0][0] + sL[0][1]) + sL[0][2]) + sL[0][3]);
    st_through(&tile_loss[4 * tile + 1], ((sL[1][0] + sL[1][1]) + sL[1][2]) + sL[1][3]);
  }
}

// The tile's U (sU[5][256] in LDS, published by a barrier) -> its bf16 fragments in UF: 384 (side,
// pair, lane) fragment sets over the block's 256 threads; pair 2 (dW, dD) only with a depth gradient.
__device__ __forceinline__ void tile_fragments(const float (*sU)[TP], uint4* __restrict__ fr, int tid, int pieces, bool depth) {
  for (int cmb = tid; cmb < 2 * 3 * 64; cmb += 256) {
    const int side = cmb / 192, pr = (cmb / 64) % 3, l = cmb & 63;
    if (!depth && pr == 2) continue;  // never read
    const int r = l & 31, h = l >> 5, ch = pair_channel(pr, r >> 4, depth), i = r & 15;
    uint4* o = fr + ((side * 3 + pr) * 3) * 64 + l;
    // no_depth_grad views: two round-to-nearest pieces (split2_frag); with a depth gradient the colour
    // pairs take them too (contracted against three-piece B, mfma_split_a2b3): only the (dW, dD) pair
    // cancels in the per-pair epilogue and needs the exact three-piece split
    if (pieces == 2 || (depth && pr < 2)) {
      float val[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int kk = kslot_pixel(h, j);
        val[j] = ch < 0 ? 0.0f : (side == 0 ? sU[ch][i * T + kk] : sU[ch][kk * T + i]);
      }
      s16x8 f2[2];
      split2_frag(val, f2);
      __builtin_memcpy(&o[0], &f2[0], 16);
      __builtin_memcpy(&o[64], &f2[1], 16);
      continue;
    }
    float hi[8], mid[8], lo[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int kk = kslot_pixel(h, j);
      const float val = ch < 0 ? 0.0f : (side == 0 ? sU[ch][i * T + kk] : sU[ch][kk * T + i]);
      split3(val, hi[j], mid[j], lo[j]);
    }
    o[0] = make_uint4(pack_bf16(hi[0], hi[1]), pack_bf16(hi[2], hi[3]), pack_bf16(hi[4], hi[5]), pack_bf16(hi[6], hi[7]));
    o[64] = make_uint4(pack_bf16(mid[0], mid[1]), pack_bf16(mid[2], mid[3]), pack_bf16(mid[4], mid[5]),
                       pack_bf16(mid[6], mid[7]));
    o[128] = make_uint4(pack_bf16(lo[0], lo[1]), pack_bf16(lo[2], lo[3]), pack_bf16(lo[4], lo[5]), pack_bf16(lo[6], lo[7]));
  }
}

// With the fit loss (l1.t_rgb) the last tile to finish (arrive_last_tile) also writes the view loss.
__device__ __forceinline__ void k_pixel_grads_body(ViewK v, const float4* __restrict__ saved4,
                                                     const float* __restrict__ savedD, const float* __restrict__ g_rgb,
                                                     const float* __restrict__ g_alpha, const float* __restrict__ g_depth,
                                                     uint4* __restrict__ UF, int pieces, L1Args l1, bool depth,
                                                     int* __restrict__ ticket, const BI blockIdx, const BI gridDim) {
  const int tile = blockIdx.x, tid = threadIdx.x;
  const int tx = tile % v.tiles_x, ty = tile / v.tiles_x;
  const int x = tx * T + (tid & (T - 1)), y = ty * T + (tid >> 4);
  float u[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  float l_rgb = 0.f, l_sil = 0.f;
  if (x < v.W && y < v.H) {
    const int p = y * v.W + x;
    pixel_upstream(v, p, saved4[p], savedD[p], g_rgb, g_alpha, g_depth, l1, u, l_rgb, l_sil);
  }
  if (l1.tile_loss) tile_loss_sums(tile, tid, l_rgb, l_sil, l1.tile_loss);
  // six rows, not five: the last tile reuses the buffer as tile_loss_total's double[3][256] (6 KiB)
  __shared__ __attribute__((aligned(16))) float sU[6][TP];
  static_assert(sizeof(sU) >= 3 * 256 * sizeof(double), "tile_loss_total scratch");
#pragma unroll
  for (int k = 0; k < 5; ++k) sU[k][tid] = u[k];
  __syncthreads();
  tile_fragments(sU, reinterpret_cast<uint4*>(UF) + (size_t)tile * UF_FRAGS, tid, pieces, depth);
  if (l1.tile_loss && l1.loss_out) {  // (tile_loss_sums' stores are write-through)
    __shared__ int last;
    const int tiles = v.tiles_x * v.tiles_y;
    if (arrive_last_tile(ticket, tiles, tile, &last))
      tile_loss_total<true>(l1.tile_loss, tiles, l1.n1, l1.n2, l1.w_sil, l1.t_depth ? l1.n1 / 3 : 0, l1.w_depth,
                            l1.loss_out, reinterpret_cast<double (*)[256]>(&sU[0][0]));
  }
}
__global__ __launch_bounds__(256) void k_pixel_grads(ViewK v, const float4* __restrict__ saved4,
                                                     const float* __restrict__ savedD, const float* __restrict__ g_rgb,
                                                     const float* __restrict__ g_alpha, const float* __restrict__ g_depth,
                                                     uint4* __restrict__ UF, int pieces, L1Args l1, bool depth,
                                                     int* __restrict__ ticket) {
  k_pixel_grads_body(v, saved4, savedD, g_rgb, g_alpha, g_depth, UF, pieces, l1, depth, ticket, BI{(int)blockIdx.x, (int)blockIdx.y}, BI{(int)gridDim.x, (int)gridDim.y});
}
struct k_pixel_grads_args {
  ViewK v;
  const float4* saved4;
  const float* savedD;
  const float* g_rgb;
  const float* g_alpha;
  const float* g_depth;
  uint4* UF;
  int pieces;
  L1Args l1;
  bool depth;
  int* ticket;
};
__global__ __launch_bounds__(256) void k_pixel_grads_views(VBatch<k_pixel_grads_args> B) {
  const int vb = vbatch_view(B, (int)blockIdx.x);
  const k_pixel_grads_args& a = B.a[vb];
  const int lb = (int)blockIdx.x - B.first[vb], gx = B.gx[vb];
  k_pixel_grads_body(a.v, a.saved4, a.savedD, a.g_rgb, a.g_alpha, a.g_depth, a.UF, a.pieces, a.l1, a.depth, a.ticket, BI{lb % gx, lb / gx}, BI{gx, (B.first[vb + 1] - B.first[vb]) / gx});
}


// gr_fwd_render_l1: a finished tile's pixel sums -> the fit loss's upstream fragments (the backward's
// A operands, two pieces, no depth gradient) and the tile's L1 sums, in the forward's epilogue instead
// of a k_pixel_grads pass over saved sums.  `lds` holds >= 4 x TP free floats; every thread of the block
// calls this (two barriers).
__device__ __forceinline__ void l1_tile_epilogue(const ViewK& v, int tile, int tid, const float (&acc)[5], bool inside,
                                                 int p, const L1Args& l1, uint4* __restrict__ UF, float* lds,
                                                 bool fragments = true) {
  float u[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  float l_rgb = 0.f, l_sil = 0.f;
  if (inside)
    pixel_upstream(v, p, make_float4(acc[0], acc[1], acc[2], acc[3]), acc[4], nullptr, nullptr, nullptr, l1, u, l_rgb,
                   l_sil);
  tile_loss_sums(tile, tid, l_rgb, l_sil, l1.tile_loss);  // its barrier also ends every read of lds
  if (!fragments) return;  // uniform per block
  float (*sU)[TP] = reinterpret_cast<float (*)[TP]>(lds);
#pragma unroll
  for (int k = 0; k < 4; ++k) sU[k][tid] = u[k];
  __syncthreads();
  tile_fragments(sU, UF + (size_t)tile * UF_FRAGS, tid, l1.pieces, false);
}

// MODE 1: split bf16, W and D f32-grade; 2: split bf16, W and D within 2^-16 (views rendered with
// no_depth_grad); 3: as 2 without the depth channel (no_depth_grad views rendered with no depth output;
// the saved depth sums are then 0 and unused); 4: as 3, with the fit loss's upstream fragments and tile
// L1 sums made in the epilogue (gr_fwd_render_l1, the fused fit path); 5: the fused fit path at
// f32 grade (no_depth_grad = 2): MODE 1's splits without the depth channel, MODE 4's epilogue with
// three-piece upstream fragments.
// Modes 1/2 at 5 waves per SIMD: at 6 they spill (MODE 1: 5 VGPRs); same-box A/B, C4 depth-loss views,
// MODE 1: 330/334 -> 320/318 us (profiles/r02o_ab_variants.txt).
#ifndef GR_FWD_WAVES
#define GR_FWD_WAVES 5
#endif
#ifndef GR_FWD_WAVES3
#define GR_FWD_WAVES3 6
#endif
template <int MODE>
__device__ __forceinline__ void k_raster_fwd_mfma_body(ViewK v, int n, const int4* __restrict__ items,
                                                         const int* __restrict__ num_items, const int2* __restrict__ ranges,
                                                         const int* __restrict__ pairs, const float4* __restrict__ rec,
                                                         float* __restrict__ fwd_part, float* __restrict__ out_rgb,
                                                         float* __restrict__ out_alpha, float* __restrict__ out_depth,
                                                         float4* __restrict__ saved4, float* __restrict__ savedD,
                                                         L1Args l1, uint4* __restrict__ UF, const int* __restrict__ f16_sa,
                                                         const int* __restrict__ tile_item0, int* __restrict__ ticket,
                                                         int ch, const BI blockIdx, const BI gridDim) {
  // LDS: two staged record buffers (2 x 9 KiB) during the loop, then the 4-wave reduction (20 KiB).
  __shared__ __attribute__((aligned(16))) float smem[4 * 5 * TP];
  __shared__ int last_flag;
  // the non-empty items spread over the XCDs (xcd_item), then the empty tiles' items (background and loss terms)
  const int nitems = num_items[0], nfull = num_items[1];
  if ((int)blockIdx.x >= nitems) return;
  const int item = (int)blockIdx.x < nfull ? xcd_item(blockIdx.x, nfull) : (int)blockIdx.x;
  const int4 it = items[item];
  const int tile = it.x >> 1, k0 = it.y, k1 = it.z;
  const int tx = tile % v.tiles_x, ty = tile / v.tiles_x;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int li = lane & 15, gs = lane >> 4;
  const float xc = (float)(tx * T + li) + 0.5f;  // A row = x
  const float yc = (float)(ty * T + li) + 0.5f;  // B col = y
  f32x4 cW = {0.f, 0.f, 0.f, 0.f}, cR = cW, cG = cW, cB = cW, cD = cW;
  constexpr bool PREC = MODE == 1 || MODE == 5, ZCHK = MODE < 3, F16K = GR_FWD_F16 && (MODE == 3 || MODE == 4);
  const int sa = F16K && f16_sa ? *f16_sa : GR_F16_SA;  // the view's A pre-scale (f16_sa_of; none: no pair to scale)
  if (k1 > k0) {  // (an empty tile's one item has no pair)
    if (it.x & 1)  // tail items: W and D only, two-piece splits (GR_TAIL2)
      fwd_accumulate_bf16<true, PREC && !GR_TAIL2, ZCHK>(smem, n, k0, k1, tid, wave, xc, yc, gs, pairs, rec, cW, cR, cG, cB, cD, (float)sa);
    else
      fwd_accumulate_bf16<false, PREC, ZCHK>(smem, n, k0, k1, tid, wave, xc, yc, gs, pairs, rec, cW, cR, cG, cB, cD, (float)sa);
  }
  if (F16K && !(it.x & 1)) {  // a core item's operands carried 2^sa and 2^SB (exact power-of-two rescale)
    const float sc = __builtin_ldexpf(1.0f, -(sa + GR_F16_SB));
    cW *= sc;
    cR *= sc;
    cG *= sc;
    cB *= sc;
    cD *= sc;
  }
  __syncthreads();
  {  // lane holds C[x = 4*gs + r][y = li]: pixel index y*16 + x, 4 consecutive x
    float* rw = smem + wave * 5 * TP + li * T + 4 * gs;
    *reinterpret_cast<f32x4*>(rw + 0 * TP) = cW;
    *reinterpret_cast<f32x4*>(rw + 1 * TP) = cR;
    *reinterpret_cast<f32x4*>(rw + 2 * TP) = cG;
    *reinterpret_cast<f32x4*>(rw + 3 * TP) = cB;
    *reinterpret_cast<f32x4*>(rw + 4 * TP) = cD;
  }
  __syncthreads();
  float acc[5];
#pragma unroll
  for (int c = 0; c < 5; ++c)
    acc[c] = ((smem[0 * 5 * TP + c * TP + tid] + smem[1 * 5 * TP + c * TP + tid]) + smem[2 * 5 * TP + c * TP + tid]) +
             smem[3 * 5 * TP + c * TP + tid];
  const int nch = tile_chunks(ranges[2 * tile], ch) + tile_chunks(ranges[2 * tile + 1], ch);
  if (nch > 1) {
    // a tile split over several items: each leaves its partial sums (write-through) and takes the tile's ticket;
    // the last to arrive sums every item's partials in item order (deterministic) and finishes the tile
    float* dst = fwd_part + (size_t)item * 5 * TP;
#pragma unroll
    for (int c = 0; c < 5; ++c) st_through(dst + c * TP + tid, acc[c]);
    if (!arrive_last(&ticket[tile], nch, &last_flag)) return;
    const float* src = fwd_part + (size_t)tile_item0[2 * tile] * 5 * TP;
#pragma unroll
    for (int c = 0; c < 5; ++c) acc[c] = 0.f;
    for (int q = 0; q < nch; ++q)
#pragma unroll
      for (int c = 0; c < 5; ++c) acc[c] += ld_through(src + (size_t)q * 5 * TP + c * TP + tid);
    if (tid == 0) ticket[tile] = 0;  // left zero for a later render of the same bins
  }
  const int x = tx * T + (tid & (T - 1)), y = ty * T + (tid >> 4);
  const bool inside = x < v.W && y < v.H && ty >= v.ty0 && ty < v.ty1;  // (a band view: its rows only)
  if (inside) write_pixel(v, y * v.W + x, acc, out_rgb, out_alpha, out_depth, saved4, savedD);
  if constexpr (MODE == 4 || MODE == 5) {
    // an empty tile has no backward work item: only its loss terms are needed, not its fragments
    l1_tile_epilogue(v, tile, tid, acc, inside, y * v.W + x, l1, UF, smem, nch > 0);
    // the view loss: the last tile to finish sums the tiles' L1 sums (tile_loss_total, a fixed order)
    const int tiles = v.tiles_x * v.tiles_y;
    if (arrive_last_tile(ticket, tiles, tile, &last_flag))
      tile_loss_total<true>(l1.tile_loss, tiles, l1.n1, l1.n2, l1.w_sil, 0, 0.0f, l1.loss_out,
                            reinterpret_cast<double (*)[256]>(smem));
  }
}
template <int MODE>
__global__ __launch_bounds__(256, MODE >= 3 ? GR_FWD_WAVES3 : GR_FWD_WAVES) void k_raster_fwd_mfma(ViewK v, int n, const int4* __restrict__ items,
                                                         const int* __restrict__ num_items, const int2* __restrict__ ranges,
                                                         const int* __restrict__ pairs, const float4* __restrict__ rec,
                                                         float* __restrict__ fwd_part, float* __restrict__ out_rgb,
                                                         float* __restrict__ out_alpha, float* __restrict__ out_depth,
                                                         float4* __restrict__ saved4, float* __restrict__ savedD,
                                                         L1Args l1, uint4* __restrict__ UF, const int* __restrict__ f16_sa,
                                                         const int* __restrict__ tile_item0, int* __restrict__ ticket,
                                                         int ch) {
  k_raster_fwd_mfma_body<MODE>(v, n, items, num_items, ranges, pairs, rec, fwd_part, out_rgb, out_alpha, out_depth, saved4, savedD, l1, UF, f16_sa, tile_item0, ticket, ch, BI{(int)blockIdx.x, (int)blockIdx.y}, BI{(int)gridDim.x, (int)gridDim.y});
}
struct k_raster_fwd_mfma_args {
  ViewK v;
  int n;
  const int4* items;
  const int* num_items;
  const int2* ranges;
  const int* pairs;
  const float4* rec;
  float* fwd_part;
  float* out_rgb;
  float* out_alpha;
  float* out_depth;
  float4* saved4;
  float* savedD;
  L1Args l1;
  uint4* UF;
  const int* f16_sa;
  const int* tile_item0;
  int* ticket;
  int ch;
};
template <int MODE>
__global__ __launch_bounds__(256, MODE >= 3 ? GR_FWD_WAVES3 : GR_FWD_WAVES) void k_raster_fwd_mfma_views(VBatch<k_raster_fwd_mfma_args> B) {
  const int vb = vbatch_view(B, (int)blockIdx.x);
  const k_raster_fwd_mfma_args& a = B.a[vb];
  const int lb = (int)blockIdx.x - B.first[vb], gx = B.gx[vb];
  k_raster_fwd_mfma_body<MODE>(a.v, a.n, a.items, a.num_items, a.ranges, a.pairs, a.rec, a.fwd_part, a.out_rgb, a.out_alpha, a.out_depth, a.saved4, a.savedD, a.l1, a.UF, a.f16_sa, a.tile_item0, a.ticket, a.ch, BI{lb % gx, lb / gx}, BI{gx, (B.first[vb + 1] - B.first[vb]) / gx});
}


// Sum over the 4 lane rows (lanes l, l+16, l+32, l+48) of a pair of values with one
// v_permlane16_swap: returns rows {a01, b01, a23, b23} (row r of the result holds the named sum).
__device__ __forceinline__ float pair16(float a, float b) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// Second level with v_permlane32_swap: rows {a, b, c, d} fully reduced from two pair16 results.
__device__ __forceinline__ float pair32(float ab, float cd) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(ab), __float_as_uint(cd), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// ------------------------------------------------------------------------------------------------
// Backward splat, split-precision form: per work item the two contractions
//   T_k[y][g] = sum_x U_k[x][y] ex_g(x),   R_k[x][g] = sum_y U_k[x][y] ey_g(y),
// on v_mfma_f32_32x32x16_bf16 (K = the 16 pixels of a tile row / column, N = 32 Gaussians, M = two
// channels x 16 pixels) with both operands split exactly into three bf16 pieces, x = x0 + x1 + x2,
// and the six products of weight >= 2^-16 accumulated in f32 (smallest first): every dropped
// cross term is below 2^-23 of its product, so the result is as accurate as the f32 contraction.
// An f32 MFMA runs on the vector ALU's issue cycles (it cannot overlap VALU work); a bf16 MFMA is
// 16x the rate and overlaps, so the splitting VALU work is bought back many times.
// A = the tile's upstream vectors, pre-split by k_pixel_grads (UF); B = the Gaussian's exponentials,
// split here.  Lane l (r = l & 31, h = l >> 5) owns Gaussian r of the group and pixels
// kslot_pixel(h, 0..7) on both axes: its B operand for T is ex at those x, for R ey at those y, and
// its accumulator rows of T (R) are exactly those y (x), so each exponential is computed once.
// ------------------------------------------------------------------------------------------------

// A * B over the six significant piece products, smallest first.  A's pieces are read from LDS
// (lane-linear fragments, one ds_read_b128 each) next to their use rather than held in registers:
// that keeps the kernel at 4 waves per SIMD.
__device__ __forceinline__ f32x16 mfma_split(const uint4* __restrict__ A, int lane, const s16x8 (&B)[3]) {
  f32x16 c = {};
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_frag(A[128 + lane]), B[0], c, 0, 0, 0);
  const s16x8 a1 = as_frag(A[64 + lane]);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, B[1], c, 0, 0, 0);
  const s16x8 a0 = as_frag(A[lane]);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, B[2], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, B[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, B[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, B[0], c, 0, 0, 0);
  return c;
}

// A in two round-to-nearest pieces (split2_frag), B in an exact three-piece split: the four products of
// weight >= 2^-17 (a1 b1 ~ 2^-17 is dropped, unbiased: a1 has either sign); the colour channel pairs of
// the depth-gradient backward.
__device__ __forceinline__ f32x16 mfma_split_a2b3(const uint4* __restrict__ A, int lane, const s16x8 (&B)[3]) {
  f32x16 c = {};
  const s16x8 a0 = as_frag(A[lane]);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_frag(A[64 + lane]), B[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, B[2], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, B[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, B[0], c, 0, 0, 0);
  return c;
}

// A * B over two round-to-nearest pieces each (split2_frag; no_depth_grad views): three products.
__device__ __forceinline__ f32x16 mfma_split2(const uint4* __restrict__ A, int lane, const s16x8 (&B)[2]) {
  f32x16 c = {};
  const s16x8 a0 = as_frag(A[lane]);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_frag(A[64 + lane]), B[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, B[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, B[0], c, 0, 0, 0);
  return c;
}

// eight f32 values -> three bf16x8 operand fragments (exact split)
__device__ __forceinline__ void split_frag(const float (&v)[8], s16x8 (&f)[3]) {
  float hi[8], mid[8], lo[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) split3(v[j], hi[j], mid[j], lo[j]);
  f[0] = as_frag(make_uint4(pack_bf16(hi[0], hi[1]), pack_bf16(hi[2], hi[3]), pack_bf16(hi[4], hi[5]), pack_bf16(hi[6], hi[7])));
  f[1] = as_frag(make_uint4(pack_bf16(mid[0], mid[1]), pack_bf16(mid[2], mid[3]), pack_bf16(mid[4], mid[5]),
                            pack_bf16(mid[6], mid[7])));
  f[2] = as_frag(make_uint4(pack_bf16(lo[0], lo[1]), pack_bf16(lo[2], lo[3]), pack_bf16(lo[4], lo[5]), pack_bf16(lo[6], lo[7])));
}

// LDS image of a tile's A fragments in the backward: NPR channel pairs x NPC pieces per side (the full
// 3 x 3 with a depth gradient or three pieces; 2 x 2 for the no-depth two-piece kernel, whose smaller
// footprint lets more blocks share a CU).  Chunk (side, pair, piece) of 64 uint4 at uf_chunk().
template <bool DEPTH, int PIECES>
struct UFLayout {
  static constexpr int NPR = DEPTH ? 3 : 2, NPC = (DEPTH || PIECES == 3) ? 3 : 2;
  static constexpr int CHUNKS = 2 * NPR * NPC;
  __device__ static constexpr int chunk(int side, int pr, int piece) { return (side * NPR + pr) * NPC + piece; }
};

template <bool TAIL, bool DEPTH, int PIECES>
__device__ __forceinline__ void bwd_item_bf16(int n, int k0, int k1, int tid, int wave, int tx, int ty,
                                              const int* __restrict__ pairs, const float4* __restrict__ rec,
                                              float* __restrict__ partials, float4 (*sA)[TP], float4 (*sB)[TP],
                                              float* sZ, const uint4* sUF, float* __restrict__ depth3) {
  using UL = UFLayout<DEPTH, PIECES>;
  static_assert(DEPTH || !TAIL, "tail items carry only depth-coupled terms");
  constexpr int P0 = TAIL ? 2 : 0;      // first channel pair contracted
  constexpr int P1 = DEPTH ? 3 : 2;     // one past the last (pair_channel)
  const int lane = tid & 63, r = lane & 31, h = lane >> 5;
  // pixel centres of the lane's 8 contraction slots (x for T, y for R): base + compile-time offset
  const float pxb = (float)(tx * T + 4 * h) + 0.5f, pyb = (float)(ty * T + 4 * h) + 0.5f;
#define PX0(q) (pxb + (float)((q) < 4 ? (q) : (q) + 4))
#define PY0(q) (pyb + (float)((q) < 4 ? (q) : (q) + 4))
  auto stage = [&](int gid, int b) {
    const float4* p = rec_of(gid, n, rec);
    glds16(p, &sA[b][64 * wave]);
    glds16(p + 1, &sB[b][64 * wave]);
    if constexpr (DEPTH) glds4(zrec_of(gid, n, rec), &sZ[b * TP + 64 * wave]);  // z enters only the depth-coupled terms
  };
  stage(stage_pair(stage_id(k0 + tid, k1, pairs), k0 + tid, k1), 0);
  int idn = stage_id(k0 + TP + tid, k1, pairs);  // raw: batch base + TP
  int buf = 0;
  for (int base = k0; base < k1; base += TP, buf ^= 1) {
    stage_wait();
    GR_STAGE_SYNC();
    if (base + TP < k1) stage(stage_pair(idn, base + TP + tid, k1), buf ^ 1);
    idn = stage_id(base + 2 * TP + tid, k1, pairs);
    const int nb = min(TP, k1 - base);
    for (int gi = 0; gi < 2; ++gi) {
      const int g0 = wave * 64 + gi * 32;
      if (g0 >= nb) break;  // wave-uniform
      const int j = g0 + r;
      const float4 a = sA[buf][j];
      const float4 b = sB[buf][j];
      const float z = DEPTH ? sZ[buf * TP + j] : 0.0f;
      const int myslot = j < nb ? base + j : -1;  // the pair's sorted position = its partial-sum row
      float ex[8], ey[8];
      if constexpr (!DEPTH && PIECES == 2) {
        // the lane's 8 pixel slots sit at constant offsets o_q from its first pixel centre, so the exponent
        // q (d0 + o_q)^2 = q d0^2 + 2 o_q (q d0) + o_q^2 q is two fmas with constant coefficients per slot
        // (instead of a subtraction and two products); rounding ~|q| o_q^2 ulp, well inside the two-piece
        // mode's 2^-16 (padding: q d0^2 = -inf, still exactly 0)
        const float d0x = pxb - a.x, d0y = pyb - a.y;
        const float tx = a.z * d0x, ty = a.w * d0y;
        const float cx = tx * d0x, cy = ty * d0y;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const float oq = (float)(q < 4 ? q : q + 4);
          ex[q] = __builtin_amdgcn_exp2f(q == 0 ? cx : fmaf(tx, 2.0f * oq, fmaf(a.z, oq * oq, cx)));
          ey[q] = __builtin_amdgcn_exp2f(q == 0 ? cy : fmaf(ty, 2.0f * oq, fmaf(a.w, oq * oq, cy)));
        }
      } else {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const float dx = PX0(q) - a.x, dy = PY0(q) - a.y;
          ex[q] = __builtin_amdgcn_exp2f(dx * a.z * dx);  // exactly 0 for padding
          ey[q] = __builtin_amdgcn_exp2f(dy * a.w * dy);
        }
      }
      // -0 starts: -0 + x == x for every x, so the first accumulation folds into a plain product
      float S[NPART] = {-0.f, -0.f, -0.f, -0.f, -0.f, -0.f, -0.f, -0.f, -0.f};
      {
      // both contractions are issued before either epilogue, so the T epilogue's VALU work runs while
      // the R MFMAs execute
      f32x16 DT[3], DR[3];
      if constexpr (PIECES == 3) {
        s16x8 BT[3], BR[3];
        split_frag(ex, BT);
        split_frag(ey, BR);
#pragma unroll
        for (int pr = P0; pr < P1; ++pr)
          DT[pr] = (DEPTH && pr < 2) ? mfma_split_a2b3(sUF + UL::chunk(0, pr, 0) * 64, lane, BT)
                                     : mfma_split(sUF + UL::chunk(0, pr, 0) * 64, lane, BT);
#pragma unroll
        for (int pr = P0; pr < P1; ++pr)
          DR[pr] = (DEPTH && pr < 2) ? mfma_split_a2b3(sUF + UL::chunk(1, pr, 0) * 64, lane, BR)
                                     : mfma_split(sUF + UL::chunk(1, pr, 0) * 64, lane, BR);
      } else {
        s16x8 BT[2], BR[2];
        split2_frag(ex, BT);
        split2_frag(ey, BR);
#pragma unroll
        for (int pr = P0; pr < P1; ++pr) DT[pr] = mfma_split2(sUF + UL::chunk(0, pr, 0) * 64, lane, BT);
#pragma unroll
        for (int pr = P0; pr < P1; ++pr) DR[pr] = mfma_split2(sUF + UL::chunk(1, pr, 0) * 64, lane, BR);
      }
      {
      if constexpr (!DEPTH && PIECES == 2) {
        // Moments about the lane's first pixel centre: dy_q = d0 + o_q with o_q = kslot offset (a compile-
        // time constant), so sum t dy = d0 S4 + sum t o_q and sum t dy^2 = d0^2 S4 + 2 d0 sum t o_q +
        // sum t o_q^2: two constant-coefficient fmas per pixel instead of a subtraction, two products and
        // two sums (the same for dx).  Cancellation is bounded by the tile's 16 px (two-piece mode only).
        const float d0y = pyb - a.y, d0x = pxb - a.x;
        float S6c = -0.f, S8c = -0.f, U0 = -0.f, S5c = -0.f, S7c = -0.f;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const float oq = (float)(q < 4 ? q : q + 4);
          const float T0 = DT[0][q], T1 = DT[0][8 + q], T2 = DT[1][q], T3 = DT[1][8 + q];
          S[0] = fmaf(ey[q], T0, S[0]);
          S[1] = fmaf(ey[q], T1, S[1]);
          S[2] = fmaf(ey[q], T2, S[2]);
          const float t = ey[q] * fmaf(b.w, T2, fmaf(b.z, T1, fmaf(b.y, T0, T3)));
          S[4] += t;
          if (q != 0) {  // slot 0 is the origin of the moments
            S6c = fmaf(t, oq, S6c);
            S8c = fmaf(t, oq * oq, S8c);
          }
          const float u = ex[q] * fmaf(b.w, DR[1][q], fmaf(b.z, DR[0][8 + q], fmaf(b.y, DR[0][q], DR[1][8 + q])));
          U0 += u;
          if (q != 0) {
            S5c = fmaf(u, oq, S5c);
            S7c = fmaf(u, oq * oq, S7c);
          }
        }
        S[6] = fmaf(d0y, S[4], S6c);
        S[8] = fmaf(d0y * d0y, S[4], fmaf(2.0f * d0y, S6c, S8c));
        S[5] = fmaf(d0x, U0, S5c);
        S[7] = fmaf(d0x * d0x, U0, fmaf(2.0f * d0x, S5c, S7c));
      } else {
      // T: rows y = kslot_pixel(h, q) of channels pair_channel(pr, c) at register 8c + q
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float dy = PY0(q) - a.y;
        float GT;
        if constexpr (!DEPTH) {  // T4 = 0
          const float T0 = DT[0][q], T1 = DT[0][8 + q], T2 = DT[1][q], T3 = DT[1][8 + q];
          S[0] = fmaf(ey[q], T0, S[0]);
          S[1] = fmaf(ey[q], T1, S[1]);
          S[2] = fmaf(ey[q], T2, S[2]);
          GT = fmaf(b.w, T2, fmaf(b.z, T1, fmaf(b.y, T0, T3)));
        } else if constexpr (TAIL) {
          const float T3 = DT[2][q], T4 = DT[2][8 + q];
          GT = fmaf(z, T4, T3);
          S[3] = fmaf(ey[q], T4, S[3]);
        } else {
          const float T0 = DT[0][q], T1 = DT[0][8 + q], T2 = DT[1][q], T3 = DT[2][q], T4 = DT[2][8 + q];
          S[0] = fmaf(ey[q], T0, S[0]);
          S[1] = fmaf(ey[q], T1, S[1]);
          S[2] = fmaf(ey[q], T2, S[2]);
          GT = fmaf(z, T4, fmaf(b.w, T2, fmaf(b.z, T1, fmaf(b.y, T0, T3))));
          S[3] = fmaf(ey[q], T4, S[3]);
        }
        const float t = ey[q] * GT;
        S[4] += t;
        const float tdy = t * dy;
        S[6] += tdy;
        S[8] = fmaf(tdy, dy, S[8]);
      }
      // R: rows x = kslot_pixel(h, q)
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float dx = PX0(q) - a.x;
        float GR;
        if constexpr (!DEPTH) {
          GR = fmaf(b.w, DR[1][q], fmaf(b.z, DR[0][8 + q], fmaf(b.y, DR[0][q], DR[1][8 + q])));
        } else if constexpr (TAIL) {
          GR = fmaf(z, DR[2][8 + q], DR[2][q]);
        } else {
          GR = fmaf(z, DR[2][8 + q], fmaf(b.w, DR[1][q], fmaf(b.z, DR[0][8 + q], fmaf(b.y, DR[0][q], DR[2][q]))));
        }
        const float tdx = (ex[q] * GR) * dx;  // (0 * G) * dx: padding stays 0, never 0 * inf
        S[5] += tdx;
        S[7] = fmaf(tdx, dx, S[7]);
      }
      }
      }
      }
      // lanes r and r + 32 hold the two halves of Gaussian r's pixels; pair32 leaves half 0 with the
      // total of its first argument, half 1 with that of its second
      if constexpr (!DEPTH) {
        // S3 (the depth sum) is zero: 8-float rows ROW8 = [o S0, o S2, S4, S6 | o S1, S8, S5, S7], half h
        // writes float4 h: one aligned, fully coalesced 16-byte store per lane (32 rows = 1 KiB)
        const float Pa = pair32(S[0], S[1]), Pb = pair32(S[2], S[8]), Pc = pair32(S[4], S[5]);
        const float Pd = pair32(S[6], S[7]);
        if (myslot >= 0)
          reinterpret_cast<float4*>(partials)[2 * (size_t)myslot + h] =
              h == 0 ? make_float4(b.x * Pa, b.x * Pb, Pc, Pd) : make_float4(b.x * Pa, Pb, Pc, Pd);
      } else {
        // half 0 ends with the totals of S0, S2, S4, S6, S8, half 1 with S1, S3, S5, S7, S8: the same
        // 32-byte rows as without a depth gradient (float4 h of the row), the depth sum o S3 in its own
        // array behind the rows (depth3[slot]), so the gather reads aligned rows either way
        const float P01 = pair32(S[0], S[1]), P23 = pair32(S[2], S[3]), P45 = pair32(S[4], S[5]);
        const float P67 = pair32(S[6], S[7]), P8 = pair32(S[8], S[8]);
        if (myslot >= 0) {  // colour / depth sums carry the opacity
          reinterpret_cast<float4*>(partials)[2 * (size_t)myslot + h] =
              h == 0 ? make_float4(b.x * P01, b.x * P23, P45, P67) : make_float4(b.x * P01, P8, P45, P67);
          if (h == 1) depth3[myslot] = b.x * P23;
        }
      }
    }
  }
#undef PX0
#undef PY0
}

#ifndef GR_BF16_WAVES
#define GR_BF16_WAVES 3  // 168 VGPRs (one spilled) instead of 170 at 2 waves: default mode +3.5% (C4d 600 -> 619)
#endif
#ifndef GR_BF16_WAVES_ND
#define GR_BF16_WAVES_ND 2
#endif

// DEPTH = 0: no upstream depth gradient (4 channels, tail items skipped) — its own kernel, so its
// register budget is not set by the 5-channel form's.
// PIECES = 2: no_depth_grad views (two round-to-nearest pieces per operand, three products).
template <bool DEPTH, int PIECES>
__device__ __forceinline__ void k_raster_bwd_bf16_body(ViewK v, int n, const int4* __restrict__ items,
                                                           const int* __restrict__ num_items, const int* __restrict__ pairs,
                                                           const float4* __restrict__ rec, const uint4* __restrict__ UF,
                                                           float* __restrict__ partials, float* __restrict__ depth3, const BI blockIdx, const BI gridDim) {
  using UL = UFLayout<DEPTH, PIECES>;
  __shared__ __attribute__((aligned(16))) float4 sA[2][TP];
  __shared__ __attribute__((aligned(16))) float4 sB[2][TP];
  __shared__ float sZ[2][DEPTH ? TP : 1];
  __shared__ __attribute__((aligned(16))) uint4 sUF[UL::CHUNKS * 64];
  const int nitems = num_items[1];  // the non-empty items (listed first): an empty tile has nothing to differentiate
  if ((int)blockIdx.x >= nitems) return;
  const int item = xcd_item(blockIdx.x, nitems);
  const int4 it = items[item];
  const bool tail = it.x & 1;
  if (tail && !DEPTH) return;
  const int tile = it.x >> 1, k0 = it.y, k1 = it.z;
  if (k1 <= k0) return;  // an empty tile's item: nothing to differentiate
  const int tx = tile % v.tiles_x, ty = tile / v.tiles_x;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  {  // the tile's A fragments this item contracts -> LDS (DMA): chunk (side * 3 + pair) * 3 + piece
    const uint4* src = UF + (size_t)tile * UF_FRAGS;
    const int p0 = tail ? 2 : 0, p1 = DEPTH ? 3 : 2;
    for (int cc = wave; cc < UL::CHUNKS; cc += 4) {
      const int side = cc / (UL::NPR * UL::NPC), pr = (cc / UL::NPC) % UL::NPR, piece = cc % UL::NPC;
      const int c = (side * 3 + pr) * 3 + piece;  // chunk of the tile's full image (tile_fragments)
      if (piece < PIECES && pr >= p0 && pr < p1) glds16(src + 64 * c + lane, sUF + 64 * cc);
    }
    stage_wait();
    __syncthreads();
  }
  if constexpr (!DEPTH)
    bwd_item_bf16<false, false, PIECES>(n, k0, k1, tid, wave, tx, ty, pairs, rec, partials, sA, sB, &sZ[0][0], sUF, depth3);
  else if (tail)  // the tail's depth-coupled pair on two-piece operands (GR_TAIL2)
    bwd_item_bf16<true, true, GR_TAIL2 ? 2 : PIECES>(n, k0, k1, tid, wave, tx, ty, pairs, rec, partials, sA, sB, &sZ[0][0], sUF, depth3);
  else
    bwd_item_bf16<false, true, PIECES>(n, k0, k1, tid, wave, tx, ty, pairs, rec, partials, sA, sB, &sZ[0][0], sUF, depth3);
}
template <bool DEPTH, int PIECES>
__global__ __launch_bounds__(256, DEPTH ? GR_BF16_WAVES : GR_BF16_WAVES_ND) void k_raster_bwd_bf16(ViewK v, int n, const int4* __restrict__ items,
                                                           const int* __restrict__ num_items, const int* __restrict__ pairs,
                                                           const float4* __restrict__ rec, const uint4* __restrict__ UF,
                                                           float* __restrict__ partials, float* __restrict__ depth3) {
  k_raster_bwd_bf16_body<DEPTH, PIECES>(v, n, items, num_items, pairs, rec, UF, partials, depth3, BI{(int)blockIdx.x, (int)blockIdx.y}, BI{(int)gridDim.x, (int)gridDim.y});
}
struct k_raster_bwd_bf16_args {
  ViewK v;
  int n;
  const int4* items;
  const int* num_items;
  const int* pairs;
  const float4* rec;
  const uint4* UF;
  float* partials;
  float* depth3;
};
template <bool DEPTH, int PIECES>
__global__ __launch_bounds__(256, DEPTH ? GR_BF16_WAVES : GR_BF16_WAVES_ND) void k_raster_bwd_bf16_views(VBatch<k_raster_bwd_bf16_args> B) {
  const int vb = vbatch_view(B, (int)blockIdx.x);
  const k_raster_bwd_bf16_args& a = B.a[vb];
  const int lb = (int)blockIdx.x - B.first[vb], gx = B.gx[vb];
  k_raster_bwd_bf16_body<DEPTH, PIECES>(a.v, a.n, a.items, a.num_items, a.pairs, a.rec, a.UF, a.partials, a.depth3, BI{lb % gx, lb / gx}, BI{gx, (B.first[vb + 1] - B.first[vb]) / gx});
}


// k_fwd32_l1 at 4 waves/SIMD with its record fields loaded axis by axis (116 VGPRs, no spill);
// loading all five fields up front needs 124 VGPRs (3 waves; 15 spilled at 4).  Same box, three rounds each:
// forward 161-165 -> 160-162 us, step +0.6% (profiles/r05_ab_fwd32_stream.txt)
#ifndef GR_FWD32_WAVES
#define GR_FWD32_WAVES 4
#endif
#ifndef GR_BWD32_WAVES
#define GR_BWD32_WAVES 3
#endif
#ifndef GR_BWD32_BATCH
#define GR_BWD32_BATCH 256
#endif
// phase fences of k_bwd32 (GR_BWD32_FENCE = 1): the compiler may not move instructions across them, so a pass's
// MFMAs are not hoisted above the previous pass's epilogue (which would keep every accumulator live at once)
#ifndef GR_BWD32_FENCE
#define GR_BWD32_FENCE 1
#endif
#if GR_BWD32_FENCE
#define GR_BWD32_PHASE() __builtin_amdgcn_sched_barrier(0)
#else
#define GR_BWD32_PHASE() ((void)0)
#endif
// ================================================================================================
// 32-pixel tiles (gr_view.tile = 32): the fused fit path's forward (gr_fwd_render_l1, no_depth_grad = 1) and
// backward splat (gr_bwd_splat).  With a ~3-pixel sigma the 5-sigma footprint spans ~32 pixels: 16-pixel tiles
// give 7.8 (Gaussian, tile) pairs per Gaussian at C4, 32-pixel tiles 3.7, so the binning, the per-pair gradient
// rows and their gather halve, while the separable splat's per-Gaussian slot work (exponentials, operand splits,
// epilogue) stays the same: ~32 x and ~32 y slots per Gaussian either way.  The contractions move
// to v_mfma_f32_32x32x16 with M = 32 pixels of ONE channel (the 16-pixel kernels pack two channels of 16).
// Operand layout of v_mfma_f32_32x32x16_{f16,bf16} (gfx950): lane l (r = l & 31, h = l >> 5) supplies
// A[m = r][k = kslot_pixel(h, j)] and B[k = kslot_pixel(h, j)][n = r], j = 0..7, and holds D[m][n = r] for
// m = 16 (i >> 3) + kslot_pixel(h, i & 7), i = 0..15 — so with K = 16 pixels per step s (pixel 16 s + k) the
// rows a lane holds are exactly the pixels whose exponentials it computed for its own B operands.
// ================================================================================================
constexpr int F32_PLANES = 8;  // staged record fields (px py qx qy o r g b): no depth channel on the fit path
constexpr int F32_BUF = F32_PLANES * TP;  // floats per staging buffer (256 Gaussians)
constexpr int F32_LD = T32 + 1;            // padded row of the forward's reduction / upstream tiles in LDS
__device__ __forceinline__ f32x16 mfma32h(const s16x8& a, const s16x8& b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8_t, a), __builtin_bit_cast(f16x8_t, b), c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 mfma32b(const s16x8& a, const s16x8& b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
// offset of kslot j from the lane's first slot (kslot_pixel(h, j) - 4 h)
__device__ __forceinline__ constexpr int kslot_off(int j) { return j < 4 ? j : j + 4; }

// Forward of one work item of a 32-pixel tile: every wave contracts its 64 Gaussians of each 256-Gaussian batch
// over the whole tile (4 K-steps of 16 per batch), C_k[x][y] += sum_g A_k[x][g] B[g][y] with A = o v_k ex * 2^sa
// (v = 1, r, g, b) and B = ey * 2^SB on f16 two-piece operands (split2h_frag2, MODE 4's precision), four f32x16
// accumulators per lane.  The four waves' sums meet in LDS (fixed wave order), a split tile's items through the
// write-through partials of the last item to arrive (item order), then the L1 epilogue per pixel (four pixels per
// thread), the backward's upstream fragments (UF32) and the view loss by the last tile (as k_raster_fwd_mfma<4>).
__device__ __forceinline__ void k_fwd32_l1_body(ViewK v, int n, const int4* __restrict__ items,
                                                                 const int* __restrict__ num_items,
                                                                 const int2* __restrict__ ranges, const int* __restrict__ pairs,
                                                                 const float4* __restrict__ rec, float* __restrict__ fwd_part,
                                                                 float* __restrict__ out_rgb, float* __restrict__ out_alpha,
                                                                 L1Args l1, uint4* __restrict__ UF, const int* __restrict__ f16_sa,
                                                                 const int* __restrict__ tile_item0, int* __restrict__ ticket,
                                                                 int ch, const BI blockIdx, const BI gridDim) {
  // LDS: the staged batches (2 x 8 planes x 256 floats) during the loop; then the waves' sums of two channels
  // (4 waves x 2 x 32 x 33); then the tile's upstream vectors (4 x 32 x 33); then the view loss's double[3][256]
  __shared__ __attribute__((aligned(16))) float smem[4 * 2 * T32 * F32_LD];
  static_assert(sizeof(smem) >= 2 * F32_BUF * sizeof(float) && sizeof(smem) >= 3 * 256 * sizeof(double), "k_fwd32_l1 LDS");
  __shared__ int last_flag;
  const int nitems = num_items[0], nfull = num_items[1];
  if ((int)blockIdx.x >= nitems) return;
  const int item = (int)blockIdx.x < nfull ? xcd_item(blockIdx.x, nfull) : (int)blockIdx.x;
  const int4 it = items[item];
  const int tile = it.x >> 1, k0 = it.y, k1 = it.z;
  const int tx = tile % v.tiles_x, ty = tile / v.tiles_x;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
  const int sa = f16_sa ? *f16_sa : GR_F16_SA;
  f32x16 cW = {}, cR = {}, cG = {}, cB = {};
  if (k1 > k0) {
    auto stage = [&](int g, int b) { glds4_planes<false, false>(rec_of(g, n, rec), nullptr, smem + b * F32_BUF + 64 * wave); };
    stage(stage_pair(stage_id(k0 + tid, k1, pairs), k0 + tid, k1), 0);
    int idn = stage_id(k0 + TP + tid, k1, pairs);
    int buf = 0;
    const float xc = (float)(tx * T32 + r) + 0.5f, yc = (float)(ty * T32 + r) + 0.5f;  // A row x, B column y
    const f32x2_t X = {xc, xc}, Y = {yc, yc}, SA = {(float)sa, (float)sa}, SB = {(float)GR_F16_SB, (float)GR_F16_SB};
    for (int base = k0; base < k1; base += TP, buf ^= 1) {
      stage_wait();
      if (base + TP < k1) stage(stage_pair(idn, base + TP + tid, k1), buf ^ 1);
      idn = stage_id(base + 2 * TP + tid, k1, pairs);
      const int cnt = min(TP, k1 - base) - wave * 64;
      const int nks = cnt <= 0 ? 0 : min(4, (cnt + 15) >> 4);  // K-steps of 16 (padding records are zero)
      for (int ks = 0; ks < nks; ++ks) {
        // this lane's 8 Gaussians of the K-step: kslot_pixel(h, 0..7) = 4h + {0..3} and 8 + 4h + {0..3}
        const float* s = smem + buf * F32_BUF + wave * 64 + ks * 16 + 4 * h;
        auto ld = [&](int f, f32x2_t (&q)[4]) {
          const float4 u0 = *reinterpret_cast<const float4*>(s + f * TP);
          const float4 u1 = *reinterpret_cast<const float4*>(s + f * TP + 8);
          q[0] = f32x2_t{u0.x, u0.y};
          q[1] = f32x2_t{u0.z, u0.w};
          q[2] = f32x2_t{u1.x, u1.y};
          q[3] = f32x2_t{u1.z, u1.w};
        };
        f32x2_t oe[4], bv[4];
        // the record fields loaded axis by axis behind scheduling fences (fewer live registers: 4 waves/SIMD)
        {
          f32x2_t px[4], qx[4], o[4];
          ld(0, px);
          ld(2, qx);
          ld(4, o);
#pragma unroll
          for (int p = 0; p < 4; ++p) {
            const f32x2_t dx = X - px[p];
            const f32x2_t ax = __builtin_elementwise_fma(dx * qx[p], dx, SA);
            const f32x2_t ex = {__builtin_amdgcn_exp2f(ax.x), __builtin_amdgcn_exp2f(ax.y)};
            oe[p] = o[p] * ex;
          }
        }
        __builtin_amdgcn_sched_barrier(0);
        {
          f32x2_t py[4], qy[4];
          ld(1, py);
          ld(3, qy);
#pragma unroll
          for (int p = 0; p < 4; ++p) {
            const f32x2_t dy = Y - py[p];
            const f32x2_t ay = __builtin_elementwise_fma(dy * qy[p], dy, SB);
            bv[p] = f32x2_t{__builtin_amdgcn_exp2f(ay.x), __builtin_amdgcn_exp2f(ay.y)};
          }
        }
        __builtin_amdgcn_sched_barrier(0);
        s16x8 fb[2], fa[2];
        split2h_frag2(bv, fb);
        split2h_frag2(oe, fa);
        cW = mfma32h(fa[1], fb[0], cW);
        cW = mfma32h(fa[0], fb[1], cW);
        cW = mfma32h(fa[0], fb[0], cW);
        f32x2_t c[4], a[4];
#define GR_FWD32_CH(F, ACC)                                   \
  ld(F, c);                                                   \
  _Pragma("unroll") for (int p = 0; p < 4; ++p) a[p] = oe[p] * c[p]; \
  split2h_frag2(a, fa);                                       \
  ACC = mfma32h(fa[1], fb[0], ACC);                           \
  ACC = mfma32h(fa[0], fb[1], ACC);                           \
  ACC = mfma32h(fa[0], fb[0], ACC);
        GR_FWD32_CH(5, cR)
        GR_FWD32_CH(6, cG)
        GR_FWD32_CH(7, cB)
#undef GR_FWD32_CH
      }
    }
    const float sc = __builtin_ldexpf(1.0f, -(sa + GR_F16_SB));  // the operands carried 2^sa and 2^SB (exact)
    cW *= sc;
    cR *= sc;
    cG *= sc;
    cB *= sc;
  }
  // the four waves' sums, two channels per round: wave w's rows x = 16 (i >> 3) + kslot_pixel(h, i & 7) of column y = r
  const int px0 = tid & 31, py0 = tid >> 5;  // this thread's pixels (px0, py0 + 8 q), q = 0..3
  float acc[4][4];                           // [pixel q][W, R, G, B]
#pragma unroll
  for (int round = 0; round < 2; ++round) {
    __syncthreads();  // the staging buffers (round 0) / the previous round's reads (round 1) are done
    const f32x16& c0 = round == 0 ? cW : cG;
    const f32x16& c1 = round == 0 ? cR : cB;
    float* w0 = smem + (wave * 2) * T32 * F32_LD;
    float* w1 = w0 + T32 * F32_LD;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int x = 16 * (i >> 3) + kslot_pixel(h, i & 7);
      w0[x * F32_LD + r] = c0[i];
      w1[x * F32_LD + r] = c1[i];
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int a = px0 * F32_LD + py0 + 8 * q;
#pragma unroll
      for (int cc = 0; cc < 2; ++cc) {
        const float* b = smem + cc * T32 * F32_LD + a;
        acc[q][2 * round + cc] = ((b[0] + b[2 * T32 * F32_LD]) + b[4 * T32 * F32_LD]) + b[6 * T32 * F32_LD];
      }
    }
  }
  const int nch = tile_chunks(ranges[2 * tile], ch) + tile_chunks(ranges[2 * tile + 1], ch);
  if (nch > 1) {
    // a tile split over several items: each leaves its partial sums (write-through) and takes the tile's ticket; the
    // last to arrive sums every item's partials in item order (deterministic) and finishes the tile.  An item's
    // partials are four float4 planes (plane q: thread t's four channels of its pixel q at 16 t bytes), so each of a
    // thread's four 16-byte write-through stores is part of one contiguous 4 KB block per instruction
    const __amdgpu_buffer_rsrc_t dst = through_rsrc(fwd_part + (size_t)item * 4 * TP32);
#pragma unroll
    for (int q = 0; q < 4; ++q) st_through16(dst, 16 * (256 * q + tid), make_float4(acc[q][0], acc[q][1], acc[q][2], acc[q][3]));
    if (!arrive_last(&ticket[tile], nch, &last_flag)) return;
    const __amdgpu_buffer_rsrc_t src = through_rsrc(fwd_part + (size_t)tile_item0[2 * tile] * 4 * TP32);
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[q][c] = 0.f;
    for (int e = 0; e < nch; ++e)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 pv = ld_through16(src, 4 * 4 * TP32 * e + 16 * (256 * q + tid));
        acc[q][0] += pv.x;
        acc[q][1] += pv.y;
        acc[q][2] += pv.z;
        acc[q][3] += pv.w;
      }
    if (tid == 0) ticket[tile] = 0;  // left zero for a later render of the same bins
  }
  // per pixel: outputs, the L1 terms and the upstream vector u = (dC_r, dC_g, dC_b, dW)
  float u[4][5];
  float l_rgb = 0.f, l_sil = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int x = tx * T32 + px0, y = ty * T32 + py0 + 8 * q;
#pragma unroll
    for (int c = 0; c < 5; ++c) u[q][c] = 0.f;
    if (x < v.W && y < v.H && ty >= v.ty0 && ty < v.ty1) {  // (a band view: its rows only)
      const int p = y * v.W + x;
      const float a5[5] = {acc[q][0], acc[q][1], acc[q][2], acc[q][3], 0.0f};
      write_pixel(v, p, a5, out_rgb, out_alpha, nullptr, nullptr, nullptr);
      float lr = 0.f, ls = 0.f;
      pixel_upstream(v, p, make_float4(acc[q][0], acc[q][1], acc[q][2], acc[q][3]), 0.0f, nullptr, nullptr, nullptr, l1,
                     u[q], lr, ls);
      l_rgb += lr;
      l_sil += ls;
    }
  }
  tile_loss_sums(tile, tid, l_rgb, l_sil, l1.tile_loss);  // (its barrier ends every read of smem above)
  if (nch > 0) {  // an empty tile has no backward work item: no fragments
    float* sU = smem;  // [channel][x][y], rows of F32_LD
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int c = 0; c < 4; ++c) sU[c * T32 * F32_LD + px0 * F32_LD + py0 + 8 * q] = u[q][c];
    __syncthreads();
    // the f16 operand scales from the L1 upstream's bounds (pixel_upstream, den = 1 + W >= 1): |dC_c| <= g / (3 HW),
    // |dW| <= 3 g / (3 HW) + w_sil g / HW; a pixel's value sits 1 / (1 + W) below its bound, so both f16 pieces stay
    // normal while W < 2^16 (f16_exp_of)
    const float HWf = (float)v.W * (float)v.H, gC = fabsf(l1.g_scale) / (3.0f * HWf);
    const int eC = f16_exp_of(gC), eWb = f16_exp_of(3.0f * gC + fabsf(l1.w_sil * l1.g_scale) / HWf);
    const int ex4[4] = {eC, eC, eC, eWb};
    // fragment set (side, channel, K-step s), lane l: side 0 (T, contraction over x) A[m = y][k] = U[x = 16 s + k][y],
    // side 1 (R, over y) A[m = x][k] = U[x][y = 16 s + k], k = kslot_pixel(h, j); U * 2^e_c in two round-to-nearest
    // f16 pieces (split2h_frag), the exponents e_c after the fragments
    uint4* fr = UF + (size_t)tile * UF32_STRIDE;
    if (tid == 0) fr[UF32_FRAGS] = make_uint4((unsigned)ex4[0], (unsigned)ex4[1], (unsigned)ex4[2], (unsigned)ex4[3]);
    for (int e = tid; e < 16 * 64; e += 256) {
      const int set = e >> 6, l = e & 63, side = set >> 3, c = (set >> 1) & 3, s = set & 1;
      const int sc = c == 0 ? ex4[0] : (c == 1 ? ex4[1] : (c == 2 ? ex4[2] : ex4[3]));
      float val[8];
      const int m = l & 31, hh = l >> 5;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 16 * s + kslot_pixel(hh, j);
        val[j] = ldexpf(side == 0 ? sU[c * T32 * F32_LD + k * F32_LD + m] : sU[c * T32 * F32_LD + m * F32_LD + k], sc);
      }
      s16x8 f2[2];
      split2h_frag(val, f2);
      __builtin_memcpy(&fr[(set * 2 + 0) * 64 + l], &f2[0], 16);
      __builtin_memcpy(&fr[(set * 2 + 1) * 64 + l], &f2[1], 16);
    }
  }
  // the view loss: the last tile to finish sums the tiles' L1 sums (tile_loss_total, a fixed order)
  const int tiles = v.tiles_x * v.tiles_y;
  if (arrive_last_tile(ticket, tiles, tile, &last_flag))
    tile_loss_total<true>(l1.tile_loss, tiles, l1.n1, l1.n2, l1.w_sil, 0, 0.0f, l1.loss_out,
                          reinterpret_cast<double (*)[256]>(smem));
}
__global__ __launch_bounds__(256, GR_FWD32_WAVES) void k_fwd32_l1(ViewK v, int n, const int4* __restrict__ items,
                                                                 const int* __restrict__ num_items,
                                                                 const int2* __restrict__ ranges, const int* __restrict__ pairs,
                                                                 const float4* __restrict__ rec, float* __restrict__ fwd_part,
                                                                 float* __restrict__ out_rgb, float* __restrict__ out_alpha,
                                                                 L1Args l1, uint4* __restrict__ UF, const int* __restrict__ f16_sa,
                                                                 const int* __restrict__ tile_item0, int* __restrict__ ticket,
                                                                 int ch) {
  k_fwd32_l1_body(v, n, items, num_items, ranges, pairs, rec, fwd_part, out_rgb, out_alpha, l1, UF, f16_sa, tile_item0, ticket, ch, BI{(int)blockIdx.x, (int)blockIdx.y}, BI{(int)gridDim.x, (int)gridDim.y});
}
struct k_fwd32_l1_args {
  ViewK v;
  int n;
  const int4* items;
  const int* num_items;
  const int2* ranges;
  const int* pairs;
  const float4* rec;
  float* fwd_part;
  float* out_rgb;
  float* out_alpha;
  L1Args l1;
  uint4* UF;
  const int* f16_sa;
  const int* tile_item0;
  int* ticket;
  int ch;
};
__global__ __launch_bounds__(256, GR_FWD32_WAVES) void k_fwd32_l1_views(VBatch<k_fwd32_l1_args> B) {
  const int vb = vbatch_view(B, (int)blockIdx.x);
  const k_fwd32_l1_args& a = B.a[vb];
  const int lb = (int)blockIdx.x - B.first[vb], gx = B.gx[vb];
  k_fwd32_l1_body(a.v, a.n, a.items, a.num_items, a.ranges, a.pairs, a.rec, a.fwd_part, a.out_rgb, a.out_alpha, a.l1, a.UF, a.f16_sa, a.tile_item0, a.ticket, a.ch, BI{lb % gx, lb / gx}, BI{gx, (B.first[vb + 1] - B.first[vb]) / gx});
}


// Backward of one work item of a 32-pixel tile (no upstream depth gradient): per group of 32 Gaussians (lane
// r = l & 31 owns Gaussian r, half h = l >> 5 its slots kslot_pixel(h, .) of each 16-pixel K-step s) the contractions
//   T_c[y][g] = sum_x U_c[x][y] ex_g(x)   and   R_c[x][g] = sum_y U_c[x][y] ey_g(y),   c = dC_r, dC_g, dC_b, dW,
// each 2 K-steps x 3 piece products on v_mfma_f32_32x32x16_f16 (round 6: two round-to-nearest f16 pieces, U scaled
// by 2^e_c per channel and ex / ey by 2^SB into f16's normal range, <= 3 * 2^-22 per product; the bf16 pieces before
// left ~2^-16), then the per-Gaussian epilogue over the lane's 16 rows (the same sums as the 16-pixel kernel, moments
// about the first slot of each K-step) and the 8-float row [o S0, o S2, S4, S6 | o S1, S8, S5, S7] at the pair's
// sorted position (the gather is unchanged).  Same-box A/B at C4 vs the bf16 phased form: backward 219-223 ->
// 212-216 us, step +1.5-2% (profiles/r06_ab_bwd32_f16.txt).
__device__ __forceinline__ void k_bwd32_body(ViewK v, int n, const int4* __restrict__ items,
                                                              const int* __restrict__ num_items, const int* __restrict__ pairs,
                                                              const float4* __restrict__ rec, const uint4* __restrict__ UF,
                                                              float* __restrict__ partials, const BI blockIdx, const BI gridDim) {
  constexpr int NB = GR_BWD32_BATCH;  // Gaussians staged per batch (NB / 4 per wave)
  constexpr int WG = NB / 4;          // per wave: one or two groups of 32
  __shared__ __attribute__((aligned(16))) float4 sA[2][NB];
  __shared__ __attribute__((aligned(16))) float4 sB[2][NB];
  __shared__ __attribute__((aligned(16))) uint4 sUF[2 * 4 * 2 * 2 * 64];  // (side, channel, s, piece) x 64 lanes
  const int nitems = num_items[1];
  if ((int)blockIdx.x >= nitems) return;
  const int item = xcd_item(blockIdx.x, nitems);
  const int4 it = items[item];
  const int tile = it.x >> 1, k0 = it.y, k1 = it.z;
  if (k1 <= k0) return;
  const int tx = tile % v.tiles_x, ty = tile / v.tiles_x;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
  {  // the tile's 32 fragment chunks -> LDS (DMA)
    const uint4* src = UF + (size_t)tile * UF32_STRIDE;
    for (int cc = wave; cc < 32; cc += 4) glds16(src + 64 * cc + lane, sUF + 64 * cc);
  }
  // the fragments' per-channel exponents (f16_exp_of): the contractions carry U 2^e_c and the B operands 2^SB
  const uint4 e4 = UF[(size_t)tile * UF32_STRIDE + UF32_FRAGS];
  const int eC0 = (int)e4.x, eC1 = (int)e4.y, eC2 = (int)e4.z, eW = (int)e4.w;
  // pixel centres of the lane's first slot per K-step: base + kslot offsets (compile-time)
  const float pxb[2] = {(float)(tx * T32 + 4 * h) + 0.5f, (float)(tx * T32 + 16 + 4 * h) + 0.5f};
  const float pyb[2] = {(float)(ty * T32 + 4 * h) + 0.5f, (float)(ty * T32 + 16 + 4 * h) + 0.5f};
  {  // the first batch (lanes < WG stage this wave's WG Gaussians)
    const int k = k0 + wave * WG + (lane < WG ? lane : 0);
    if (lane < WG) {
      const int gid = stage_pair(stage_id(k, k1, pairs), k, k1);
      glds16(rec_of(gid, n, rec), &sA[0][WG * wave]);
      glds16(rec_of(gid, n, rec) + 1, &sB[0][WG * wave]);
    }
  }
  int idn = stage_id(k0 + NB + wave * WG + (lane < WG ? lane : 0), k1, pairs);
  int buf = 0;
  for (int base = k0; base < k1; base += NB, buf ^= 1) {
    stage_wait();
    if (base == k0) __syncthreads();  // the fragment chunks (every wave's DMA) are in LDS
    if (base + NB < k1 && lane < WG) {
      const int gid = stage_pair(idn, base + NB + wave * WG + lane, k1);
      glds16(rec_of(gid, n, rec), &sA[buf ^ 1][WG * wave]);
      glds16(rec_of(gid, n, rec) + 1, &sB[buf ^ 1][WG * wave]);
    }
    idn = stage_id(base + 2 * NB + wave * WG + (lane < WG ? lane : 0), k1, pairs);
    const int nb = min(NB, k1 - base);
    for (int gi = 0; gi < WG / 32; ++gi) {
      const int g0 = wave * WG + gi * 32;
      if (g0 >= nb) break;  // wave-uniform
      const int j = g0 + r;
      const float4 a = sA[buf][j];
      const float4 b = sB[buf][j];
      const int myslot = j < nb ? base + j : -1;
      // exponentials of the lane's 8 slots per K-step (moments about the first slot: two constant fmas per slot)
      float ex[2][8], ey[2][8], d0x[2], d0y[2];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        d0x[s] = pxb[s] - a.x;
        d0y[s] = pyb[s] - a.y;
        const float tX = a.z * d0x[s], tY = a.w * d0y[s];
        // ex, ey by 2^SB (the f16 B operands' range, as k_fwd32_l1's ey); the epilogue's weights carry it too
        const float cX = fmaf(tX, d0x[s], (float)GR_F16_SB), cY = fmaf(tY, d0y[s], (float)GR_F16_SB);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const float oq = (float)kslot_off(q);
          ex[s][q] = __builtin_amdgcn_exp2f(q == 0 ? cX : fmaf(tX, 2.0f * oq, fmaf(a.z, oq * oq, cX)));
          ey[s][q] = __builtin_amdgcn_exp2f(q == 0 ? cY : fmaf(tY, 2.0f * oq, fmaf(a.w, oq * oq, cY)));
        }
      }
      float S[NPART] = {-0.f, -0.f, -0.f, -0.f, -0.f, -0.f, -0.f, -0.f, -0.f};
      float S4s[2] = {-0.f, -0.f}, S6c[2] = {-0.f, -0.f}, S8c[2] = {-0.f, -0.f};
      float U0[2] = {-0.f, -0.f}, S5c[2] = {-0.f, -0.f}, S7c[2] = {-0.f, -0.f};
      // one channel's contraction on one side (side 0: T over x with B = ex pieces, side 1: R over y with B = ey
      // pieces): 2 K-steps x 3 piece products (a_lo b_hi, a_hi b_lo, a_hi b_hi)
      auto contract = [&](int side, int c, const s16x8 (&B)[2][2]) {
        const uint4* A0 = sUF + ((side * 4 + c) * 2 + 0) * 2 * 64;  // (side, c, s = 0, piece 0)
        f32x16 d = {};
#pragma unroll
        for (int s = 0; s < 2; ++s) d = mfma32h(as_frag(A0[(s * 2 + 1) * 64 + lane]), B[s][0], d);
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const s16x8 a0 = as_frag(A0[(s * 2) * 64 + lane]);
          d = mfma32h(a0, B[s][1], d);
          d = mfma32h(a0, B[s][0], d);
        }
        return d;
      };
      // the channel combination p = T_W + b_r T_r + b_g T_g + b_b T_b on the scaled sums: b_c by 2^(e_W - e_c)
      const float4 bs = make_float4(b.x, ldexpf(b.y, eW - eC0), ldexpf(b.z, eW - eC1), ldexpf(b.w, eW - eC2));
      // Software-pipelined within the group, one channel per pass: each pass's 6 MFMAs share a scheduling region with
      // the previous pass's epilogue (which reads only finished accumulators), so the wave's own VALU work issues
      // between its MFMAs.  The channel combination p = fmaf(b_b, T_b, fmaf(b_g, T_g, fmaf(b_r, T_r, T_W))) is built
      // one channel at a time in that same order (the phased form's float operations, bit-identical), so only the
      // running p and two channels' accumulators are live.  Regions: [T_W] [T_r] [T_g | T_r epi] [T_b | T_g epi]
      // [ey split, R_W | T_b epi + moments] [R_r] [R_g | R_r epi] [R_b | R_g epi] [R_b epi + moments].
      s16x8 BT[2][2], BR[2][2];
      split2h_frag(ex[0], BT[0]);
      split2h_frag(ex[1], BT[1]);
      float p[16];
      {
        const f32x16 D3 = contract(0, 3, BT);
#pragma unroll
        for (int i = 0; i < 16; ++i) p[i] = D3[i];
      }
      f32x16 Dc = contract(0, 0, BT);
      GR_BWD32_PHASE();
#pragma unroll
      for (int c = 0; c < 3; ++c) {  // channel c's epilogue beside channel c + 1's MFMAs
        const float bc = c == 0 ? bs.y : (c == 1 ? bs.z : bs.w);
        f32x16 Dn;
        if (c < 2) {
          Dn = contract(0, c + 1, BT);
        } else {
          split2h_frag(ey[0], BR[0]);
          split2h_frag(ey[1], BR[1]);
          Dn = contract(1, 3, BR);
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          S[c] = fmaf(ey[i >> 3][i & 7], Dc[i], S[c]);
          p[i] = fmaf(bc, Dc[i], p[i]);
        }
        if (c == 2) {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int s = i >> 3, q = i & 7;
            const float oq = (float)kslot_off(q);
            const float t = ey[s][q] * p[i];
            S4s[s] += t;
            if (q != 0) {
              S6c[s] = fmaf(t, oq, S6c[s]);
              S8c[s] = fmaf(t, oq * oq, S8c[s]);
            }
          }
        }
        Dc = Dn;
        GR_BWD32_PHASE();
      }
      // R side: Dc = R_W
#pragma unroll
      for (int i = 0; i < 16; ++i) p[i] = Dc[i];
      Dc = contract(1, 0, BR);
      GR_BWD32_PHASE();
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float bc = c == 0 ? bs.y : (c == 1 ? bs.z : bs.w);
        f32x16 Dn;
        if (c < 2) Dn = contract(1, c + 1, BR);
#pragma unroll
        for (int i = 0; i < 16; ++i) p[i] = fmaf(bc, Dc[i], p[i]);
        if (c < 2) {
          Dc = Dn;
          GR_BWD32_PHASE();
        }
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int s = i >> 3, q = i & 7;
        const float oq = (float)kslot_off(q);
        const float u = ex[s][q] * p[i];
        U0[s] += u;
        if (q != 0) {
          S5c[s] = fmaf(u, oq, S5c[s]);
          S7c[s] = fmaf(u, oq * oq, S7c[s]);
        }
      }
      S[4] = S4s[0] + S4s[1];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        S[6] += fmaf(d0y[s], S4s[s], S6c[s]);
        S[8] += fmaf(d0y[s] * d0y[s], S4s[s], fmaf(2.0f * d0y[s], S6c[s], S8c[s]));
        S[5] += fmaf(d0x[s], U0[s], S5c[s]);
        S[7] += fmaf(d0x[s] * d0x[s], U0[s], fmaf(2.0f * d0x[s], S5c[s], S7c[s]));
      }
      // undo the scales (exact): the colour sums carry 2^(e_c + 2 SB), the rest 2^(e_W + 2 SB)
      S[0] = ldexpf(S[0], -(eC0 + 2 * GR_F16_SB));
      S[1] = ldexpf(S[1], -(eC1 + 2 * GR_F16_SB));
      S[2] = ldexpf(S[2], -(eC2 + 2 * GR_F16_SB));
#pragma unroll
      for (int k = 4; k < 9; ++k) S[k] = ldexpf(S[k], -(eW + 2 * GR_F16_SB));
      // lanes r and r + 32 hold the two halves of Gaussian r's slots (pair32); row as k_raster_bwd_bf16<false, .>
      const float Pa = pair32(S[0], S[1]), Pb = pair32(S[2], S[8]), Pc = pair32(S[4], S[5]);
      const float Pd = pair32(S[6], S[7]);
      if (myslot >= 0)
        reinterpret_cast<float4*>(partials)[2 * (size_t)myslot + h] =
            h == 0 ? make_float4(b.x * Pa, b.x * Pb, Pc, Pd) : make_float4(b.x * Pa, Pb, Pc, Pd);
    }
  }
}
__global__ __launch_bounds__(256, GR_BWD32_WAVES) void k_bwd32(ViewK v, int n, const int4* __restrict__ items,
                                                              const int* __restrict__ num_items, const int* __restrict__ pairs,
                                                              const float4* __restrict__ rec, const uint4* __restrict__ UF,
                                                              float* __restrict__ partials) {
  k_bwd32_body(v, n, items, num_items, pairs, rec, UF, partials, BI{(int)blockIdx.x, (int)blockIdx.y}, BI{(int)gridDim.x, (int)gridDim.y});
}
struct k_bwd32_args {
  ViewK v;
  int n;
  const int4* items;
  const int* num_items;
  const int* pairs;
  const float4* rec;
  const uint4* UF;
  float* partials;
};
__global__ __launch_bounds__(256, GR_BWD32_WAVES) void k_bwd32_views(VBatch<k_bwd32_args> B) {
  const int vb = vbatch_view(B, (int)blockIdx.x);
  const k_bwd32_args& a = B.a[vb];
  const int lb = (int)blockIdx.x - B.first[vb], gx = B.gx[vb];
  k_bwd32_body(a.v, a.n, a.items, a.num_items, a.pairs, a.rec, a.UF, a.partials, BI{lb % gx, lb / gx}, BI{gx, (B.first[vb + 1] - B.first[vb]) / gx});
}




// ------------------------------------------------------------------------------------------------
// Per-Gaussian reduction of pair partials + chain rule.  Deterministic.
// ------------------------------------------------------------------------------------------------
#ifndef GR_RG
#define GR_RG 64
#endif
constexpr int RG = GR_RG;        // Gaussians per reduce block (4 lanes each; one wave runs the chain rule)

// Where the chain rule puts one view's gradient of Gaussian i: GradOut writes (or adds, acc) it to the
// gradient buffers; GradRegs adds it to registers (k_reduce_views: several views, one write).
struct GradOut {
  float *dm, *ds, *dc, *dop;  // Gaussian i's entries
  bool acc;
  __device__ void put(float* d, float x) const { *d = acc ? *d + x : x; }
  __device__ void mean(int j, float x) const { put(dm + j, x); }
  __device__ void scale(int j, float x) const { put(ds + j, x); }
  __device__ void opac(float x) const { put(dop, x); }
  __device__ void color(int q, float x) const { put(dc + q, x); }
  __device__ void none(int cd) const {  // a Gaussian on no tile: zero gradient
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      mean(q, 0.f);
      scale(q, 0.f);
    }
    for (int q = 0; q < cd; ++q) color(q, 0.f);
    opac(0.f);
  }
  __device__ void scale_z() const { put(ds + 2, 0.f); }
};
template <int CD>
struct GradRegs {
  float m[3] = {0.f, 0.f, 0.f}, s[2] = {0.f, 0.f}, o = 0.f, c[CD] = {};
  __device__ void mean(int j, float x) { m[j] += x; }
  __device__ void scale(int j, float x) { s[j] += x; }
  __device__ void opac(float x) { o += x; }
  __device__ void color(int q, float x) { c[q] += x; }
  __device__ void none(int) {}
  __device__ void scale_z() {}
};

template <int CD, typename F, typename Out>
__device__ void chain_rule(const ViewK& v, int i, const F* S, unsigned cnt, const float* __restrict__ means,
                           const float* __restrict__ scales, const float* __restrict__ colors,
                           const float* __restrict__ opac, Out& out);

// Block of RG Gaussians, 4 lanes each.  A Gaussian's pairs are its emission indices: core pairs
// [c_i, c_i + core_i) and (only with an upstream depth gradient; otherwise the backward skipped them)
// tail pairs Kc + [t_i, t_i + tail_i); their partial sums sit at the pairs' sorted positions
// (pos_of), where the backward splat wrote them with coalesced stores.  Lane q sums pairs q, q+4, ...
// (core, then tail), the 4 sums are combined in a fixed order (deterministic, no atomics), and one
// lane per Gaussian applies the chain rule.
// ROW8: rows written by the no-depth split backward (8 floats, see bwd_item_bf16); else 9 floats.
template <int CD, bool ROW8>
__global__ __launch_bounds__(4 * RG) void k_reduce_bwd(ViewK v, int n, const float* __restrict__ means,
                                                    const float* __restrict__ scales, const float* __restrict__ colors,
                                                    const float* __restrict__ opac, const Cnt2* __restrict__ counts,
                                                    const Cnt2* __restrict__ offsets, const int* __restrict__ pos_of,
                                                    const float* __restrict__ partials, float* __restrict__ d_means,
                                                    float* __restrict__ d_scales, float* __restrict__ d_colors,
                                                    float* __restrict__ d_opac, int depth, int acc) {
  const int g0 = blockIdx.x * RG;
  const int tid = threadIdx.x, q4 = tid & 3;
  const int i = g0 + (tid >> 2);
  const long long Kc = (long long)offsets[n].c();
  double S[NPART];
#pragma unroll
  for (int q = 0; q < NPART; ++q) S[q] = 0.0;
  unsigned cnt = 0;
  if (i < n) {
    const Cnt2 cn = counts[i], of = offsets[i];
    cnt = cn.v != 0 ? 1u : 0u;  // any kept tile (core or tail)
    // pair e of this Gaussian (emission index) was written by the backward splat at its sorted
    // position pos_of[e]: the block's Gaussians are consecutive, so within each tile their rows are
    // one contiguous run of the sorted array
    const int* pc = pos_of + (long long)of.c();
    if constexpr (ROW8) {
      // four rows per lane in flight at a time (their positions first, then the rows), summed in the
      // same order as one row at a time
      const float4* rows = reinterpret_cast<const float4*>(partials);
      const int cc = (int)cn.c();
      for (int j0 = q4; j0 < cc; j0 += 16) {
        int pos[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) pos[u] = j0 + 4 * u < cc ? pc[j0 + 4 * u] : -1;
        float4 ru[4], rw[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const size_t r = pos[u] >= 0 ? (size_t)pos[u] : 0;
          ru[u] = rows[2 * r];
          rw[u] = rows[2 * r + 1];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (pos[u] < 0) break;
          const float4 a = ru[u], w = rw[u];  // [o S0, o S2, S4, S6], [o S1, S8, S5, S7]
          S[0] += (double)a.x;
          S[2] += (double)a.y;
          S[4] += (double)a.z;
          S[6] += (double)a.w;
          S[1] += (double)w.x;
          S[8] += (double)w.y;
          S[5] += (double)w.z;
          S[7] += (double)w.w;
        }
      }
    }
    for (int j = q4; !ROW8 && j < (int)cn.c(); j += 4) {
      {
        const float* src = partials + (size_t)pc[j] * NPART;
#pragma unroll
        for (int q = 0; q < NPART; ++q) S[q] += (double)src[q];
      }
    }
    if (depth) {
      const int* pt = pos_of + Kc + (long long)of.t();
      for (int j = q4; j < (int)cn.t(); j += 4) {
        const float* src = partials + (size_t)pt[j] * NPART;
#pragma unroll
        for (int q = 0; q < NPART; ++q) S[q] += (double)src[q];
      }
    }
  }
#pragma unroll
  for (int q = 0; q < NPART; ++q) {
    S[q] += __shfl_xor(S[q], 1);
    S[q] += __shfl_xor(S[q], 2);
  }
  // the block's sums -> LDS; then one lane per Gaussian (wave 0, every lane busy) runs the chain rule
  // in f32 (the reference's autograd precision)
  __shared__ float sS[RG][NPART + 1];
  if (q4 == 0) {
#pragma unroll
    for (int q = 0; q < NPART; ++q) sS[tid >> 2][q] = (float)S[q];
    sS[tid >> 2][NPART] = cnt ? 1.0f : 0.0f;
  }
  __syncthreads();
  if (tid >= RG || g0 + tid >= n) return;
  float Sf[NPART];
#pragma unroll
  for (int q = 0; q < NPART; ++q) Sf[q] = sS[tid][q];
  const int gi = g0 + tid;
  GradOut out{d_means + 3 * (size_t)gi, d_scales + 3 * (size_t)gi, d_colors + (size_t)CD * gi, d_opac + gi, acc != 0};
  chain_rule<CD, float>(v, gi, Sf, sS[tid][NPART] != 0.0f ? 1u : 0u, means, scales, colors, opac, out);
}

// Batched reduction (gr_reduce_views): the 8-float rows of up to GR_REDUCE_MAX_VIEWS views rendered
// without a depth gradient, one pass over the Gaussians.  Per view a Gaussian's rows are gathered as in
// k_reduce_bwd (4 lanes, fixed order, double sums); the chain rules then run one lane per Gaussian,
// wave w taking views w, w + 4 (CRW = 4 waves; SH degree 3: wave 0 alone), their gradients summed in
// registers and the wave sums combined in wave order: the parameters are read and the gradient written
// (or added to, acc) once per batch instead of once per view.  Deterministic.
struct RViewK {
  ViewK v;
  const Cnt2* offsets;  // the view's packed pair offsets (offsets[n] = totals)
  const int* pos_of;    // sorted position of each pair, by emission index
  const float4* rows;   // 8-float partial rows at sorted positions (bwd_item_bf16, no depth gradient)
};
struct RBatch {
  int nv;
  RViewK r[GR_REDUCE_MAX_VIEWS];
};

template <int CD>
__global__ __launch_bounds__(4 * RG) void k_reduce_views(RBatch B, int n, const float* __restrict__ means,
                                                      const float* __restrict__ scales, const float* __restrict__ colors,
                                                      const float* __restrict__ opac, float* __restrict__ d_means,
                                                      float* __restrict__ d_scales, float* __restrict__ d_colors,
                                                      float* __restrict__ d_opac, int acc) {
  constexpr int CRW = CD == 48 ? 1 : 4;  // waves running chain rules
  constexpr int NG = 6 + CD;             // gradient floats per Gaussian (means 3, scales 2, opacity, colours)
  constexpr int VG = 8;                  // views staged in LDS at a time
  // per view and Gaussian: the 9 sums; S3 (the depth sum) is 0 without a depth gradient, so its slot
  // carries the "on any tile" flag
  __shared__ float sS[VG][RG][NPART];
  __shared__ float sG[CRW > 1 ? CRW : 1][RG][NG + 1];
  const int g0 = blockIdx.x * RG;
  const int tid = threadIdx.x, q4 = tid & 3;
  const int i = g0 + (tid >> 2);
  const int w = tid >> 6, lane = tid & 63, gi = g0 + lane;
  GradRegs<CD> gr;
  for (int vg = 0; vg < B.nv; vg += VG) {
  const int nvg = min(VG, B.nv - vg);
  if (vg > 0) __syncthreads();  // the previous group's sums have been read
  // Three-stage pipeline over the group's views: the offsets of view vi + 2, the positions of view vi + 1
  // and the rows of view vi are in flight together (three independent loads instead of a chain of three
  // per view).  A Gaussian's first 16 pairs go through the pipeline; more are read after (rare).
  auto load_off = [&](int vi, Cnt2& a, Cnt2& b) {
    if (vi < nvg && i < n) {
      a = B.r[vg + vi].offsets[i];
      b = B.r[vg + vi].offsets[i + 1];
    } else {
      a.v = b.v = 0ull;
    }
  };
  auto load_pos = [&](int vi, Cnt2 a, Cnt2 b, int (&pos)[4]) {
    const int cc = (int)(b.c() - a.c());
#pragma unroll
    for (int u = 0; u < 4; ++u) pos[u] = q4 + 4 * u < cc ? B.r[vg + vi].pos_of[(size_t)a.c() + q4 + 4 * u] : -1;
  };
  Cnt2 a0, b0, a1, b1;
  int p0[4], p1[4];
  load_off(0, a0, b0);
  load_off(1, a1, b1);
  load_pos(0, a0, b0, p0);
  for (int vi = 0; vi < nvg; ++vi) {
    const RViewK& rv = B.r[vg + vi];
    Cnt2 a2, b2;
    load_off(vi + 2, a2, b2);
    if (vi + 1 < nvg) load_pos(vi + 1, a1, b1, p1);
    float4 ru[4], rw[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const size_t r = p0[u] >= 0 ? (size_t)p0[u] : 0;
      ru[u] = rv.rows[2 * r];
      rw[u] = rv.rows[2 * r + 1];
    }
    double S[NPART];
#pragma unroll
    for (int q = 0; q < NPART; ++q) S[q] = 0.0;
    const int cc = (int)(b0.c() - a0.c());
    const unsigned cnt = (cc != 0 || b0.t() != a0.t()) ? 1u : 0u;
    auto add_row = [&](float4 x, float4 w) {  // [o S0, o S2, S4, S6], [o S1, S8, S5, S7]
      S[0] += (double)x.x;
      S[2] += (double)x.y;
      S[4] += (double)x.z;
      S[6] += (double)x.w;
      S[1] += (double)w.x;
      S[8] += (double)w.y;
      S[5] += (double)w.z;
      S[7] += (double)w.w;
    };
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (p0[u] < 0) break;
      add_row(ru[u], rw[u]);
    }
    for (int j = q4 + 16; j < cc; j += 4) {  // pairs past the first 16, in the same lane order
      const size_t r = (size_t)rv.pos_of[(size_t)a0.c() + j];
      add_row(rv.rows[2 * r], rv.rows[2 * r + 1]);
    }
    a0 = a1;
    b0 = b1;
    a1 = a2;
    b1 = b2;
#pragma unroll
    for (int u = 0; u < 4; ++u) p0[u] = p1[u];
#pragma unroll
    for (int q = 0; q < NPART; ++q) {
      S[q] += __shfl_xor(S[q], 1);
      S[q] += __shfl_xor(S[q], 2);
    }
    if (q4 == 0) {
#pragma unroll
      for (int q = 0; q < NPART; ++q) sS[vi][tid >> 2][q] = (float)S[q];
      sS[vi][tid >> 2][3] = cnt ? 1.0f : 0.0f;
    }
  }
  __syncthreads();
  if (w < CRW && gi < n) {
    for (int vi = w; vi < nvg; vi += CRW) {
      float Sf[NPART];
#pragma unroll
      for (int q = 0; q < NPART; ++q) Sf[q] = sS[vi][lane][q];
      const unsigned on = Sf[3] != 0.0f ? 1u : 0u;
      Sf[3] = 0.0f;
      chain_rule<CD, float>(B.r[vg + vi].v, gi, Sf, on, means, scales, colors, opac, gr);
    }
  }
  }
  if constexpr (CRW > 1) {
    if (w < CRW) {
      float* mine = sG[w][lane];
#pragma unroll
      for (int q = 0; q < 3; ++q) mine[q] = gr.m[q];
      mine[3] = gr.s[0];
      mine[4] = gr.s[1];
      mine[5] = gr.o;
#pragma unroll
      for (int q = 0; q < CD; ++q) mine[6 + q] = gr.c[q];
    }
    __syncthreads();
    if (w != 0 || gi >= n) return;
#pragma unroll
    for (int q = 0; q < NG; ++q) {
      float t = sG[0][lane][q];
#pragma unroll
      for (int u = 1; u < CRW; ++u) t += sG[u][lane][q];
      sG[0][lane][q] = t;
    }
    const float* tot = sG[0][lane];
#pragma unroll
    for (int q = 0; q < 3; ++q) gr.m[q] = tot[q];
    gr.s[0] = tot[3];
    gr.s[1] = tot[4];
    gr.o = tot[5];
#pragma unroll
    for (int q = 0; q < CD; ++q) gr.c[q] = tot[6 + q];
  }
  if (w != 0 || gi >= n) return;
  GradOut out{d_means + 3 * (size_t)gi, d_scales + 3 * (size_t)gi, d_colors + (size_t)CD * gi, d_opac + gi, acc != 0};
#pragma unroll
  for (int q = 0; q < 3; ++q) out.mean(q, gr.m[q]);
  out.scale(0, gr.s[0]);
  out.scale(1, gr.s[1]);
  out.scale_z();
  out.opac(gr.o);
#pragma unroll
  for (int q = 0; q < CD; ++q) out.color(q, gr.c[q]);
}

// ------------------------------------------------------------------------------------------------
// The reduction in two stages (gr_gather_view + gr_reduce_sums): the gather of one view's pair rows into
// per-Gaussian sums runs right after the view's backward splat, as a lean kernel (few registers, no LDS)
// that fits beside the splat kernels of the other streams on the same SIMDs: its gathers overlap their
// VALU work instead of taking the CUs from them (the one-pass k_reduce_views needs 117 VGPRs for its chain
// rule and so never co-resides with a splat).  The chain rule of a batch of views then reads the sums
// (32 B per Gaussian and view, coalesced) in a short VALU pass.
// ------------------------------------------------------------------------------------------------
// Per Gaussian and view: the 8-float sums of its rows [o S0, o S2, S4, S6 | o S1, S8, S5, S7] (no depth
// gradient).  4 lanes per Gaussian, lane q sums rows q, q+4, ... in order (two rows in flight), the lane
// sums are combined in a fixed order (xor 1, then xor 2): deterministic.  Lane q writes floats 2q, 2q+1.
// xor-1 / xor-2 lane exchange inside a quad (DPP quad_perm: no LDS instruction)
__device__ __forceinline__ float quad_xor1(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
}
__device__ __forceinline__ float quad_xor2(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));
}
__device__ __forceinline__ void add4(float4& x, const float4 a) {
  x.x += a.x;
  x.y += a.y;
  x.z += a.z;
  x.w += a.w;
}
// One row in flight per lane with the next row's position prefetched: ~26 VGPRs, so a wave fits in what
// the splat kernels leave of a SIMD's registers (backward 4 x 120, forward 6 x 80 of 512).
// DEPTH (an upstream depth gradient: tail pairs were contracted too): lane q also sums the Gaussian's
// tail pairs q, q+4, ... after its core pairs, and the depth sums o S3 (depth3, by sorted position) of
// both, written to sums3[i].
template <bool DEPTH>
__device__ __forceinline__ void k_gather_view_body(int n, const Cnt2* __restrict__ offsets, const int* __restrict__ pos_of,
                                                     const float4* __restrict__ rows, float2* __restrict__ sums,
                                                     const float* __restrict__ depth3, float* __restrict__ sums3, const BI blockIdx, const BI gridDim) {
  const int tid = threadIdx.x, q4 = tid & 3;
  const int i = blockIdx.x * 64 + (tid >> 2);
  float4 x = {-0.f, -0.f, -0.f, -0.f}, y = x;
  float z3 = -0.f;
  if (i < n) {
    const Cnt2 o0 = offsets[i], o1 = offsets[i + 1];
    const unsigned a = o0.c(), cc = o1.c() - a;
    const int* pc = pos_of + a;
    unsigned j = q4;
    int p = j < cc ? pc[j] : 0;
    for (; j < cc; j += 4) {
      const int pn = j + 4 < cc ? pc[j + 4] : 0;
      add4(x, rows[2 * (size_t)p]);
      add4(y, rows[2 * (size_t)p + 1]);
      if constexpr (DEPTH) z3 += depth3[p];
      p = pn;
    }
    if constexpr (DEPTH) {
      const unsigned tc = o1.t() - o0.t();
      const int* pt = pos_of + (size_t)offsets[n].c() + o0.t();
      for (j = q4; j < tc; j += 4) {
        const int pp = pt[j];
        add4(x, rows[2 * (size_t)pp]);
        add4(y, rows[2 * (size_t)pp + 1]);
        z3 += depth3[pp];
      }
    }
  }
  if constexpr (DEPTH) {
    z3 += quad_xor1(z3);
    z3 += quad_xor2(z3);
    if (i < n && q4 == 0) sums3[i] = z3;
  }
  x.x += quad_xor1(x.x); x.y += quad_xor1(x.y); x.z += quad_xor1(x.z); x.w += quad_xor1(x.w);
  y.x += quad_xor1(y.x); y.y += quad_xor1(y.y); y.z += quad_xor1(y.z); y.w += quad_xor1(y.w);
  x.x += quad_xor2(x.x); x.y += quad_xor2(x.y); x.z += quad_xor2(x.z); x.w += quad_xor2(x.w);
  y.x += quad_xor2(y.x); y.y += quad_xor2(y.y); y.z += quad_xor2(y.z); y.w += quad_xor2(y.w);
  if (i < n) {
    const float2 o = q4 == 0 ? make_float2(x.x, x.y) : q4 == 1 ? make_float2(x.z, x.w) : q4 == 2 ? make_float2(y.x, y.y)
                                                                                        : make_float2(y.z, y.w);
    sums[4 * (size_t)i + q4] = o;
  }
}
template <bool DEPTH>
__global__ __launch_bounds__(256) void k_gather_view(int n, const Cnt2* __restrict__ offsets, const int* __restrict__ pos_of,
                                                     const float4* __restrict__ rows, float2* __restrict__ sums,
                                                     const float* __restrict__ depth3, float* __restrict__ sums3) {
  k_gather_view_body<DEPTH>(n, offsets, pos_of, rows, sums, depth3, sums3, BI{(int)blockIdx.x, (int)blockIdx.y}, BI{(int)gridDim.x, (int)gridDim.y});
}
struct k_gather_view_args {
  int n;
  const Cnt2* offsets;
  const int* pos_of;
  const float4* rows;
  float2* sums;
  const float* depth3;
  float* sums3;
};
template <bool DEPTH>
__global__ __launch_bounds__(256) void k_gather_view_views(VBatch<k_gather_view_args> B) {
  const int vb = vbatch_view(B, (int)blockIdx.x);
  const k_gather_view_args& a = B.a[vb];
  const int lb = (int)blockIdx.x - B.first[vb], gx = B.gx[vb];
  k_gather_view_body<DEPTH>(a.n, a.offsets, a.pos_of, a.rows, a.sums, a.depth3, a.sums3, BI{lb % gx, lb / gx}, BI{gx, (B.first[vb + 1] - B.first[vb]) / gx});
}


// Chain rule of up to GR_REDUCE_MAX_VIEWS views' gathered sums: one lane per Gaussian; the crw waves of a
// Gaussian group take views u, u + crw, ... (crw = 4 from three views, else the view count, so that no
// wave idles: a block holds 4 / crw groups of 64 Gaussians; SH degree 3 too: 240 VGPRs, 56 KiB LDS), the wave totals are
// combined in wave order and written (or added, acc) once.  A Gaussian whose eight sums are all zero
// touched no tile of that view (its chain rule would add zero).  Deterministic; for a given view count
// the summation order is fixed (1 or 2 views: the sums a 4-wave group gives, without its idle waves' zeros).
struct SViewK {
  ViewK v;
  const float4* sums;  // [n][2]: k_gather_view's output
  const float* sums3;  // [n] depth sums o S3 (k_gather_view<true>), or null (no depth gradient: S3 = 0)
};
struct SBatch {
  int nv;
  SViewK r[GR_REDUCE_MAX_VIEWS];
};
// waves per Gaussian group of k_reduce_sums (host and device)
__host__ __device__ constexpr int reduce_sums_crw(int nv, int cd) { return nv >= 3 ? 4 : (nv >= 1 ? nv : 1); }

template <int CD>
__global__ __launch_bounds__(256) void k_reduce_sums(SBatch B, int n, const float* __restrict__ means,
                                                     const float* __restrict__ scales, const float* __restrict__ colors,
                                                     const float* __restrict__ opac, float* __restrict__ d_means,
                                                     float* __restrict__ d_scales, float* __restrict__ d_colors,
                                                     float* __restrict__ d_opac, int acc, const int* __restrict__ sum_index) {
  // sum_index (gr_bwd_indexed): Gaussian gi's sums are row sum_index[gi] of the views' sums (a render of a permuted
  // copy); its parameters and gradients stay row gi
  constexpr int NG = 6 + CD;
  __shared__ float sG[4][64][NG + 1];
  const int crw = reduce_sums_crw(B.nv, CD);
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int gw = w / crw, u = w - gw * crw;
  const int gi = (blockIdx.x * (4 / crw) + gw) * 64 + lane;
  GradRegs<CD> gr;
  if (gi < n) {
    const size_t si = sum_index ? (size_t)sum_index[gi] : (size_t)gi;
    for (int vi = u; vi < B.nv; vi += crw) {
      const float4 a = B.r[vi].sums[2 * si], b = B.r[vi].sums[2 * si + 1];
      // [o S0, o S2, S4, S6 | o S1, S8, S5, S7] -> S0..S8 (S3, the depth sum, is 0 without a depth gradient)
      const float s3 = B.r[vi].sums3 ? B.r[vi].sums3[si] : 0.0f;
      const float Sf[NPART] = {a.x, b.x, a.y, s3, a.z, b.z, a.w, b.w, b.y};
      const unsigned on = (a.x != 0.f || a.y != 0.f || a.z != 0.f || a.w != 0.f || b.x != 0.f || b.y != 0.f ||
                           b.z != 0.f || b.w != 0.f || s3 != 0.f) ? 1u : 0u;
      chain_rule<CD, float>(B.r[vi].v, gi, Sf, on, means, scales, colors, opac, gr);
    }
  }
  {
    if (crw > 1) {  // uniform per launch
      float* mine = sG[w][lane];
#pragma unroll
      for (int q = 0; q < 3; ++q) mine[q] = gr.m[q];
      mine[3] = gr.s[0];
      mine[4] = gr.s[1];
      mine[5] = gr.o;
#pragma unroll
      for (int q = 0; q < CD; ++q) mine[6 + q] = gr.c[q];
      __syncthreads();
      if (u != 0 || gi >= n) return;
#pragma unroll
      for (int q = 0; q < NG; ++q) {
        float t = sG[w][lane][q];
        for (int v = 1; v < crw; ++v) t += sG[w + v][lane][q];
        sG[w][lane][q] = t;
      }
      const float* tot = sG[w][lane];
#pragma unroll
      for (int q = 0; q < 3; ++q) gr.m[q] = tot[q];
      gr.s[0] = tot[3];
      gr.s[1] = tot[4];
      gr.o = tot[5];
#pragma unroll
      for (int q = 0; q < CD; ++q) gr.c[q] = tot[6 + q];
    }
  }
  if (u != 0 || gi >= n) return;
  GradOut out{d_means + 3 * (size_t)gi, d_scales + 3 * (size_t)gi, d_colors + (size_t)CD * gi, d_opac + gi, acc != 0};
#pragma unroll
  for (int q = 0; q < 3; ++q) out.mean(q, gr.m[q]);
  out.scale(0, gr.s[0]);
  out.scale(1, gr.s[1]);
  out.scale_z();
  out.opac(gr.o);
#pragma unroll
  for (int q = 0; q < CD; ++q) out.color(q, gr.c[q]);
}

// The projection half of the chain rule (torch_renderer.py:57-78, 146-150) from a Gaussian's sums S (SURVEY.md
// App. A): the gradients of its clamped sigmas, of its camera-space point pc and of its clip-space point (shared
// by chain_rule and the camera gradient, k_camera_grad).
template <typename F>
struct ProjGrad {
  F dsx, dsy;   // d L / d sigma_x, sigma_y (zero where the clamp at 1 is active)
  F dpc[4];     // d L / d pc (through the clip point, and through z_abs into the depth and the sigmas)
  F dclip[4];   // d L / d clip
};
template <typename F>
__device__ __forceinline__ void proj_grads(const ViewK& v, const Proj& p, F o, const F* S, ProjGrad<F>& g) {
  const F sx = p.sx, sy = p.sy;
  // ge = o * gw * E  ->  sums over ge carry a factor o.
  const F dpx = o * S[5] / (sx * sx), dpy = o * S[6] / (sy * sy);
  F dsx = o * S[7] / (sx * sx * sx), dsy = o * S[8] / (sy * sy * sy);
  if (!(p.sxr >= 1.0f)) dsx = F(0);
  if (!(p.syr >= 1.0f)) dsy = F(0);
  g.dsx = dsx;
  g.dsy = dsy;
  const F dza = S[3] - dsx * p.sxr / p.za - dsy * p.syr / p.za;
#pragma unroll
  for (int j = 0; j < 4; ++j) g.dpc[j] = F(0);
  if (fabsf(p.pc[2]) >= 1e-6f) g.dpc[2] += dza * (p.pc[2] > 0.f ? F(1) : (p.pc[2] < 0.f ? F(-1) : F(0)));
  const F dndx = dpx * F(0.5) * (v.W - 1);
  const F dndy = -dpy * F(0.5) * (v.H - 1);
  g.dclip[0] = dndx / p.ws;
  g.dclip[1] = dndy / p.ws;
  g.dclip[2] = F(0);
  g.dclip[3] = (fabsf(p.clip[3]) < 1e-8f) ? F(0) : -(dndx * p.clip[0] + dndy * p.clip[1]) / ((F)p.ws * p.ws);
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) g.dpc[j] += (F)v.P[r * 4 + j] * g.dclip[r];
}

// The colour half (torch_renderer.py:86-106, 144): d L / d colour before the clamp (inclusive clamp mask), and
// for SH colours d L / d (cam - m) of the view direction (gd: through the normalisation; zero for RGB).
template <int CD, typename F>
struct ColGrad {
  F dcol[3];
  F d[3];    // unit view direction (SH)
  F dd[3];   // d L / d (cam - m)
};
template <int CD, typename F>
__device__ __forceinline__ void color_grads(const ViewK& v, float mx, float my, float mz, const float* __restrict__ col,
                                            const F* S, ColGrad<CD, F>& c) {
  float cpre[3];
  eval_color<CD>(v, mx, my, mz, col, cpre);
#pragma unroll
  for (int k = 0; k < 3; ++k) c.dcol[k] = (cpre[k] >= 0.0f && cpre[k] <= 1.0f) ? S[k] : F(0);
#pragma unroll
  for (int j = 0; j < 3; ++j) c.dd[j] = F(0);
  if constexpr (CD != 3) {
    const F vv[3] = {(F)v.cam[0] - mx, (F)v.cam[1] - my, (F)v.cam[2] - mz};
    const F nn = std::sqrt(vv[0] * vv[0] + vv[1] * vv[1] + vv[2] * vv[2]);
    const F ne = nn + F(1e-8);
#pragma unroll
    for (int j = 0; j < 3; ++j) c.d[j] = vv[j] / ne;
    F gd[3] = {F(0), F(0), F(0)};
    if constexpr (CD == 12) {
#pragma unroll
      for (int k = 0; k < 3; ++k)
#pragma unroll
        for (int j = 0; j < 3; ++j) gd[j] += c.dcol[k] * (F)col[(1 + j) * 3 + k];
    } else {  // degree 3: d col / d d = sum_i k_i dY_i/dd
      F G[16][3];
      sh3_basis_grad(c.d[0], c.d[1], c.d[2], G);
#pragma unroll
      for (int i = 0; i < 16; ++i)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const F t = c.dcol[k] * (F)col[3 * i + k];
#pragma unroll
          for (int j = 0; j < 3; ++j) gd[j] += t * G[i][j];
        }
    }
    if (nn > F(0)) {
      const F vg = vv[0] * gd[0] + vv[1] * gd[1] + vv[2] * gd[2];
#pragma unroll
      for (int j = 0; j < 3; ++j) c.dd[j] = gd[j] / ne - vv[j] * vg / (nn * ne * ne);
    }
  }
}

template <int CD, typename F, typename Out>
__device__ void chain_rule(const ViewK& v, int i, const F* S, unsigned cnt, const float* __restrict__ means,
                           const float* __restrict__ scales, const float* __restrict__ colors,
                           const float* __restrict__ opac, Out& out) {
  const float mx = means[3 * i], my = means[3 * i + 1], mz = means[3 * i + 2];
  const float s0 = scales[3 * i], s1 = scales[3 * i + 1];
  const float op = opac[i];
  const float* col = colors + (size_t)CD * i;
  if (cnt == 0) {
    out.none(CD);
    return;
  }
  Proj p;
  project(v, mx, my, mz, s0, s1, p);
  const F o = op < 0.0f ? F(0) : (F)op;
  ProjGrad<F> pg;
  proj_grads<F>(v, p, o, S, pg);
  const F fx = fabsf(v.P[0]), fy = fabsf(v.P[5]);
  const F kx = F(0.5) * v.W * fx / p.za, ky = F(0.5) * v.H * fy / p.za;
  const F sgx = s0 > 0.f ? F(1) : (s0 < 0.f ? F(-1) : F(0));
  const F sgy = s1 > 0.f ? F(1) : (s1 < 0.f ? F(-1) : F(0));
  out.scale(0, (float)(pg.dsx * kx * sgx));
  out.scale(1, (float)(pg.dsy * ky * sgy));
  out.scale_z();
  F dm[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    dm[j] = F(0);
#pragma unroll
    for (int r = 0; r < 4; ++r) dm[j] += (F)v.V[r * 4 + j] * pg.dpc[r];
  }
  out.opac((float)((op >= 0.0f) ? S[4] : F(0)));
  ColGrad<CD, F> cg;
  color_grads<CD, F>(v, mx, my, mz, col, S, cg);
#pragma unroll
  for (int k = 0; k < 3; ++k) out.color(k, (float)cg.dcol[k]);
  if constexpr (CD == 12) {
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int j = 0; j < 3; ++j) out.color((1 + j) * 3 + k, (float)(cg.dcol[k] * cg.d[j]));
  } else if constexpr (CD == 48) {  // d col / d k_i = Y_i(d)
    F Y[16];
    sh3_basis(cg.d[0], cg.d[1], cg.d[2], Y);
#pragma unroll
    for (int i = 1; i < 16; ++i)
#pragma unroll
      for (int k = 0; k < 3; ++k) out.color(3 * i + k, (float)(cg.dcol[k] * Y[i]));
  }
#pragma unroll
  for (int j = 0; j < 3; ++j) out.mean(j, (float)(dm[j] - cg.dd[j]));
}

// ------------------------------------------------------------------------------------------------
// Camera gradient (gr_bwd_camera).  The reference's camera is differentiable: view and proj are ordinary
// torch operands of _project, of the SH view direction (cam = inv(view)[:3,3]) and of the sigma rule
// (torch_renderer.py:57-83, 140-150), so a caller whose camera tensors require grad gets d view / d proj.
// From a view's per-Gaussian sums (k_gather_view's output, the same the chain rule reads), each Gaussian's
//   d view += d pc (m, 1)^T,   d proj += d clip pc^T,   d proj[0][0] += d sigma_x |s0| W / (2 z) sign(P00)
//   (the same for [1][1]),   d cam += d L / d (cam - m)  (SH colours),
// summed per block in double (wave butterfly, then the four waves in order) and over the blocks by
// k_camera_final (one wave per component, fixed order): deterministic.  The host turns d cam into
// d view through the inverse (torch_renderer.py:81-83).
// ------------------------------------------------------------------------------------------------
constexpr int CAM_GRADS = 35;  // d view (16, row-major), d proj (16), d cam_pos (3)
template <int CD>
__global__ __launch_bounds__(256) void k_camera_grad(ViewK v, int n, const float* __restrict__ means,
                                                     const float* __restrict__ scales, const float* __restrict__ colors,
                                                     const float* __restrict__ opac, const float4* __restrict__ sums,
                                                     const float* __restrict__ sums3, double* __restrict__ part) {
  double acc[CAM_GRADS];
#pragma unroll
  for (int q = 0; q < CAM_GRADS; ++q) acc[q] = 0.0;
  const int i = blockIdx.x * 256 + (int)threadIdx.x;
  if (i < n) {
    const float4 a = sums[2 * (size_t)i], b = sums[2 * (size_t)i + 1];
    const float s3 = sums3 ? sums3[i] : 0.0f;
    const float S[NPART] = {a.x, b.x, a.y, s3, a.z, b.z, a.w, b.w, b.y};
    const bool on = a.x != 0.f || a.y != 0.f || a.z != 0.f || a.w != 0.f || b.x != 0.f || b.y != 0.f || b.z != 0.f ||
                    b.w != 0.f || s3 != 0.f;
    if (on) {
      const float mx = means[3 * i], my = means[3 * i + 1], mz = means[3 * i + 2];
      const float s0 = scales[3 * i], s1 = scales[3 * i + 1];
      const float op = opac[i];
      Proj p;
      project(v, mx, my, mz, s0, s1, p);
      ProjGrad<float> pg;
      proj_grads<float>(v, p, op < 0.0f ? 0.0f : op, S, pg);
      const float mh[4] = {mx, my, mz, 1.0f};
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          acc[r * 4 + j] = (double)pg.dpc[r] * (double)mh[j];
          acc[16 + r * 4 + j] = (double)pg.dclip[r] * (double)p.pc[j];
        }
      const float sg0 = v.P[0] > 0.f ? 1.f : (v.P[0] < 0.f ? -1.f : 0.f);
      const float sg5 = v.P[5] > 0.f ? 1.f : (v.P[5] < 0.f ? -1.f : 0.f);
      acc[16 + 0] += (double)(pg.dsx * (fabsf(s0) * 0.5f * (float)v.W / p.za) * sg0);
      acc[16 + 5] += (double)(pg.dsy * (fabsf(s1) * 0.5f * (float)v.H / p.za) * sg5);
      if constexpr (CD != 3) {
        ColGrad<CD, float> cg;
        color_grads<CD, float>(v, mx, my, mz, colors + (size_t)CD * i, S, cg);
#pragma unroll
        for (int j = 0; j < 3; ++j) acc[32 + j] = (double)cg.dd[j];
      }
    }
  }
#pragma unroll
  for (int q = 0; q < CAM_GRADS; ++q)
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) acc[q] += __shfl_xor(acc[q], m);
  __shared__ double sh[4][CAM_GRADS];
  const int w = (int)threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int q = 0; q < CAM_GRADS; ++q) sh[w][q] = acc[q];
  __syncthreads();
  if ((int)threadIdx.x < CAM_GRADS) {
    const int q = threadIdx.x;
    part[(size_t)blockIdx.x * CAM_GRADS + q] = ((sh[0][q] + sh[1][q]) + sh[2][q]) + sh[3][q];
  }
}

// Block partials -> the view's camera gradient: block q sums component q over the blocks (lane l takes blocks
// l, l + 64, ..., then a butterfly), in a fixed order.
__global__ __launch_bounds__(64) void k_camera_final(const double* __restrict__ part, int blocks, float* __restrict__ out) {
  const int q = blockIdx.x, lane = threadIdx.x;
  double s = 0.0;
  for (int b = lane; b < blocks; b += 64) s += part[(size_t)b * CAM_GRADS + q];
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m);
  if (lane == 0) out[q] = (float)s;
}

// ------------------------------------------------------------------------------------------------
// Legacy uint8 surface (renderer_cpu.cpp:34-260 semantics).
// ------------------------------------------------------------------------------------------------
struct LegacyRec {
  float4* a;   // px, py, 1/sx^2, 1/sy^2
  float4* c;   // r, g, b, opacity (unclamped, as the reference)
  int4* box;   // xmin, xmax, ymin, ymax (3-sigma, inclusive)
  int4* rect;  // tile rectangle
  int* counts;
  int* offsets;
  uint32_t* depth_key;  // descending camera z -> ascending key
};

__global__ __launch_bounds__(256) void k_preprocess_u8(ViewK v, int n, const float* __restrict__ means,
                                                       const float* __restrict__ scales, const float* __restrict__ colors,
                                                       const float* __restrict__ opac, LegacyRec g) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == n) g.counts[n] = 0;
  if (i >= n) return;
  const float x = means[3 * i], y = means[3 * i + 1], z = means[3 * i + 2];
  float pc[4], cl[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) pc[r] = v.V[r * 4 + 0] * x + v.V[r * 4 + 1] * y + v.V[r * 4 + 2] * z + v.V[r * 4 + 3] * 1.0f;
#pragma unroll
  for (int r = 0; r < 4; ++r) cl[r] = v.P[r * 4 + 0] * pc[0] + v.P[r * 4 + 1] * pc[1] + v.P[r * 4 + 2] * pc[2] + v.P[r * 4 + 3] * pc[3];
  // depth key: larger camera z first (renderer_cpu.cpp:144-146); -0 folded onto +0.
  uint32_t zb = __float_as_uint(pc[2] + 0.0f);
  zb = (zb & 0x80000000u) ? ~zb : (zb | 0x80000000u);
  g.depth_key[i] = ~zb;
  g.counts[i] = 0;
  g.rect[i] = make_int4(0, 0, -1, -1);
  const float z_abs = fabsf(pc[2]) + 1e-6f;
  if (cl[3] == 0.0f) return;
  const float inv_w = 1.0f / cl[3];
  const float nx = cl[0] * inv_w, ny = cl[1] * inv_w, nz = cl[2] * inv_w;
  if (nz < -1.0f || nz > 1.0f) return;
  const float px = (nx * 0.5f + 0.5f) * (float)(v.W - 1);
  const float py = (1.0f - (ny * 0.5f + 0.5f)) * (float)(v.H - 1);
  float sx = scales[3 * i] * 0.5f * (float)v.W * fabsf(v.P[0]) / z_abs;
  float sy = scales[3 * i + 1] * 0.5f * (float)v.H * fabsf(v.P[5]) / z_abs;
  sx = sx > 1.0f ? sx : 1.0f;
  sy = sy > 1.0f ? sy : 1.0f;
  const float rx = 3.0f * sx, ry = 3.0f * sy;
  if (!(px + rx >= 0.0f) || !(px - rx <= (float)(v.W - 1)) || !(py + ry >= 0.0f) || !(py - ry <= (float)(v.H - 1))) return;
  const int xmin = (px - rx <= 0.0f) ? 0 : (int)floorf(px - rx);
  const int xmax = (px + rx >= (float)(v.W - 1)) ? v.W - 1 : (int)ceilf(px + rx);
  const int ymin = (py - ry <= 0.0f) ? 0 : (int)floorf(py - ry);
  const int ymax = (py + ry >= (float)(v.H - 1)) ? v.H - 1 : (int)ceilf(py + ry);
  g.a[i] = make_float4(px, py, 1.0f / (sx * sx), 1.0f / (sy * sy));
  g.c[i] = make_float4(colors[3 * i], colors[3 * i + 1], colors[3 * i + 2], opac[i]);
  g.box[i] = make_int4(xmin, xmax, ymin, ymax);
  const int4 r = make_int4(xmin / T, ymin / T, xmax / T, ymax / T);
  g.rect[i] = r;
  g.counts[i] = (r.z - r.x + 1) * (r.w - r.y + 1);
}

// Exact 64-bit total of the per-Gaussian pair counts: the int32 scan that places the pairs can wrap
// past 2^32 back to a positive total, so the total is checked here before anything is sized from it.
__global__ __launch_bounds__(256) void k_count_total64(int n, const int* __restrict__ counts,
                                                       unsigned long long* __restrict__ total) {
  unsigned long long s = 0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) s += (unsigned)counts[i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if ((threadIdx.x & 63) == 0 && s) atomicAdd(total, s);
}

template <bool SORTED>
__global__ __launch_bounds__(256) void k_raster_u8(ViewK v, const int2* __restrict__ ranges, const int* __restrict__ ids,
                                                   const float4* __restrict__ ga, const float4* __restrict__ gc,
                                                   const int4* __restrict__ gbox, uint8_t* __restrict__ rgba) {
  __shared__ float4 sA[TP];
  __shared__ float4 sC[TP];
  __shared__ int4 sBox[TP];
  const int tile = blockIdx.x;
  const int tx = tile % v.tiles_x, ty = tile / v.tiles_x;
  const int tid = threadIdx.x;
  const int x = tx * T + (tid & (T - 1)), y = ty * T + (tid >> 4);
  const float xc = (float)x + 0.5f, yc = (float)y + 0.5f;
  const int2 rg = ranges[tile];
  float r = 0.f, g = 0.f, b = 0.f, a = 0.f;
  bool done = !(x < v.W && y < v.H);
  for (int base = rg.x; base < rg.y; base += TP) {
    if (SORTED) {
      if (__syncthreads_and(done)) break;  // front-to-back: every pixel of the tile saturated
    } else {
      __syncthreads();
    }
    const int cnt = min(TP, rg.y - base);
    if (tid < cnt) {
      const int id = ids[base + tid];
      sA[tid] = ga[id];
      sC[tid] = gc[id];
      sBox[tid] = gbox[id];
    }
    __syncthreads();
    for (int j = 0; j < cnt; ++j) {
      const int4 bx = sBox[j];
      if (x < bx.x || x > bx.y || y < bx.z || y > bx.w) continue;
      const float4 ga_ = sA[j];
      const float4 gc_ = sC[j];
      const float dx = xc - ga_.x, dy = yc - ga_.y;
      const float e = -0.5f * (dx * dx * ga_.z + dy * dy * ga_.w);
      float w = gc_.w * expf(e);
      if (w < 1e-5f) continue;
      if (!SORTED) {
        r += w * gc_.x;
        g += w * gc_.y;
        b += w * gc_.z;
        a += w;
      } else {
        w = clamp01(w);
        const float contrib = (1.0f - a) * w;
        if (contrib <= 0.0f) continue;
        r += contrib * gc_.x;
        g += contrib * gc_.y;
        b += contrib * gc_.z;
        a += contrib;
        if (a >= 1.0f) done = true;
      }
    }
  }
  if (!(x < v.W && y < v.H)) return;
  float rr, gg, bb;
  if (!SORTED) {
    const float den = 1.0f + a;
    rr = (v.bg[0] + r) / den;
    gg = (v.bg[1] + g) / den;
    bb = (v.bg[2] + b) / den;
  } else {
    const float al = clamp01(a);
    rr = r + (1.0f - al) * v.bg[0];
    gg = g + (1.0f - al) * v.bg[1];
    bb = b + (1.0f - al) * v.bg[2];
  }
  const int p = y * v.W + x;
  uchar4 o;
  o.x = (uint8_t)(clamp01(rr) * 255.0f + 0.5f);
  o.y = (uint8_t)(clamp01(gg) * 255.0f + 0.5f);
  o.z = (uint8_t)(clamp01(bb) * 255.0f + 0.5f);
  o.w = 255;
  reinterpret_cast<uchar4*>(rgba)[p] = o;
}

// Sorted mode: OR each pair's Gaussian depth key into the low 32 bits of its 64-bit key.
__global__ __launch_bounds__(256) void k_patch_depth(int64_t K, uint64_t* keys, const int* __restrict__ ids,
                                                     const uint32_t* __restrict__ dk) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < K) keys[k] |= (uint64_t)dk[ids[k]];
}

// ------------------------------------------------------------------------------------------------
// Fit-loop loss (the caller's side of the render op): loss = mean|a - b| + w2 * mean|c - d|, the
// photometric L1 and the silhouette L1 of fit_multiview_stub.py:292-299, in two kernels per
// direction instead of torch's chain of elementwise + reduction launches.  Deterministic: a fixed
// grid, fixed per-thread strides, block tree sums, and an in-order final sum in double.
// ------------------------------------------------------------------------------------------------
constexpr int LOSS_BLOCKS = 512;

__global__ __launch_bounds__(256) void k_l1_partial(const float* __restrict__ a, const float* __restrict__ b, int64_t n1,
                                                    const float* __restrict__ c, const float* __restrict__ d, int64_t n2,
                                                    float* __restrict__ partial) {
  __shared__ float red[256];
  const bool second = blockIdx.y == 1;
  const float* x = second ? c : a;
  const float* y = second ? d : b;
  const int64_t n = second ? n2 : n1;
  float acc = 0.0f;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)LOSS_BLOCKS * 256) acc += fabsf(x[e] - y[e]);
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.y * LOSS_BLOCKS + blockIdx.x] = red[0];
}

__global__ __launch_bounds__(256) void k_l1_final(const float* __restrict__ partial, int64_t n1, int64_t n2, float w2,
                                                  float* __restrict__ loss) {
  __shared__ double r1[256], r2[256];
  const int t = threadIdx.x;
  double s1 = 0.0, s2 = 0.0;
  for (int i = t; i < LOSS_BLOCKS; i += 256) {
    s1 += (double)partial[i];
    s2 += (double)partial[LOSS_BLOCKS + i];
  }
  r1[t] = s1;
  r2[t] = s2;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w) {
      r1[t] += r1[t + w];
      r2[t] += r2[t + w];
    }
    __syncthreads();
  }
  if (t != 0) return;
  const float m1 = (float)(r1[0] / (double)n1);
  *loss = n2 > 0 ? m1 + w2 * (float)(r2[0] / (double)n2) : m1;
}

// The view loss of gr_bwd_l1 from its per-tile sums (double, fixed order): mean|out - t| +
// w_sil mean|alpha - m|, the value k_l1_final gives for the same images.
// The view loss from the per-tile sums (fixed order, double): mean|out - t| + w_sil mean|alpha - m|
// (n2 = HW with a mask, else 0) + w_depth mean|d_pred - t_d| (n3 = HW with a depth target, else 0).
// d/da = g sign(a - b) / n1, d/dc = (w2 g) sign(c - d) / n2 (torch: abs' = sign, sign(0) = 0).
__global__ __launch_bounds__(256) void k_l1_grad(const float* __restrict__ a, const float* __restrict__ b, int64_t n1,
                                                 const float* __restrict__ c, const float* __restrict__ d, int64_t n2,
                                                 float w2, const float* __restrict__ g_loss, float* __restrict__ ga,
                                                 float* __restrict__ gc) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const float g = *g_loss;
  if (e < n1) {
    const float t = a[e] - b[e];
    ga[e] = (t > 0.0f ? 1.0f : (t < 0.0f ? -1.0f : 0.0f)) * (g / (float)n1);
  }
  if (e < n2) {
    const float t = c[e] - d[e];
    gc[e] = (t > 0.0f ? 1.0f : (t < 0.0f ? -1.0f : 0.0f)) * ((w2 * g) / (float)n2);
  }
}

// The fit loop's parameter update (fit_multiview_stub.py:268-275 activations, :307-308 regulariser,
// :311 Adam) for one parameter tensor, fused into one pass over its elements (gr_fit_param_step):
//   g_raw = act'(raw) * (((acc0 + acc1) + ...) + reg)     d loss / d raw parameter (torch's backward of
//                                                         softplus(x) + 1e-3 / sigmoid / identity)
//   then, with Adam, torch.optim.Adam's foreach update in its own operation order:
//   m = m + (1 - b1)(g - m); v = v b2 + ((1 - b2) g) g; p = p + step_size m / (sqrt(v) / bc2_sqrt + eps).
// act: 0 identity, 1 softplus (threshold 20, as torch), 2 sigmoid.
struct AccList {
  const float* p[GR_FIT_MAX_ACC];
  int n;
};
__global__ __launch_bounds__(256) void k_fit_param_step(int64_t count, int act, float* __restrict__ p,
                                                        float* __restrict__ grad, AccList acc, float reg, int adam, float* __restrict__ m, float* __restrict__ v,
                                                        float neg_step, float bc2_sqrt, float b1, float b2, float b2_c,
                                                        float eps) {
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < count; e += (int64_t)gridDim.x * 256) {
    float gact = acc.n > 0 ? acc.p[0][e] : 0.0f;
    for (int a = 1; a < acc.n; ++a) gact = gact + acc.p[a][e];  // in stream order
    gact = gact + reg;
    const float x = p[e];
    float g;
    if (act == 1) {  // softplus backward: g z / (z + 1), z = exp(x) (x <= 20), else g
      const float z = expf(x);
      g = x > 20.0f ? gact : gact * z / (z + 1.0f);
    } else if (act == 2) {  // sigmoid backward: g (1 - y) y
      const float y = 1.0f / (1.0f + expf(-x));
      g = gact * (1.0f - y) * y;
    } else {
      g = gact;
    }
    if (grad) grad[e] = g;
    if (adam) {  // b1 here is 1 - beta1 and b2 is (beta2, 1 - beta2) rounded from double on the host, as torch's scalars
      const float mm = fmaf(b1, g - m[e], m[e]);
      const float vv = fmaf(b2_c, g * g, v[e] * b2);
      m[e] = mm;
      v[e] = vv;
      p[e] = fmaf(neg_step, mm / (sqrtf(vv) / bc2_sqrt + eps), x);
    }
  }
}

// k_fit_param_step over several parameter tensors (gr_fit_param_steps): block b belongs to the tensor whose block
// range [first[t], first[t + 1]) holds it and grid-strides over that tensor alone.
struct ParamSteps {
  gr_param_step s[GR_FIT_MAX_PARAMS];
  int first[GR_FIT_MAX_PARAMS + 1];
  int vec4[GR_FIT_MAX_PARAMS];  // 1: count % 4 == 0 and every array 16-byte aligned (float4 loads and stores)
  int num;
};
// One element of k_fit_param_steps: the activation's backward on the summed gradient, then Adam (torch's
// single-tensor update order).  Returns the gradient; m, v and x are updated in place.
__device__ __forceinline__ float fit_param_elem(int act, float gact, float& x, float& m, float& v, float neg_step,
                                                float bc2s, float b1, float b2, float b2_c, float eps) {
  float g;
  if (act == 1) {  // softplus backward: g z / (z + 1), z = exp(x) (x <= 20), else g
    const float z = expf(x);
    g = x > 20.0f ? gact : gact * z / (z + 1.0f);
  } else if (act == 2) {  // sigmoid backward: g (1 - y) y
    const float y = 1.0f / (1.0f + expf(-x));
    g = gact * (1.0f - y) * y;
  } else {
    g = gact;
  }
  m = fmaf(b1, g - m, m);
  v = fmaf(b2_c, g * g, v * b2);
  x = fmaf(neg_step, m / (sqrtf(v) / bc2s + eps), x);
  return g;
}
// sched (gr_fit_param_steps_sched): the step's (neg_step_size, bias_correction2_sqrt) are sched[2 *step_dev + 0/1], and a
// step whose views overflowed their capacities (*ovf) updates nothing.
__global__ __launch_bounds__(256) void k_fit_param_steps(ParamSteps P, float b1, float b2, float b2_c, float eps,
                                                         const float* __restrict__ sched, const int* __restrict__ step_dev,
                                                         const int* __restrict__ ovf) {
  if (ovf && *ovf) return;  // (uniform)
  int t = 0;
  while (t + 1 < P.num && (int)blockIdx.x >= P.first[t + 1]) ++t;
  const gr_param_step& q = P.s[t];
  const int ts = sched ? *step_dev : 0;
  const float neg_step = sched ? sched[2 * ts] : q.neg_step_size, bc2s = sched ? sched[2 * ts + 1] : q.bias_correction2_sqrt;
  const int nb = P.first[t + 1] - P.first[t];
  float* __restrict__ p = q.param;
  float* __restrict__ m = q.exp_avg;
  float* __restrict__ v = q.exp_avg_sq;
  const int64_t e0 = (int64_t)(blockIdx.x - P.first[t]) * 256 + threadIdx.x, stride = (int64_t)nb * 256;
  if (P.vec4[t]) {  // the same per-element arithmetic, four elements per thread
    for (int64_t e = e0; e < q.count / 4; e += stride) {
      float4 ga = q.num_accs > 0 ? ((const float4*)q.accs[0])[e] : make_float4(0.f, 0.f, 0.f, 0.f);
      for (int a = 1; a < q.num_accs; ++a) {  // in stream order
        const float4 u = ((const float4*)q.accs[a])[e];
        ga.x = ga.x + u.x;
        ga.y = ga.y + u.y;
        ga.z = ga.z + u.z;
        ga.w = ga.w + u.w;
      }
      float4 x = ((float4*)p)[e], mm = ((float4*)m)[e], vv = ((float4*)v)[e], g;
      g.x = fit_param_elem(q.act, ga.x + q.reg, x.x, mm.x, vv.x, neg_step, bc2s, b1, b2, b2_c, eps);
      g.y = fit_param_elem(q.act, ga.y + q.reg, x.y, mm.y, vv.y, neg_step, bc2s, b1, b2, b2_c, eps);
      g.z = fit_param_elem(q.act, ga.z + q.reg, x.z, mm.z, vv.z, neg_step, bc2s, b1, b2, b2_c, eps);
      g.w = fit_param_elem(q.act, ga.w + q.reg, x.w, mm.w, vv.w, neg_step, bc2s, b1, b2, b2_c, eps);
      if (q.grad) ((float4*)q.grad)[e] = g;
      ((float4*)m)[e] = mm;
      ((float4*)v)[e] = vv;
      ((float4*)p)[e] = x;
    }
    return;
  }
  for (int64_t e = e0; e < q.count; e += stride) {
    float gact = q.num_accs > 0 ? q.accs[0][e] : 0.0f;
    for (int a = 1; a < q.num_accs; ++a) gact = gact + q.accs[a][e];  // in stream order
    float x = p[e], mm = m[e], vv = v[e];
    const float g = fit_param_elem(q.act, gact + q.reg, x, mm, vv, neg_step, bc2s, b1, b2, b2_c, eps);
    if (q.grad) q.grad[e] = g;
    m[e] = mm;
    v[e] = vv;
    p[e] = x;
  }
}

// After a gr_fit_param_steps_sched update: the step counter advances when the update ran; an overflow is reported
// to the host (sticky flag in pinned memory) and cleared for the next step.
__global__ void k_step_advance(int* __restrict__ step_dev, int* __restrict__ ovf, int* host_flags) {
  if (threadIdx.x != 0) return;
  const int o = *ovf;
  const int t = *step_dev + (o ? 0 : 1);
  *step_dev = t;
  *ovf = 0;
  if (o) host_flags[0] = 1;
  host_flags[1] = t;
  __threadfence_system();
}

// The fit loop's activations (gr_fit_activations) with torch's float formulas (softplus: x > 20 ? x : log1p(exp(x));
// sigmoid: 1 / (1 + exp(-x))), and optionally the regulariser's two sums: per block in double, the last block to
// arrive adds the blocks' sums in block order.
constexpr int ACT_BLOCKS = 1024;
__global__ __launch_bounds__(256) void k_fit_activations(int64_t n, const float* __restrict__ s_raw,
                                                         const float* __restrict__ o_raw, const float* __restrict__ c_raw,
                                                         int64_t nc, float* __restrict__ s, float* __restrict__ o,
                                                         float* __restrict__ c, float w_s, float w_o,
                                                         float* __restrict__ reg_out, double* __restrict__ part,
                                                         int* __restrict__ ticket) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  double ss = 0.0, so = 0.0;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < 3 * n; e += stride) {
    const float x = s_raw[e];
    const float y = (x > 20.0f ? x : log1pf(expf(x))) + 1e-3f;
    s[e] = y;
    ss += (double)y;
  }
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += stride) {
    const float y = 1.0f / (1.0f + expf(-o_raw[e]));
    o[e] = y;
    so += (double)y;
  }
  if (c_raw)
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < nc; e += stride) c[e] = 1.0f / (1.0f + expf(-c_raw[e]));
  if (!reg_out) return;  // (uniform)
  __shared__ double sh[2][4];
  __shared__ int last;
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    ss += __shfl_xor(ss, m);
    so += __shfl_xor(so, m);
  }
  if ((threadIdx.x & 63) == 0) {
    sh[0][threadIdx.x >> 6] = ss;
    sh[1][threadIdx.x >> 6] = so;
  }
  __syncthreads();
  if (threadIdx.x < 2) st_through(&part[2 * blockIdx.x + threadIdx.x], (sh[threadIdx.x][0] + sh[threadIdx.x][1]) + (sh[threadIdx.x][2] + sh[threadIdx.x][3]));
  if (!arrive_last(ticket, (int)gridDim.x, &last)) return;
  // the last block: thread t sums blocks t, t + 256, ... in order, then the 256 partial sums in a fixed tree
  double ts = 0.0, to = 0.0;
  for (int b = threadIdx.x; b < (int)gridDim.x; b += 256) {
    ts += ld_through(&part[2 * b]);
    to += ld_through(&part[2 * b + 1]);
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) {
    ts += __shfl_xor(ts, m);
    to += __shfl_xor(to, m);
  }
  __syncthreads();
  if ((threadIdx.x & 63) == 0) {
    sh[0][threadIdx.x >> 6] = ts;
    sh[1][threadIdx.x >> 6] = to;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const double ms = ((sh[0][0] + sh[0][1]) + (sh[0][2] + sh[0][3])) / (double)(3 * n);
    const double mo = ((sh[1][0] + sh[1][1]) + (sh[1][2] + sh[1][3])) / (double)n;
    *reg_out = w_o * (float)mo + w_s * (float)ms;
    *ticket = 0;
  }
}

// Adam alone on an assembled (e.g. all-reduced) gradient.
__global__ __launch_bounds__(256) void k_adam_step(int64_t count, float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, float neg_step,
                                                   float bc2_sqrt, float b1, float b2, float b2_c, float eps) {
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < count; e += (int64_t)gridDim.x * 256) {
    const float ge = g[e];
    const float mm = fmaf(b1, ge - m[e], m[e]);
    const float vv = fmaf(b2_c, ge * ge, v[e] * b2);
    m[e] = mm;
    v[e] = vv;
    p[e] = fmaf(neg_step, mm / (sqrtf(vv) / bc2_sqrt + eps), p[e]);
  }
}

// Optional per-kernel timing with HIP events on the launch stream (gr_profile_begin/end), used by
// bench.py to time the dominant kernels live.  Off by default; host-side state only.
enum { PROF_RASTER_FWD = 0, PROF_RASTER_BWD = 1, PROF_REDUCE = 2, PROF_BINNING = 3, PROF_SLOTS = 4 };
struct ProfSlot {
  std::vector<hipEvent_t> ev;
  size_t used = 0;
};
std::mutex g_prof_mu;
std::atomic<bool> g_prof_on{false};
ProfSlot g_prof[PROF_SLOTS];

// Off (the default): one relaxed atomic load per mark, no lock on the launch path.
void prof_mark(int which, hipStream_t s) {
  if (!g_prof_on.load(std::memory_order_relaxed)) return;
  std::lock_guard<std::mutex> lk(g_prof_mu);
  if (!g_prof_on.load(std::memory_order_relaxed)) return;
  ProfSlot& sl = g_prof[which];
  if (sl.used == sl.ev.size()) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return;
    sl.ev.push_back(e);
  }
  (void)hipEventRecord(sl.ev[sl.used++], s);
}

inline int blocks_for(int64_t n, int bs = 256) { return (int)((n + bs - 1) / bs); }

gr_status check_view(const gr_view* v) {
  if (!v) return set_error(GR_ERR_INVALID_ARGUMENT, "view is null");
  if (v->width <= 0 || v->height <= 0) return set_error(GR_ERR_INVALID_ARGUMENT, "width/height must be positive");
  if ((int64_t)v->width * v->height > (1ll << 30)) return set_error(GR_ERR_INVALID_ARGUMENT, "image too large");
  if (v->tile != 0 && v->tile != T && v->tile != T32) return set_error(GR_ERR_INVALID_ARGUMENT, "tile must be 0, 16 or 32");
  if (v->rows < 0 || (v->rows > 0 && (v->row0 < 0 || v->row0 >= tiles_y_of(v->height, tile_of(v)))))
    return set_error(GR_ERR_INVALID_ARGUMENT, "row0 / rows: a band of the view's tile rows");
  return GR_OK;
}

}  // namespace

// ================================================================================================
// C ABI
// ================================================================================================
extern "C" {

const char* gr_last_error(void) { return g_last_error.c_str(); }

// the native fit executor (gr_fit_exec.cpp) reports its errors through the same thread-local message
gr_status gr_exec_set_error(gr_status st, const char* msg) { return set_error(st, msg); }

void gr_profile_begin(void) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  for (auto& sl : g_prof) sl.used = 0;
  g_prof_on.store(true, std::memory_order_relaxed);
}

gr_status gr_profile_end(double total_ms[4], int launches[4]) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  g_prof_on.store(false, std::memory_order_relaxed);
  for (int k = 0; k < PROF_SLOTS; ++k) {
    ProfSlot& sl = g_prof[k];
    double tot = 0.0;
    int cnt = 0;
    for (size_t i = 0; i + 1 < sl.used; i += 2) {
      // a pair recorded while a stream was being captured (a HIP graph's step) has no timing: skipped
      float ms = 0.f;
      if (hipEventSynchronize(sl.ev[i + 1]) != hipSuccess || hipEventElapsedTime(&ms, sl.ev[i], sl.ev[i + 1]) != hipSuccess) {
        (void)hipGetLastError();
        continue;
      }
      tot += ms;
      ++cnt;
    }
    total_ms[k] = tot;
    launches[k] = cnt;
    sl.used = 0;
  }
  return GR_OK;
}
const char* gr_version(void) { return GR_VERSION_STR; }

void gr_geom_layout(int n, size_t offsets_out[GR_GEOM_PARTS]) { geom_fixed(n, offsets_out); }

void gr_bins_layout(const gr_view* v, int n, const gr_plan* plan, size_t offsets_out[4]) {
  (void)n;
  size_t off[8];
  bins_fixed(vtiles_of(v), plan ? plan->num_pairs : 0, off, tile_cfg(v, plan ? plan->num_pairs : 0).ch);
  offsets_out[0] = off[0];
  offsets_out[1] = off[1];
  offsets_out[2] = off[2];
  offsets_out[3] = off[6];
}

size_t gr_geom_bytes(int n) {
  size_t off[GR_GEOM_PARTS];
  return geom_fixed(n, off) + align_up(scan_tmp_bytes(n > 0 ? n : 1));
}

size_t gr_saved_floats(const gr_view* v) { return (size_t)5 * v->width * v->height; }

size_t gr_bins_bytes(const gr_view* v, int n, const gr_plan* plan) {
  (void)n;
  size_t off[8];
  return bins_fixed(vtiles_of(v), plan->num_pairs, off, tile_cfg(v, plan->num_pairs).ch);
}

size_t gr_fwd_scratch_bytes(const gr_view* v, int n, const gr_plan* plan) {
  const int vtiles = vtiles_of(v);
  const TileCfg tc = tile_cfg(v, plan->num_pairs);
  size_t off[5];
  return scratch_fixed(vtiles, plan->num_pairs, off, tc.ch, tc.part_floats) + align_up(tile_sort_tmp_bytes(n, plan->num_pairs, vtiles));
}

// Backward workspace: pair partials (one 9-float slot per rectangle tile) + per-pixel upstream
// vectors (tiles x 5 x 256).
size_t gr_bwd_bytes(const gr_view* v, int n, const gr_plan* plan) {
  (void)n;
  const size_t tiles = (size_t)tiles_of(v);
  const size_t per_tile = tile_cfg(v).uf_frags * sizeof(uint4);
  return align_up((size_t)(plan->num_slots > 0 ? plan->num_slots : 1) * NPART * sizeof(float)) + align_up(tiles * per_tile) +
         align_up(tiles * 4 * sizeof(float)) + align_up(tiles * 2 * sizeof(float)) +
         align_up(4 * sizeof(float)) +  // per-tile loss sums, per-tile depth max / arg-max counts, depth scalars
         align_up((size_t)8 * (n > 0 ? n : 1) * sizeof(float)) +  // per-Gaussian row sums (gather + chain rule)
         align_up((size_t)(n > 0 ? n : 1) * sizeof(float)) +      // and depth sums
         align_up((size_t)blocks_for(n > 0 ? n : 1) * CAM_GRADS * sizeof(double));  // camera-gradient partials
}

// Decode the scanned totals (core, tail pairs) into the plan; a count that does not fit int32 is
// flagged as num_pairs = -1 (gr_fwd_render then reports the overflow).
// Exclusive scan of one value per thread over a block of NW waves (wave shuffles, then the wave totals
// through LDS); `total` = the block's sum.


// One workgroup of PLAN_THREADS (256 fits beside the render streams' splat kernels; see WI_THREADS).
#ifndef GR_PLAN_THREADS
#define GR_PLAN_THREADS 256
#endif
constexpr int PLAN_THREADS = GR_PLAN_THREADS;
// Pair totals and the block level of the offsets scan (one workgroup): bsum[b] (k_preprocess's packed
// block sums) is replaced by its exclusive scan, offsets[n] gets the packed grand total.  The packed
// words cannot carry into each other as long as K < 2^31, which is checked against the exact total
// (the sum of every block's two words) before the plan is trusted.
// cap (device-side sizing, gr_fwd_prepare_views_sized): the view's capacities; counts beyond them leave the device
// plan and the offsets' end at zero (the binning then emits nothing: a view without pairs) and raise *ovf.
__device__ __forceinline__ void plan_scan(unsigned long long* __restrict__ bsum, int blocks,
                                          unsigned long long* __restrict__ off_end, gr_plan* plan, gr_plan* host_plan,
                                          const float* __restrict__ omax, int* __restrict__ f16_sa,
                                          const gr_plan* cap = nullptr, int* ovf = nullptr) {
  __shared__ unsigned long long sh[PLAN_THREADS / 64];
  __shared__ float shm[PLAN_THREADS / 64];
  const int tid = (int)threadIdx.x, per = (blocks + PLAN_THREADS - 1) / PLAN_THREADS;
  const int b0 = min(blocks, tid * per), b1 = min(blocks, b0 + per);
  // a thread's run of block sums is loaded PLAN_Q at a time, together (one memory latency per PLAN_Q blocks, not one
  // per block: 1M Gaussians are 3,907 blocks, 16 per thread), and kept in registers for the write-back when it fits
  constexpr int PLAN_Q = 16;
  unsigned long long v[PLAN_Q];
  float m[PLAN_Q];
  auto load_run = [&](int b) {
#pragma unroll
    for (int q = 0; q < PLAN_Q; ++q) {
      v[q] = b + q < b1 ? bsum[b + q] : 0ull;
      m[q] = b + q < b1 ? omax[b + q] : 0.0f;
    }
  };
  unsigned long long acc = 0, ex = 0;
  float om = 0.0f;
  for (int b = b0; b < b1; b += PLAN_Q) {
    load_run(b);
#pragma unroll
    for (int q = 0; q < PLAN_Q; ++q) {
      acc += v[q];
      ex += (v[q] & 0xffffffffull) + (v[q] >> 32);
      om = fmaxf(om, m[q]);
    }
  }
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) om = fmaxf(om, __shfl_xor(om, m));
  if ((tid & 63) == 0) shm[tid >> 6] = om;
  unsigned long long grand, exact;
  const unsigned long long base = block_exclusive_scan<PLAN_THREADS / 64>(acc, sh, grand);
  (void)block_exclusive_scan<PLAN_THREADS / 64>(ex, sh, exact);
  unsigned long long run = base;
  for (int b = b0; b < b1; b += PLAN_Q) {
    if (b1 - b0 > PLAN_Q) load_run(b);  // (a run of at most PLAN_Q blocks is still in registers)
#pragma unroll
    for (int q = 0; q < PLAN_Q; ++q)
      if (b + q < b1) {
        bsum[b + q] = run;
        run += v[q];
      }
  }
  if (tid != 0) return;
#pragma unroll
  for (int w = 1; w < PLAN_THREADS / 64; ++w) om = fmaxf(om, shm[w]);  // published by the scans' barriers
  *f16_sa = f16_sa_of(om);
  const bool ok = exact < (1ull << 31);  // then neither packed word carried
  const long long np = ok ? (long long)exact : -1, nc = ok ? (long long)(grand & 0xffffffffull) : -1;
  const bool fits = !cap || (ok && nc <= cap->num_core_pairs && np - nc <= cap->num_pairs - cap->num_core_pairs);
  *off_end = fits ? grand : 0ull;
  plan->num_pairs = fits ? np : 0;
  plan->num_slots = fits ? np : 0;  // one partial-sum slot per pair
  plan->num_core_pairs = fits ? nc : 0;
  if (!fits) *ovf = 1;
  if (host_plan) {  // pinned host memory (gr_fwd_prepare_async): no copy command behind the scan; the true counts
    host_plan->num_pairs = np;
    host_plan->num_slots = np;
    host_plan->num_core_pairs = nc;
    __threadfence_system();
  }
}

__global__ __launch_bounds__(PLAN_THREADS) void k_plan(unsigned long long* __restrict__ bsum, int blocks,
                                               unsigned long long* __restrict__ off_end, gr_plan* plan,
                                               gr_plan* host_plan, const float* __restrict__ omax,
                                               int* __restrict__ f16_sa) {
  plan_scan(bsum, blocks, off_end, plan, host_plan, omax, f16_sa);
}

// Gaussian level of the offsets scan: offsets[i] = its block's offset + the exclusive scan of the packed
// counts inside the block (the blocks are k_preprocess's).
__device__ __forceinline__ void offsets_scan(int n, int b, const unsigned long long* __restrict__ counts,
                                             const unsigned long long* __restrict__ boff,
                                             unsigned long long* __restrict__ offsets) {
  __shared__ unsigned long long sh[4];
  const int i = (int)(b * 256 + threadIdx.x);
  unsigned long long tot;
  const unsigned long long e = block_exclusive_scan<4>(i < n ? counts[i] : 0ull, sh, tot);
  if (i < n) offsets[i] = boff[b] + e;
}
__global__ __launch_bounds__(256) void k_offsets(int n, const unsigned long long* __restrict__ counts,
                                                 const unsigned long long* __restrict__ boff,
                                                 unsigned long long* __restrict__ offsets) {
  offsets_scan(n, (int)blockIdx.x, counts, boff, offsets);
}

// The two scans for a batch of views (gr_fwd_prepare_views_async): block / row k = view k.
struct HostPlans {
  gr_plan* p[PREP_MAX_VIEWS];
  gr_plan cap[PREP_MAX_VIEWS];  // device-side sizing (ovf != null): the views' capacities
  int* ovf;
};
__global__ __launch_bounds__(PLAN_THREADS) void k_plan_views(PrepBatch B, int n, HostPlans hp) {
  const Geom& g = B.g[blockIdx.x];
  plan_scan(g.total, (n + 256) / 256, g.offsets + n, g.plan, hp.p[blockIdx.x], g.omax, g.f16_sa,
            hp.ovf ? &hp.cap[blockIdx.x] : nullptr, hp.ovf);
}

gr_status gr_fwd_prepare_async(const gr_view* v, int n, const float* means, const float* scales, const float* colors,
                               int color_dim, const float* opacities, void* geom, size_t geom_bytes, gr_plan* plan,
                               void* stream) {
  gr_status st = check_view(v);
  if (st != GR_OK) return st;
  if (v->device_counts) return set_error(GR_ERR_INVALID_ARGUMENT, "device_counts views are prepared by gr_fwd_prepare_views_sized");
  if (n < 0) return set_error(GR_ERR_INVALID_ARGUMENT, "n must be >= 0");
  if (color_dim != 3 && color_dim != 12 && color_dim != 48)
    return set_error(GR_ERR_INVALID_ARGUMENT, "colors must be (N,3) or SH coeffs (N,4,3) / (N,16,3)");
  if (!plan) return set_error(GR_ERR_INVALID_ARGUMENT, "plan is null");
  if (n == 0) {
    plan->num_pairs = 0;
    plan->num_slots = 0;
    plan->num_core_pairs = 0;
    return GR_OK;
  }
  if (!means || !scales || !colors || !opacities || !geom) return set_error(GR_ERR_INVALID_ARGUMENT, "null pointer");
  if (geom_bytes < gr_geom_bytes(n)) return set_error(GR_ERR_WORKSPACE, "geom workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const ViewK vk = make_viewk(v);
  Geom g = geom_view(geom, n);
  if (color_dim == 3)
    hipLaunchKernelGGL(k_preprocess<3>, dim3(blocks_for(n + 1)), dim3(256), 0, s, vk, n, means, scales, colors, opacities, g);
  else if (color_dim == 12)
    hipLaunchKernelGGL(k_preprocess<12>, dim3(blocks_for(n + 1)), dim3(256), 0, s, vk, n, means, scales, colors, opacities, g);
  else
    hipLaunchKernelGGL(k_preprocess<48>, dim3(blocks_for(n + 1)), dim3(256), 0, s, vk, n, means, scales, colors, opacities, g);
  GR_HIP_TRY(hipGetLastError());
  // a plan in pinned (device-mapped) host memory is written by k_plan itself; pageable memory gets a copy
  gr_plan* mapped = nullptr;
  hipPointerAttribute_t attr;
  if (hipPointerGetAttributes(&attr, plan) == hipSuccess && attr.type == hipMemoryTypeHost && attr.devicePointer)
    mapped = (gr_plan*)attr.devicePointer;
  (void)hipGetLastError();  // a pageable pointer leaves an error code behind
  // exclusive scan of the packed counts over the 256-Gaussian blocks (k_plan); the Gaussian level of the scan is
  // the binning's (k_emit_count writes the offsets as it emits)
  hipLaunchKernelGGL(k_plan, dim3(1), dim3(PLAN_THREADS), 0, s, g.total, blocks_for(n + 1), g.offsets + n, g.plan, mapped,
                     (const float*)g.omax, g.f16_sa);
  GR_HIP_TRY(hipGetLastError());
  if (!mapped) GR_HIP_TRY(hipMemcpyAsync(plan, g.plan, sizeof(gr_plan), hipMemcpyDeviceToHost, s));
  return GR_OK;
}

static gr_status prepare_views_impl(int num_views, const gr_view* views, int n, const float* means, const float* scales,
                                    const float* colors, int color_dim, const float* opacities, void* const* geoms,
                                    size_t geom_bytes, gr_plan* const* plans, const gr_plan* caps, int* ovf,
                                    void* stream) {
  if (num_views < 1 || num_views > PREP_MAX_VIEWS)
    return set_error(GR_ERR_INVALID_ARGUMENT, "gr_fwd_prepare_views_async: num_views must be in [1, GR_PREPARE_MAX_VIEWS]");
  if (!views || !geoms || (!plans && !caps)) return set_error(GR_ERR_INVALID_ARGUMENT, "null pointer");
  if (num_views == 1 && !caps)
    return gr_fwd_prepare_async(&views[0], n, means, scales, colors, color_dim, opacities, geoms[0], geom_bytes, plans[0],
                                stream);
  for (int k = 0; k < num_views; ++k) {
    gr_status st = check_view(&views[k]);
    if (st != GR_OK) return st;
    if ((!caps && !plans[k]) || !geoms[k]) return set_error(GR_ERR_INVALID_ARGUMENT, "null pointer");
    if (caps) {
      if (!views[k].device_counts)
        return set_error(GR_ERR_INVALID_ARGUMENT, "gr_fwd_prepare_views_sized: the views must have device_counts = 1");
      if (!short_keys(vtiles_of(&views[k])))
        return set_error(GR_ERR_INVALID_ARGUMENT, "gr_fwd_prepare_views_sized: more than 8,192 screen tiles");
      if (caps[k].num_core_pairs < 0 || caps[k].num_pairs < caps[k].num_core_pairs || caps[k].num_pairs >= (1ll << 31) ||
          caps[k].num_slots < caps[k].num_pairs)
        return set_error(GR_ERR_INVALID_ARGUMENT, "gr_fwd_prepare_views_sized: bad capacities");
    } else if (views[k].device_counts) {
      return set_error(GR_ERR_INVALID_ARGUMENT, "device_counts views are prepared by gr_fwd_prepare_views_sized");
    }
  }
  if (caps && !ovf) return set_error(GR_ERR_INVALID_ARGUMENT, "gr_fwd_prepare_views_sized: overflow is null");
  if (n < 0) return set_error(GR_ERR_INVALID_ARGUMENT, "n must be >= 0");
  if (color_dim != 3 && color_dim != 12 && color_dim != 48)
    return set_error(GR_ERR_INVALID_ARGUMENT, "colors must be (N,3) or SH coeffs (N,4,3) / (N,16,3)");
  if (n == 0) {
    if (plans)
      for (int k = 0; k < num_views; ++k)
        if (plans[k]) *plans[k] = gr_plan{0, 0, 0};
    return GR_OK;
  }
  if (!means || !scales || !colors || !opacities) return set_error(GR_ERR_INVALID_ARGUMENT, "null pointer");
  if (geom_bytes < gr_geom_bytes(n)) return set_error(GR_ERR_WORKSPACE, "geom workspace too small");
  hipStream_t s = (hipStream_t)stream;
  PrepBatch B;
  HostPlans hp;
  hp.ovf = caps ? ovf : nullptr;
  bool all_mapped = true;
  B.nv = num_views;
  for (int k = 0; k < num_views; ++k) {
    B.v[k] = make_viewk(&views[k]);
    B.g[k] = geom_view(geoms[k], n);
    hp.cap[k] = caps ? caps[k] : gr_plan{0, 0, 0};
    hipPointerAttribute_t attr;
    hp.p[k] = nullptr;
    if (plans && plans[k] && hipPointerGetAttributes(&attr, plans[k]) == hipSuccess && attr.type == hipMemoryTypeHost &&
        attr.devicePointer)
      hp.p[k] = (gr_plan*)attr.devicePointer;
    (void)hipGetLastError();
    // (device-side sizing: an observed plan that is not mapped host memory is left unwritten; nothing waits for it)
    all_mapped = all_mapped && (hp.p[k] || caps);
  }
  const int blocks = blocks_for(n + 1);
  // rows of views: at least ~1024 blocks (4 per CU) when the views allow, each view still run by one row alone
  const dim3 pgrid(blocks, std::max(1, std::min(num_views, (1024 + blocks - 1) / blocks)));
  for (int rep = 0; rep < GR_DEBUG_PREP_REPS; ++rep) {  // > 1: timing experiments only (idempotent repeats)
  if (color_dim == 3)
    hipLaunchKernelGGL(k_preprocess_views<3>, pgrid, dim3(256), 0, s, B, n, means, scales, colors, opacities);
  else if (color_dim == 12)
    hipLaunchKernelGGL(k_preprocess_views<12>, pgrid, dim3(256), 0, s, B, n, means, scales, colors, opacities);
  else
    hipLaunchKernelGGL(k_preprocess_views<48>, pgrid, dim3(256), 0, s, B, n, means, scales, colors, opacities);
  GR_HIP_TRY(hipGetLastError());
  hipLaunchKernelGGL(k_plan_views, dim3(num_views), dim3(PLAN_THREADS), 0, s, B, n, hp);
  GR_HIP_TRY(hipGetLastError());
  }
  if (!all_mapped)
    for (int k = 0; k < num_views; ++k)
      if (!hp.p[k]) GR_HIP_TRY(hipMemcpyAsync(plans[k], B.g[k].plan, sizeof(gr_plan), hipMemcpyDeviceToHost, s));
  return GR_OK;
}

gr_status gr_fwd_prepare_views_async(int num_views, const gr_view* views, int n, const float* means,
                                     const float* scales, const float* colors, int color_dim, const float* opacities,
                                     void* const* geoms, size_t geom_bytes, gr_plan* const* plans, void* stream) {
  return prepare_views_impl(num_views, views, n, means, scales, colors, color_dim, opacities, geoms, geom_bytes, plans,
                            nullptr, nullptr, stream);
}

gr_status gr_fwd_prepare_views_sized(int num_views, const gr_view* views, int n, const float* means,
                                     const float* scales, const float* colors, int color_dim, const float* opacities,
                                     void* const* geoms, size_t geom_bytes, const gr_plan* caps, gr_plan* const* observed,
                                     int* overflow, void* stream) {
  if (!caps) return set_error(GR_ERR_INVALID_ARGUMENT, "gr_fwd_prepare_views_sized: caps is null");
  return prepare_views_impl(num_views, views, n, means, scales, colors, color_dim, opacities, geoms, geom_bytes, observed,
                            caps, overflow, stream);
}

gr_status gr_fwd_prepare(const gr_view* v, int n, const float* means, const float* scales, const float* colors,
                         int color_dim, const float* opacities, void* geom, size_t geom_bytes, gr_plan* plan,
                         void* stream) {
  if (plan) {
    plan->num_pairs = 0;
    plan->num_slots = 0;
    plan->num_core_pairs = 0;
  }
  gr_status st = gr_fwd_prepare_async(v, n, means, scales, colors, color_dim, opacities, geom, geom_bytes, plan, stream);
  if (st != GR_OK || n == 0) return st;
  GR_HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
  if (plan->num_pairs < 0) return set_error(GR_ERR_OVERFLOW, "pair count overflows int32");
  return GR_OK;
}

}  // extern "C" (fwd_impl and the backward workspace layout are internal)

// The backward workspace (gr_bwd_bytes): pair partials, then the per-tile upstream fragments, then the
// per-tile loss sums.
struct BwdWs {
  float* partials;
  uint4* UF;
  float* tile_loss;  // [tiles][4]
  float* tile_aux;   // [tiles][2]: depth max, arg-max pixels (gr_bwd_fit)
  float* dscal;      // [4]: max(depth), the max's gradient per arg-max pixel
  float* sums;       // [n][8]: per-Gaussian row sums (k_gather_view)
  float* sums3;      // [n]: per-Gaussian depth sums (k_gather_view<true>, with an upstream depth gradient)
  double* cam_part;  // [blocks][CAM_GRADS]: per-block camera-gradient partials (gr_bwd_camera)
};
static BwdWs bwd_ws(const gr_view* v, int n, const gr_plan* plan, void* ws) {
  const size_t tiles = (size_t)tiles_of(v);
  BwdWs w;
  w.partials = (float*)ws;
  w.UF = (uint4*)((char*)ws + align_up((size_t)(plan->num_slots > 0 ? plan->num_slots : 1) * NPART * sizeof(float)));
  w.tile_loss = (float*)((char*)w.UF + align_up(tiles * tile_cfg(v).uf_frags * sizeof(uint4)));
  w.tile_aux = (float*)((char*)w.tile_loss + align_up(tiles * 4 * sizeof(float)));
  w.dscal = (float*)((char*)w.tile_aux + align_up(tiles * 2 * sizeof(float)));
  w.sums = (float*)((char*)w.dscal + align_up(4 * sizeof(float)));
  w.sums3 = (float*)((char*)w.sums + align_up((size_t)8 * (n > 0 ? n : 1) * sizeof(float)));
  w.cam_part = (double*)((char*)w.sums3 + align_up((size_t)(n > 0 ? n : 1) * sizeof(float)));
  return w;
}

// The view's binning (pair emission, the stable counting sort by tile, work items): gr_fwd_bin, or the
// first half of fwd_impl when the view is not already binned.
static gr_status bin_impl(const gr_view* v, int n, const gr_plan* plan, const void* geom, const Bins& b,
                          const Scratch& sc, const ViewK& vk, hipStream_t s) {
  const int64_t num_pairs = plan->num_pairs;
  const int tiles = vk.tiles_x * vk.tiles_y, vtiles = 2 * tiles;
  prof_mark(PROF_BINNING, s);
  if (n > 0 && num_pairs > 0) {
    Geom g = geom_view((void*)geom, n);
    const Cnt2* cnt = (const Cnt2*)g.counts;
    const Cnt2* offs = (const Cnt2*)g.offsets;
    if (short_keys(vtiles)) {
      // counting sort of each region (core pairs [0, Kc), tail pairs [Kc, K)) on 16-bit tile keys, columns of G
      // Gaussians: emission + per-column counts + offsets, the column scan, the placement + work items
      const int64_t Kc = plan->num_core_pairs, Kr[2] = {Kc, num_pairs - Kc};
      const int cw = col_width(num_pairs, tiles);
      const size_t cells = (size_t)tiles * cols_of(num_pairs, cw);
      const int waves = tsort_waves(tiles);
      TZones Z;
      Z.cw = cw;
      Z.ch = tile_cfg(v, num_pairs).ch;
      // device-side sizing: Kr are the regions' capacities (columns = grid); the true counts are read on the device
      Z.kdev = v->device_counts ? (const unsigned long long*)(g.offsets + n) : nullptr;
      char* q = (char*)sc.sort_tmp;
      for (int z = 0; z < 2; ++z) {
        TZone& zz = Z.z[z];
        zz.K = Kr[z];
        zz.cols = cols_of(Kr[z], cw);
        zz.zbase = z == 0 ? 0 : (int)Kc;
        zz.keys = (const uint16_t*)sc.keys_in + (z == 0 ? 0 : Kc);
        zz.ids = sc.ids_in + (z == 0 ? 0 : Kc);
        zz.M = (int*)q;
        q += align_up(cells * sizeof(int));
        zz.S = (int*)q;
        q += align_up(cells * sizeof(int));
        zz.T = (int*)q;
        q += align_up((size_t)tiles * sizeof(int));
      }
      int* fan = b.ticket + fan_offset(tiles);
      hipLaunchKernelGGL(k_emit_offsets, dim3(blocks_for(n)), dim3(256), 0, s, vk, n, (const int4*)g.rect, cnt,
                         (const unsigned long long*)g.total, (Cnt2*)g.offsets, (const float4*)g.rec,
                         (uint16_t*)sc.keys_in, sc.ids_in, fan);
      GR_HIP_TRY(hipGetLastError());
      const int blocks = Z.z[0].cols + Z.z[1].cols;
      hipLaunchKernelGGL(k_tile_count, dim3(blocks), dim3(256), (size_t)tiles * sizeof(int), s, Z, tiles);
      GR_HIP_TRY(hipGetLastError());
      hipLaunchKernelGGL(k_tile_colscan, dim3((tiles + CS_T - 1) / CS_T, 2), dim3(CS_T * CS_G), 0, s, Z, tiles, b.ranges,
                         b.items, b.num_items, b.tile_item0, b.ticket);
      GR_HIP_TRY(hipGetLastError());
      const size_t lds = (size_t)tiles * sizeof(int) * waves;
      const int bits = bits_for((uint32_t)tiles);
      if (waves == 8)
        hipLaunchKernelGGL(k_tile_place<8>, dim3(blocks), dim3(512), lds, s, Z, tiles, bits, (const int2*)b.ranges, b.pairs,
                           b.pos_of);
      else if (waves == 4)
        hipLaunchKernelGGL(k_tile_place<4>, dim3(blocks), dim3(256), lds, s, Z, tiles, bits, (const int2*)b.ranges, b.pairs,
                           b.pos_of);
      else if (waves == 2)
        hipLaunchKernelGGL(k_tile_place<2>, dim3(blocks), dim3(128), lds, s, Z, tiles, bits, (const int2*)b.ranges, b.pairs,
                           b.pos_of);
      else
        hipLaunchKernelGGL(k_tile_place<1>, dim3(blocks), dim3(64), lds, s, Z, tiles, bits, (const int2*)b.ranges, b.pairs,
                           b.pos_of);
      GR_HIP_TRY(hipGetLastError());
    } else {
      if (v->device_counts)
        return set_error(GR_ERR_INVALID_ARGUMENT, "device_counts views need the counting-sort binning (<= 8,192 tiles)");
      // radix sort of the whole pair array on virtual-tile keys (> TSORT_MAX_TILES tiles); the Gaussians' offsets
      // first (the counting-sort path's emission writes them itself)
      hipLaunchKernelGGL(k_offsets, dim3(blocks_for(n)), dim3(256), 0, s, n, (const unsigned long long*)g.counts,
                         (const unsigned long long*)g.total, g.offsets);
      GR_HIP_TRY(hipGetLastError());
      hipLaunchKernelGGL((k_emit_zones<uint32_t, true>), dim3(blocks_for(n)), dim3(256), 0, s, vk, n,
                         (const int4*)g.rect, cnt, offs, (const float4*)g.rec, sc.keys_in, sc.ids_in);
      GR_HIP_TRY(hipGetLastError());
      hipLaunchKernelGGL(k_pair_values, dim3(blocks_for(num_pairs)), dim3(256), 0, s, num_pairs, (const int*)sc.ids_in,
                         sc.pairs_in);
      GR_HIP_TRY(hipGetLastError());
      GR_HIP_TRY(hipMemsetAsync(b.ranges, 0, sizeof(int2) * vtiles, s));
      const int bits = bits_for((uint32_t)vtiles);
      size_t tmp = tile_sort_tmp_bytes(n, num_pairs, vtiles);
      GR_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(sc.sort_tmp, tmp, sc.keys_in, b.keys, sc.pairs_in, sc.pairs_sorted,
                                                    (int)num_pairs, 0, bits, s));
      hipLaunchKernelGGL(k_ranges<uint32_t>, dim3(blocks_for(num_pairs)), dim3(256), 0, s, num_pairs, b.keys, b.ranges);
      GR_HIP_TRY(hipGetLastError());
      hipLaunchKernelGGL(k_pos_of, dim3(blocks_for(num_pairs)), dim3(256), 0, s, num_pairs, (const int2*)sc.pairs_sorted,
                         b.pairs, b.pos_of);
      GR_HIP_TRY(hipGetLastError());
      hipLaunchKernelGGL(k_work_items, dim3(1), dim3(WI_THREADS), 0, s, vtiles, (const int2*)b.ranges, b.items, b.num_items,
                         b.tile_item0, b.ticket, tile_cfg(v, num_pairs).ch);
    }
  } else {
    // no pair: the Gaussians' offsets (written by the emission otherwise) are all zero
    if (n > 0) GR_HIP_TRY(hipMemsetAsync(geom_view((void*)geom, n).offsets, 0, (size_t)n * sizeof(unsigned long long), s));
    GR_HIP_TRY(hipMemsetAsync(b.ranges, 0, sizeof(int2) * vtiles, s));
    hipLaunchKernelGGL(k_work_items, dim3(1), dim3(WI_THREADS), 0, s, vtiles, (const int2*)b.ranges, b.items, b.num_items,
                       b.tile_item0, b.ticket, tile_cfg(v, num_pairs).ch);
  }
  GR_HIP_TRY(hipGetLastError());
  prof_mark(PROF_BINNING, s);
  return GR_OK;
}

// l1 != nullptr (gr_fwd_render_l1): no_depth_grad view without depth output; the fit loss's upstream
// fragments and tile sums go to the backward workspace `ws`, the view loss to l1_loss_out.
static gr_status fwd_impl(const gr_view* v, int n, const gr_plan* plan, const void* geom, void* bins, size_t bins_bytes,
                          void* scratch, size_t scratch_bytes, float* out_rgb, float* out_alpha, float* out_depth,
                          float* saved, void* stream, const L1Args* l1, float* l1_loss_out, void* ws, size_t ws_bytes,
                          bool depth_sums = false) {
  gr_status st = check_view(v);
  if (st != GR_OK) return st;
  if (!plan) return set_error(GR_ERR_INVALID_ARGUMENT, "plan is null");
  if (plan->num_pairs < 0 || plan->num_slots < 0) return set_error(GR_ERR_OVERFLOW, "pair count overflows int32");
  if (!l1 && !saved) return set_error(GR_ERR_INVALID_ARGUMENT, "saved is required");
  if (l1 && (!ws || ws_bytes < gr_bwd_bytes(v, n, plan) || !l1_loss_out))
    return set_error(GR_ERR_WORKSPACE, "gr_fwd_render_l1: backward workspace too small (or null loss)");
  if (n > 0 && (!geom || !bins)) return set_error(GR_ERR_INVALID_ARGUMENT, "null workspace");
  const int64_t num_pairs = plan->num_pairs;
  if (bins_bytes < gr_bins_bytes(v, n, plan)) return set_error(GR_ERR_WORKSPACE, "bins workspace too small");
  if (scratch_bytes < gr_fwd_scratch_bytes(v, n, plan) || !scratch)
    return set_error(GR_ERR_WORKSPACE, "forward scratch workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const ViewK vk = make_viewk(v);
  const int tiles = vk.tiles_x * vk.tiles_y, vtiles = 2 * tiles;
  const TileCfg tc = tile_cfg(v, num_pairs);
  if (v->rows > 0 && !l1)
    return set_error(GR_ERR_INVALID_ARGUMENT, "a band of tile rows (gr_view.rows): gr_fwd_render_l1 only (the fit loss)");
  if (tc.T == T32 && (!l1 || v->no_depth_grad != 1))
    return set_error(GR_ERR_INVALID_ARGUMENT, "32-pixel tiles (gr_view.tile = 32): gr_fwd_render_l1 with no_depth_grad = 1 only");
  if (tc.T == T32 && vk.core != vk.cutoff)
    return set_error(GR_ERR_INVALID_ARGUMENT, "32-pixel tiles (gr_view.tile = 32): one-zone footprint only (core_cutoff <= 0 or >= cutoff)");
  Bins b = bins_view(bins, vtiles, num_pairs, tc.ch);
  Scratch sc = scratch_view(scratch, vtiles, num_pairs, tc.ch, tc.part_floats);
  if (!v->binned) {
    for (int rep = 0; rep < GR_DEBUG_BIN_REPS; ++rep) {  // > 1: timing experiments only (idempotent repeats)
      st = bin_impl(v, n, plan, geom, b, sc, vk, s);
      if (st != GR_OK) return st;
    }
  }
  Geom g = geom_view((void*)geom, n > 0 ? n : 1);
  const size_t HW = (size_t)v->width * v->height;
  const int64_t cap = item_cap(vtiles, num_pairs, tc.ch);
  L1Args la{nullptr, nullptr, 0.f, 0.f, nullptr};
  uint4* UF = nullptr;
  if (l1) {
    const BwdWs w = bwd_ws(v, n, plan, ws);
    la = *l1;
    la.tile_loss = w.tile_loss;
    la.loss_out = l1_loss_out;
    la.n1 = (int64_t)(3 * HW);
    la.n2 = (int64_t)(l1->t_mask ? HW : 0);
    UF = w.UF;
  }
  float4* saved4 = saved ? (float4*)saved : nullptr;
  float* savedD = saved ? saved + 4 * HW : nullptr;
  if (!(GR_DEBUG_SKIP & 1)) {
    // every tile has a work item (an empty tile its one empty item): the splat writes every output pixel, finishes
    // the tiles split over several items (the last item to arrive) and, with the fit loss, the view loss (the last
    // tile to finish)
    prof_mark(PROF_RASTER_FWD, s);
    // no_depth_grad: 0 default (f32-grade W / D), 1 two-piece splits, 2 f32-grade without a depth gradient
    const bool f32g = v->no_depth_grad != 1;
    if (tc.T == T32)
      hipLaunchKernelGGL(k_fwd32_l1, dim3((unsigned)cap), dim3(256), 0, s, vk, n, (const int4*)b.items, (const int*)b.num_items,
                         (const int2*)b.ranges, (const int*)b.pairs, (const float4*)g.rec, sc.fwd_part, out_rgb, out_alpha, la,
                         UF, (const int*)(n > 0 && num_pairs > 0 ? g.f16_sa : nullptr), (const int*)b.tile_item0, b.ticket,
                         tc.ch);
    else
    hipLaunchKernelGGL(l1 ? (f32g ? k_raster_fwd_mfma<5> : k_raster_fwd_mfma<4>)
                          : (f32g ? k_raster_fwd_mfma<1>
                                  : (out_depth || depth_sums ? k_raster_fwd_mfma<2> : k_raster_fwd_mfma<3>)),
                       dim3((unsigned)cap), dim3(256), 0, s, vk, n, (const int4*)b.items,
                       (const int*)b.num_items, (const int2*)b.ranges, (const int*)b.pairs, (const float4*)g.rec,
                       sc.fwd_part, out_rgb, out_alpha, out_depth, saved4, savedD, la, UF,
                       (const int*)(n > 0 && num_pairs > 0 ? g.f16_sa : nullptr), (const int*)b.tile_item0, b.ticket,
                       tc.ch);
    GR_HIP_TRY(hipGetLastError());
    prof_mark(PROF_RASTER_FWD, s);
  }
  return GR_OK;
}

extern "C" {

gr_status gr_fwd_render(const gr_view* v, int n, const gr_plan* plan, const void* geom, void* bins, size_t bins_bytes,
                        void* scratch, size_t scratch_bytes, float* out_rgb, float* out_alpha, float* out_depth,
                        float* saved, void* stream) {
  return fwd_impl(v, n, plan, geom, bins, bins_bytes, scratch, scratch_bytes, out_rgb, out_alpha, out_depth, saved, stream,
                  nullptr, nullptr, nullptr, 0);
}

gr_status gr_fwd_render_saved(const gr_view* v, int n, const gr_plan* plan, const void* geom, void* bins,
                              size_t bins_bytes, void* scratch, size_t scratch_bytes, float* saved, void* stream) {
  return fwd_impl(v, n, plan, geom, bins, bins_bytes, scratch, scratch_bytes, nullptr, nullptr, nullptr, saved, stream,
                  nullptr, nullptr, nullptr, 0, true);
}

gr_status gr_fwd_compose(const gr_view* v, const float* saved, float* out_rgb, float* out_alpha, float* out_depth,
                         void* stream) {
  gr_status st = check_view(v);
  if (st != GR_OK) return st;
  if (!saved) return set_error(GR_ERR_INVALID_ARGUMENT, "gr_fwd_compose: saved is null");
  const int hw = v->width * v->height;
  hipLaunchKernelGGL(k_compose, dim3(blocks_for(hw)), dim3(256), 0, (hipStream_t)stream, make_viewk(v), hw,
                     (const float4*)saved, saved + 4 * (size_t)hw, out_rgb, out_alpha, out_depth);
  GR_HIP_TRY(hipGetLastError());
  return GR_OK;
}

gr_status gr_fwd_bin(const gr_view* v, int n, const gr_plan* plan, const void* geom, void* bins, size_t bins_bytes,
                     void* scratch, size_t scratch_bytes, void* stream) {
  gr_status st = check_view(v);
  if (st != GR_OK) return st;
  if (!plan) return set_error(GR_ERR_INVALID_ARGUMENT, "plan is null");
  if (plan->num_pairs < 0 || plan->num_slots < 0) return set_error(GR_ERR_OVERFLOW, "pair count overflows int32");
  if (n > 0 && (!geom || !bins)) return set_error(GR_ERR_INVALID_ARGUMENT, "null workspace");
  if (bins_bytes < gr_bins_bytes(v, n, plan)) return set_error(GR_ERR_WORKSPACE, "bins workspace too small");
  if (scratch_bytes < gr_fwd_scratch_bytes(v, n, plan) || !scratch)
    return set_error(GR_ERR_WORKSPACE, "forward scratch workspace too small");
  const ViewK vk = make_viewk(v);
  const int vtiles = 2 * vk.tiles_x * vk.tiles_y;
  const TileCfg tc = tile_cfg(v, plan->num_pairs);
  return bin_impl(v, n, plan, geom, bins_view(bins, vtiles, plan->num_pairs, tc.ch),
                  scratch_view(scratch, vtiles, plan->num_pairs, tc.ch, tc.part_floats), vk, (hipStream_t)stream);
}

gr_status gr_fwd_render_l1(const gr_view* v, int n, const gr_plan* plan, const void* geom, void* bins, size_t bins_bytes,
                           void* scratch, size_t scratch_bytes, const float* target_rgb, const float* target_mask,
                           float w_sil, float g_scale, float* loss_out, float* out_rgb, float* out_alpha, void* ws,
                           size_t ws_bytes, void* stream) {
  if (!v || !v->no_depth_grad)
    return set_error(GR_ERR_INVALID_ARGUMENT, "gr_fwd_render_l1: the view must have no_depth_grad = 1 or 2");
  if (!target_rgb) return set_error(GR_ERR_INVALID_ARGUMENT, "gr_fwd_render_l1: target_rgb is null");
  L1Args l1{target_rgb, target_mask, w_sil, g_scale, nullptr};
  l1.pieces = v->no_depth_grad == 1 ? 2 : 3;
  return fwd_impl(v, n, plan, geom, bins, bins_bytes, scratch, scratch_bytes, out_rgb, out_alpha, nullptr, nullptr, stream,
                  &l1, loss_out, ws, ws_bytes);
}

}  // extern "C" (bwd_impl is internal)

static gr_status bwd_impl(const gr_view* v, int n, const gr_plan* plan, const float* means, const float* scales,
                          const float* colors, int color_dim, const float* opacities, const void* geom, const void* bins,
                          const float* saved, const float* g_rgb, const float* g_alpha, const float* g_depth,
                          const float* t_rgb, const float* t_mask, float w_sil, float g_scale, float* loss_out,
                          float* d_means, float* d_scales, float* d_colors, float* d_opacities, int accumulate, void* ws,
                          size_t ws_bytes, void* stream, const float* t_depth = nullptr, float w_depth = 0.0f,
                          const int* sum_index = nullptr, float* g_sums = nullptr, float* g_sums3 = nullptr) {
  gr_status st = check_view(v);
  if (st != GR_OK) return st;
  if ((g_depth || (t_rgb && t_depth)) && v->no_depth_grad)
    return set_error(GR_ERR_INVALID_ARGUMENT,
                     "depth gradient for a view rendered with no_depth_grad (render it with depth_grad=True)");
  if (tile_of(v) != T)
    return set_error(GR_ERR_INVALID_ARGUMENT, "32-pixel tiles (gr_view.tile = 32): the fused fit path only (gr_bwd_splat)");
  if (v->rows > 0)
    return set_error(GR_ERR_INVALID_ARGUMENT, "a band of tile rows (gr_view.rows): the fused fit path only (gr_bwd_splat)");
  if (!plan) return set_error(GR_ERR_INVALID_ARGUMENT, "plan is null");
  if (color_dim != 3 && color_dim != 12 && color_dim != 48)
    return set_error(GR_ERR_INVALID_ARGUMENT, "colors must be (N,3) or SH coeffs (N,4,3) / (N,16,3)");
  if (n == 0) return GR_OK;
  const bool gather_only = g_sums != nullptr;  // gr_bwd_fit_gather: the per-Gaussian sums to the caller, no chain rule
  if ((!g_rgb && !t_rgb) || !saved || !geom || !bins ||
      (!gather_only && (!d_means || !d_scales || !d_colors || !d_opacities)))
    return set_error(GR_ERR_INVALID_ARGUMENT, "null pointer");
  if (t_rgb && (!loss_out || !ws)) return set_error(GR_ERR_INVALID_ARGUMENT, "gr_bwd_l1: null loss or workspace");
  const int64_t num_pairs = plan->num_pairs;
  if ((num_pairs > 0 || t_rgb) && (!ws || ws_bytes < gr_bwd_bytes(v, n, plan)))
    return set_error(GR_ERR_WORKSPACE, "backward workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const ViewK vk = make_viewk(v);
  const int tiles = vk.tiles_x * vk.tiles_y;
  Geom g = geom_view((void*)geom, n);
  Bins b = bins_view((void*)bins, 2 * tiles, num_pairs, tile_cfg(v, num_pairs).ch);
  const size_t HW = (size_t)v->width * v->height;
  const BwdWs w = bwd_ws(v, n, plan, ws);
  float* partials = w.partials;
  uint4* UF = w.UF;
  float* tile_loss = w.tile_loss;
  const bool dfit = t_rgb && t_depth;  // fused depth loss (gr_bwd_fit)
  L1Args l1{t_rgb, t_mask, w_sil, g_scale, t_rgb ? tile_loss : nullptr};
  if (t_rgb) {  // the view loss: written by k_pixel_grads' last tile
    l1.loss_out = loss_out;
    l1.n1 = (int64_t)(3 * HW);
    l1.n2 = (int64_t)(t_mask ? HW : 0);
  }
  // the arrival tickets of the one-launch reductions below: the bins' (zeroed by the work-item builder, left zero
  // by every kernel that takes one)
  int* ticket = b.ticket;
  if (dfit) {
    l1.t_depth = t_depth;
    l1.w_depth = w_depth;
    l1.dscal = w.dscal;
    const float4* s4 = (const float4*)saved;
    const float* sD = saved + 4 * HW;
    hipLaunchKernelGGL(k_depth_tile_max, dim3(tiles), dim3(256), 0, s, vk, s4, sD, w.tile_aux, w.dscal, ticket);
    hipLaunchKernelGGL(k_depth_tile_sums, dim3(tiles), dim3(256), 0, s, vk, s4, sD, t_depth, w.dscal, tile_loss, w.tile_aux,
                       (int64_t)HW, w_depth, g_scale, ticket);
    GR_HIP_TRY(hipGetLastError());
  }
  const bool depth = g_depth != nullptr || dfit;  // an upstream depth gradient reaches the splat
  // Without an upstream depth gradient nothing in the backward cancels (the depth gradient's
  // (z - depth) / (W + 1e-6) is what needs f32-grade W and D): the splat runs on two round-to-nearest
  // pieces (~2^-16 per product, unbiased) whatever the view's mode, except at f32 grade (no_depth_grad = 2).
  const int pieces = (v->no_depth_grad == 2 || depth) ? 3 : 2;
  if (num_pairs > 0 || t_rgb) {
    hipLaunchKernelGGL(k_pixel_grads, dim3(tiles), dim3(256), 0, s, vk, (const float4*)saved, saved + 4 * HW, g_rgb,
                       g_alpha, g_depth, UF, pieces, l1, depth, ticket);
    GR_HIP_TRY(hipGetLastError());
  }
  if (num_pairs > 0) {
    const int64_t cap = item_cap(2 * tiles, num_pairs, tile_cfg(v, num_pairs).ch);
    prof_mark(PROF_RASTER_BWD, s);
    auto kern = depth ? k_raster_bwd_bf16<true, 3> : (pieces == 2 ? k_raster_bwd_bf16<false, 2> : k_raster_bwd_bf16<false, 3>);
    hipLaunchKernelGGL(kern, dim3((unsigned)cap), dim3(256), 0, s, vk, n, (const int4*)b.items, (const int*)b.num_items,
                       (const int*)b.pairs, (const float4*)g.rec, (const uint4*)UF, partials,
                       partials + 8 * (size_t)plan->num_slots);
    GR_HIP_TRY(hipGetLastError());
    prof_mark(PROF_RASTER_BWD, s);
  }
  prof_mark(PROF_REDUCE, s);
  if (num_pairs > 0) {
    // 32-byte rows: the lean gather into per-Gaussian sums (with a depth gradient also the tail pairs and
    // the depth sums), then the chain rule of that one view (the two stages of gr_gather_view +
    // gr_reduce_sums; k_reduce_bwd's one pass needs 117 VGPRs for the chain rule while it gathers)
    float* depth3 = partials + 8 * (size_t)plan->num_slots;
    float* sums = gather_only ? g_sums : w.sums;
    float* sums3 = gather_only ? g_sums3 : w.sums3;
    if (depth)
      hipLaunchKernelGGL(k_gather_view<true>, dim3((n + 63) / 64), dim3(256), 0, s, n, (const Cnt2*)g.offsets,
                         (const int*)b.pos_of, (const float4*)partials, (float2*)sums, (const float*)depth3, sums3);
    else
      hipLaunchKernelGGL(k_gather_view<false>, dim3((n + 63) / 64), dim3(256), 0, s, n, (const Cnt2*)g.offsets,
                         (const int*)b.pos_of, (const float4*)partials, (float2*)sums, (const float*)nullptr,
                         (float*)nullptr);
    if (gather_only) {
      if (!depth && sums3) GR_HIP_TRY(hipMemsetAsync(sums3, 0, (size_t)n * sizeof(float), s));
      GR_HIP_TRY(hipGetLastError());
      prof_mark(PROF_REDUCE, s);
      return GR_OK;
    }
    SBatch B;
    B.nv = 1;
    B.r[0].v = vk;
    B.r[0].sums = (const float4*)w.sums;
    B.r[0].sums3 = depth ? w.sums3 : nullptr;
    const int gpb = 64 * (4 / reduce_sums_crw(1, color_dim));
    const dim3 grid((n + gpb - 1) / gpb), block(256);
    if (color_dim == 3)
      hipLaunchKernelGGL(k_reduce_sums<3>, grid, block, 0, s, B, n, means, scales, colors, opacities, d_means, d_scales,
                         d_colors, d_opacities, accumulate, sum_index);
    else if (color_dim == 12)
      hipLaunchKernelGGL(k_reduce_sums<12>, grid, block, 0, s, B, n, means, scales, colors, opacities, d_means, d_scales,
                         d_colors, d_opacities, accumulate, sum_index);
    else
      hipLaunchKernelGGL(k_reduce_sums<48>, grid, block, 0, s, B, n, means, scales, colors, opacities, d_means, d_scales,
                         d_colors, d_opacities, accumulate, sum_index);
  } else if (gather_only) {  // no pair: every sum is zero
    GR_HIP_TRY(hipMemsetAsync(g_sums, 0, gr_view_sums_floats(n) * sizeof(float), s));
    if (g_sums3) GR_HIP_TRY(hipMemsetAsync(g_sums3, 0, (size_t)n * sizeof(float), s));
  } else {
    // the backward without a depth gradient writes 8-float rows (bwd_item_bf16).  No pair: every sum is zero, so
    // the one-pass kernel's rows are the parameters' own (the gradients are zero or the accumulator unchanged in any
    // order: sum_index needs no mapping here)
    const bool row8 = !depth;
    auto launch = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3((n + RG - 1) / RG), dim3(4 * RG), 0, s, vk, n, means, scales, colors, opacities,
                         (const Cnt2*)g.counts, (const Cnt2*)g.offsets, (const int*)b.pos_of, (const float*)partials,
                         d_means, d_scales, d_colors, d_opacities, depth ? 1 : 0, accumulate);
    };
    if (color_dim == 3)
      row8 ? launch(k_reduce_bwd<3, true>) : launch(k_reduce_bwd<3, false>);
    else if (color_dim == 12)
      row8 ? launch(k_reduce_bwd<12, true>) : launch(k_reduce_bwd<12, false>);
    else
      row8 ? launch(k_reduce_bwd<48, true>) : launch(k_reduce_bwd<48, false>);
  }
  GR_HIP_TRY(hipGetLastError());
  prof_mark(PROF_REDUCE, s);
  return GR_OK;
}

extern "C" {

gr_status gr_bwd(const gr_view* v, int n, const gr_plan* plan, const float* means, const float* scales,
                 const float* colors, int color_dim, const float* opacities, const void* geom, const void* bins,
                 const float* saved, const float* g_rgb, const float* g_alpha, const float* g_depth, float* d_means,
                 float* d_scales, float* d_colors, float* d_opacities, void* ws, size_t ws_bytes, void* stream) {
  return bwd_impl(v, n, plan, means, scales, colors, color_dim, opacities, geom, bins, saved, g_rgb, g_alpha, g_depth,
                  nullptr, nullptr, 0.0f, 0.0f, nullptr, d_means, d_scales, d_colors, d_opacities, 0, ws, ws_bytes, stream);
}

gr_status gr_bwd_indexed(const gr_view* v, int n, const gr_plan* plan, const float* means, const float* scales,
                         const float* colors, int color_dim, const float* opacities, const void* geom, const void* bins,
                         const float* saved, const float* g_rgb, const float* g_alpha, const float* g_depth,
                         const int* index, float* d_means, float* d_scales, float* d_colors, float* d_opacities, void* ws,
                         size_t ws_bytes, void* stream) {
  return bwd_impl(v, n, plan, means, scales, colors, color_dim, opacities, geom, bins, saved, g_rgb, g_alpha, g_depth,
                  nullptr, nullptr, 0.0f, 0.0f, nullptr, d_means, d_scales, d_colors, d_opacities, 0, ws, ws_bytes, stream,
                  nullptr, 0.0f, index);
}

gr_status gr_bwd_fit(const gr_view* v, int n, const gr_plan* plan, const float* means, const float* scales,
                     const float* colors, int color_dim, const float* opacities, const void* geom, const void* bins,
                     const float* saved, const float* target_rgb, const float* target_mask, float w_sil,
                     const float* target_depth, float w_depth, float g_scale, float* loss_out, float* d_means,
                     float* d_scales, float* d_colors, float* d_opacities, int accumulate, void* ws, size_t ws_bytes,
                     void* stream) {
  if (!target_rgb) return set_error(GR_ERR_INVALID_ARGUMENT, "gr_bwd_fit: target_rgb is null");
  return bwd_impl(v, n, plan, means, scales, colors, color_dim, opacities, geom, bins, saved, nullptr, nullptr, nullptr,
                  target_rgb, target_mask, w_sil, g_scale, loss_out, d_means, d_scales, d_colors, d_opacities,
                  accumulate, ws, ws_bytes, stream, target_depth, w_depth);
}

gr_status gr_bwd_fit_gather(const gr_view* v, int n, const gr_plan* plan, const void* geom, const void* bins,
                            const float* saved, const float* target_rgb, const float* target_mask, float w_sil,
                            const float* target_depth, float w_depth, float g_scale, float* loss_out, void* ws,
                            size_t ws_bytes, float* sums, float* sums3, void* stream) {
  if (!target_rgb) return set_error(GR_ERR_INVALID_ARGUMENT, "gr_bwd_fit_gather: target_rgb is null");
  if (!sums) return set_error(GR_ERR_INVALID_ARGUMENT, "gr_bwd_fit_gather: sums is null");
  return bwd_impl(v, n, plan, nullptr, nullptr, nullptr, 3, nullptr, geom, bins, saved, nullptr, nullptr, nullptr,
                  target_rgb, target_mask, w_sil, g_scale, loss_out, nullptr, nullptr, nullptr, nullptr, 0, ws, ws_bytes,
                  stream, target_depth, w_depth, nullptr, sums, sums3);
}

gr_status gr_bwd_l1(const gr_view* v, int n, const gr_plan* plan, const float* means, const float* scales,
                    const float* colors, int color_dim, const float* opacities, const void* geom, const void* bins,
                    const float* saved, const float* target_rgb, const float* target_mask, float w_sil, float g_scale,
                    float* loss_out, float* d_means, float* d_scales, float* d_colors, float* d_opacities,
                    int accumulate, void* ws, size_t ws_bytes, void* stream) {
  if (!target_rgb) return set_error(GR_ERR_INVALID_ARGUMENT, "gr_bwd_l1: target_rgb is null");
  return bwd_impl(v, n, plan, means, scales, colors, color_dim, opacities, geom, bins, saved, nullptr, nullptr, nullptr,
                  target_rgb, target_mask, w_sil, g_scale, loss_out, d_means, d_scales, d_colors, d_opacities,
                  accumulate, ws, ws_bytes, stream);
}

}  // extern "C" (the batching helpers are templates)

// ---- gr_fit_views_batched: the fused fit path's per-view chain for several views, one launch per kernel -----------
template <class A>
static void vb_add(VBatch<A>& B, const A& a, int blocks, int gx = 0) {
  B.a[B.nv] = a;
  B.gx[B.nv] = gx > 0 ? gx : (blocks > 0 ? blocks : 1);
  B.first[B.nv + 1] = B.first[B.nv] + (blocks > 0 ? blocks : 0);
  ++B.nv;
}
template <class A>
static VBatch<A> vb_new() {
  static_assert(sizeof(VBatch<A>) <= 4096, "batched kernel arguments exceed 4 KiB");
  VBatch<A> B;
  B.nv = 0;
  B.first[0] = 0;
  return B;
}
#define GR_VB_LAUNCH(kern, B, threads, lds, s)                                                   \
  do {                                                                                           \
    if ((B).first[(B).nv] > 0) {                                                                 \
      hipLaunchKernelGGL(kern, dim3((unsigned)(B).first[(B).nv]), dim3(threads), lds, s, (B));   \
      GR_HIP_TRY(hipGetLastError());                                                             \
    }                                                                                            \
  } while (0)

extern "C" {

gr_status gr_fit_views_batched(int num_views, const gr_batch_view* bv, int n, float w_sil, float w_depth,
                                          float g_scale, void* stream) {
  if (num_views < 1 || num_views > GR_BATCH_MAX_VIEWS || !bv)
    return set_error(GR_ERR_INVALID_ARGUMENT, "gr_fit_views_batched: num_views must be in [1, GR_BATCH_MAX_VIEWS]");
  if (n <= 0) return set_error(GR_ERR_INVALID_ARGUMENT, "gr_fit_views_batched: n must be > 0");
  static_assert(GR_BATCH_MAX_VIEWS == GR_BATCH_MAX, "gr_hip.h GR_BATCH_MAX_VIEWS");
  const gr_view& v0 = bv[0].view;
  const bool depth = bv[0].target_depth != nullptr;
  for (int j = 0; j < num_views; ++j) {
    const gr_batch_view& b = bv[j];
    gr_status st = check_view(&b.view);
    if (st != GR_OK) return st;
    if (b.view.width != v0.width || b.view.height != v0.height || tile_of(&b.view) != tile_of(&v0) ||
        b.view.no_depth_grad != v0.no_depth_grad || b.view.cutoff != v0.cutoff || b.view.core_cutoff != v0.core_cutoff ||
        b.view.device_counts != v0.device_counts || (b.target_depth != nullptr) != depth)
      return set_error(GR_ERR_INVALID_ARGUMENT, "gr_fit_views_batched: the views differ in size, tile, footprint or mode");
    if (b.plan.num_pairs <= 0 || b.plan.num_slots < b.plan.num_pairs)
      return set_error(GR_ERR_INVALID_ARGUMENT, "gr_fit_views_batched: every view needs pairs (or capacities)");
    if (!b.geom || !b.bins || !b.scratch || !b.ws || !b.target_rgb || !b.sums || !b.loss || (depth && (!b.saved || !b.sums3)))
      return set_error(GR_ERR_INVALID_ARGUMENT, "gr_fit_views_batched: null pointer");
    if (b.bins_bytes < gr_bins_bytes(&b.view, n, &b.plan) || b.scratch_bytes < gr_fwd_scratch_bytes(&b.view, n, &b.plan) ||
        b.ws_bytes < gr_bwd_bytes(&b.view, n, &b.plan))
      return set_error(GR_ERR_WORKSPACE, "gr_fit_views_batched: a workspace is too small");
  }
  if (!short_keys(vtiles_of(&v0)))
    return set_error(GR_ERR_INVALID_ARGUMENT, "gr_fit_views_batched: more than 8,192 screen tiles");
  if (depth ? v0.no_depth_grad != 0 : v0.no_depth_grad != 1)
    return set_error(GR_ERR_INVALID_ARGUMENT, "gr_fit_views_batched: depth loss needs no_depth_grad = 0, the L1 path 1");
  if (depth && tile_of(&v0) != T)
    return set_error(GR_ERR_INVALID_ARGUMENT, "gr_fit_views_batched: the depth-loss path runs at 16-pixel tiles");
  for (int j = 0; j < num_views && depth; ++j)
    if (bv[j].view.rows > 0)
      return set_error(GR_ERR_INVALID_ARGUMENT, "gr_fit_views_batched: a band of tile rows needs the L1 path (no depth loss)");
  hipStream_t s = (hipStream_t)stream;
  const int tiles = vtiles_of(&v0) / 2;
  const size_t HW = (size_t)v0.width * v0.height;
  const int waves = tsort_waves(tiles), bits = bits_for((uint32_t)tiles);
  auto Be = vb_new<k_emit_offsets_args>();
  auto Bc = vb_new<k_tile_count_args>();
  auto Bs = vb_new<k_tile_colscan_args>();
  auto Bp = vb_new<k_tile_place_args>();
  for (int j = 0; j < num_views; ++j) {  // the binning (bin_impl's counting-sort path, per view)
    const gr_batch_view& b = bv[j];
    const ViewK vk = make_viewk(&b.view);
    const TileCfg tc = tile_cfg(&b.view, b.plan.num_pairs);
    const Bins bn = bins_view(b.bins, 2 * tiles, b.plan.num_pairs, tc.ch);
    const Scratch sc = scratch_view(b.scratch, 2 * tiles, b.plan.num_pairs, tc.ch, tc.part_floats);
    Geom g = geom_view((void*)b.geom, n);
    const int64_t K = b.plan.num_pairs, Kc = b.plan.num_core_pairs, Kr[2] = {Kc, K - Kc};
    TZones Z;
    Z.cw = col_width(K, tiles);
    Z.ch = tc.ch;
    Z.kdev = b.view.device_counts ? (const unsigned long long*)(g.offsets + n) : nullptr;
    const size_t cells = (size_t)tiles * cols_of(K, Z.cw);
    char* q = (char*)sc.sort_tmp;
    for (int z = 0; z < 2; ++z) {
      TZone& zz = Z.z[z];
      zz.K = Kr[z];
      zz.cols = cols_of(Kr[z], Z.cw);
      zz.zbase = z == 0 ? 0 : (int)Kc;
      zz.keys = (const uint16_t*)sc.keys_in + (z == 0 ? 0 : Kc);
      zz.ids = sc.ids_in + (z == 0 ? 0 : Kc);
      zz.M = (int*)q;
      q += align_up(cells * sizeof(int));
      zz.S = (int*)q;
      q += align_up(cells * sizeof(int));
      zz.T = (int*)q;
      q += align_up((size_t)tiles * sizeof(int));
    }
    const int cols = Z.z[0].cols + Z.z[1].cols;
    vb_add(Be, k_emit_offsets_args{vk, n, (const int4*)g.rect, (const Cnt2*)g.counts, (const unsigned long long*)g.total,
                                   (Cnt2*)g.offsets, (const float4*)g.rec, (uint16_t*)sc.keys_in, sc.ids_in,
                                   bn.ticket + fan_offset(tiles)},
           blocks_for(n));
    vb_add(Bc, k_tile_count_args{Z, tiles}, cols);
    const int gxs = (tiles + CS_T - 1) / CS_T;
    vb_add(Bs, k_tile_colscan_args{Z, tiles, bn.ranges, bn.items, bn.num_items, bn.tile_item0, bn.ticket}, 2 * gxs, gxs);
    vb_add(Bp, k_tile_place_args{Z, tiles, bits, (const int2*)bn.ranges, bn.pairs, bn.pos_of}, cols);
  }
  GR_VB_LAUNCH(k_emit_offsets_views, Be, 256, 0, s);
  GR_VB_LAUNCH(k_tile_count_views, Bc, 256, (size_t)tiles * sizeof(int), s);
  GR_VB_LAUNCH(k_tile_colscan_views, Bs, CS_T * CS_G, 0, s);
  const size_t lds = (size_t)tiles * sizeof(int) * waves;
  if (waves == 8) GR_VB_LAUNCH(k_tile_place_views<8>, Bp, 512, lds, s);
  else if (waves == 4) GR_VB_LAUNCH(k_tile_place_views<4>, Bp, 256, lds, s);
  else if (waves == 2) GR_VB_LAUNCH(k_tile_place_views<2>, Bp, 128, lds, s);
  else GR_VB_LAUNCH(k_tile_place_views<1>, Bp, 64, lds, s);

  auto Bg = vb_new<k_gather_view_args>();
  if (!depth) {  // the fused fit path: forward with the L1 epilogue, backward splat, gather
    auto Bf = vb_new<k_fwd32_l1_args>();
    auto Bf16 = vb_new<k_raster_fwd_mfma_args>();
    auto Bb = vb_new<k_bwd32_args>();
    auto Bb16 = vb_new<k_raster_bwd_bf16_args>();
    for (int j = 0; j < num_views; ++j) {
      const gr_batch_view& b = bv[j];
      const ViewK vk = make_viewk(&b.view);
      const TileCfg tc = tile_cfg(&b.view, b.plan.num_pairs);
      const Bins bn = bins_view(b.bins, 2 * tiles, b.plan.num_pairs, tc.ch);
      const Scratch sc = scratch_view(b.scratch, 2 * tiles, b.plan.num_pairs, tc.ch, tc.part_floats);
      const Geom g = geom_view((void*)b.geom, n);
      const BwdWs w = bwd_ws(&b.view, n, &b.plan, b.ws);
      L1Args la{b.target_rgb, b.target_mask, w_sil, g_scale, w.tile_loss};
      la.pieces = 2;
      la.loss_out = b.loss;
      la.n1 = (int64_t)(3 * HW);
      la.n2 = (int64_t)(b.target_mask ? HW : 0);
      const int cap = (int)item_cap(2 * tiles, b.plan.num_pairs, tc.ch);
      if (tc.T == T32) {
        vb_add(Bf, k_fwd32_l1_args{vk, n, (const int4*)bn.items, (const int*)bn.num_items, (const int2*)bn.ranges,
                                   (const int*)bn.pairs, (const float4*)g.rec, sc.fwd_part, nullptr, nullptr, la, w.UF,
                                   (const int*)g.f16_sa, (const int*)bn.tile_item0, bn.ticket, tc.ch},
               cap);
        vb_add(Bb, k_bwd32_args{vk, n, (const int4*)bn.items, (const int*)bn.num_items, (const int*)bn.pairs,
                                (const float4*)g.rec, (const uint4*)w.UF, w.partials},
               cap);
      } else {
        vb_add(Bf16, k_raster_fwd_mfma_args{vk, n, (const int4*)bn.items, (const int*)bn.num_items, (const int2*)bn.ranges,
                                            (const int*)bn.pairs, (const float4*)g.rec, sc.fwd_part, nullptr, nullptr,
                                            nullptr, nullptr, nullptr, la, w.UF, (const int*)g.f16_sa,
                                            (const int*)bn.tile_item0, bn.ticket, tc.ch},
               cap);
        vb_add(Bb16, k_raster_bwd_bf16_args{vk, n, (const int4*)bn.items, (const int*)bn.num_items, (const int*)bn.pairs,
                                            (const float4*)g.rec, (const uint4*)w.UF, w.partials, nullptr},
               cap);
      }
      vb_add(Bg, k_gather_view_args{n, (const Cnt2*)g.offsets, (const int*)bn.pos_of, (const float4*)w.partials,
                                    (float2*)b.sums, nullptr, nullptr},
             (n + 63) / 64);
    }
    GR_VB_LAUNCH(k_fwd32_l1_views, Bf, 256, 0, s);
    GR_VB_LAUNCH(k_raster_fwd_mfma_views<4>, Bf16, 256, 0, s);
    GR_VB_LAUNCH(k_bwd32_views, Bb, 256, 0, s);
    GR_VB_LAUNCH((k_raster_bwd_bf16_views<false, 2>), Bb16, 256, 0, s);
    GR_VB_LAUNCH(k_gather_view_views<false>, Bg, 256, 0, s);
    return GR_OK;
  }
  // the depth-loss path (gr_fwd_render + gr_bwd_fit_gather per view): forward into saved sums, the depth loss's max
  // and sums, the upstream fragments and view loss, the three-piece backward with the tail pairs, the gather
  auto Bf = vb_new<k_raster_fwd_mfma_args>();
  auto Bm = vb_new<k_depth_tile_max_args>();
  auto Bd = vb_new<k_depth_tile_sums_args>();
  auto Bu = vb_new<k_pixel_grads_args>();
  auto Bb = vb_new<k_raster_bwd_bf16_args>();
  for (int j = 0; j < num_views; ++j) {
    const gr_batch_view& b = bv[j];
    const ViewK vk = make_viewk(&b.view);
    const TileCfg tc = tile_cfg(&b.view, b.plan.num_pairs);
    const Bins bn = bins_view(b.bins, 2 * tiles, b.plan.num_pairs, tc.ch);
    const Scratch sc = scratch_view(b.scratch, 2 * tiles, b.plan.num_pairs, tc.ch, tc.part_floats);
    const Geom g = geom_view((void*)b.geom, n);
    const BwdWs w = bwd_ws(&b.view, n, &b.plan, b.ws);
    float4* s4 = (float4*)b.saved;
    float* sD = b.saved + 4 * HW;
    const int cap = (int)item_cap(2 * tiles, b.plan.num_pairs, tc.ch);
    L1Args none{nullptr, nullptr, 0.f, 0.f, nullptr};
    vb_add(Bf, k_raster_fwd_mfma_args{vk, n, (const int4*)bn.items, (const int*)bn.num_items, (const int2*)bn.ranges,
                                      (const int*)bn.pairs, (const float4*)g.rec, sc.fwd_part, nullptr, nullptr, nullptr,
                                      s4, sD, none, nullptr, (const int*)g.f16_sa, (const int*)bn.tile_item0, bn.ticket,
                                      tc.ch},
           cap);
    vb_add(Bm, k_depth_tile_max_args{vk, s4, sD, w.tile_aux, w.dscal, bn.ticket}, tiles);
    vb_add(Bd, k_depth_tile_sums_args{vk, s4, sD, b.target_depth, w.dscal, w.tile_loss, w.tile_aux, (int64_t)HW, w_depth,
                                      g_scale, bn.ticket},
           tiles);
    L1Args l1{b.target_rgb, b.target_mask, w_sil, g_scale, w.tile_loss};
    l1.loss_out = b.loss;
    l1.n1 = (int64_t)(3 * HW);
    l1.n2 = (int64_t)(b.target_mask ? HW : 0);
    l1.t_depth = b.target_depth;
    l1.w_depth = w_depth;
    l1.dscal = w.dscal;
    vb_add(Bu, k_pixel_grads_args{vk, s4, sD, nullptr, nullptr, nullptr, w.UF, 3, l1, true, bn.ticket}, tiles);
    vb_add(Bb, k_raster_bwd_bf16_args{vk, n, (const int4*)bn.items, (const int*)bn.num_items, (const int*)bn.pairs,
                                      (const float4*)g.rec, (const uint4*)w.UF, w.partials,
                                      w.partials + 8 * (size_t)b.plan.num_slots},
           cap);
    vb_add(Bg, k_gather_view_args{n, (const Cnt2*)g.offsets, (const int*)bn.pos_of, (const float4*)w.partials,
                                  (float2*)b.sums, (const float*)(w.partials + 8 * (size_t)b.plan.num_slots), b.sums3},
           (n + 63) / 64);
  }
  GR_VB_LAUNCH(k_raster_fwd_mfma_views<1>, Bf, 256, 0, s);
  GR_VB_LAUNCH(k_depth_tile_max_views, Bm, 256, 0, s);
  GR_VB_LAUNCH(k_depth_tile_sums_views, Bd, 256, 0, s);
  GR_VB_LAUNCH(k_pixel_grads_views, Bu, 256, 0, s);
  GR_VB_LAUNCH((k_raster_bwd_bf16_views<true, 3>), Bb, 256, 0, s);
  GR_VB_LAUNCH(k_gather_view_views<true>, Bg, 256, 0, s);
  return GR_OK;
}

gr_status gr_bwd_splat(const gr_view* v, int n, const gr_plan* plan, const void* geom, const void* bins, void* ws,
                       size_t ws_bytes, void* stream) {
  gr_status st = check_view(v);
  if (st != GR_OK) return st;
  if (!v->no_depth_grad)
    return set_error(GR_ERR_INVALID_ARGUMENT, "gr_bwd_splat: the view must have no_depth_grad = 1 or 2");
  if (!plan) return set_error(GR_ERR_INVALID_ARGUMENT, "plan is null");
  if (plan->num_pairs < 0) return set_error(GR_ERR_OVERFLOW, "pair count overflows int32");
  if (n <= 0 || plan->num_pairs == 0) return GR_OK;
  if (!geom || !bins) return set_error(GR_ERR_INVALID_ARGUMENT, "null pointer");
  if (!ws || ws_bytes < gr_bwd_bytes(v, n, plan)) return set_error(GR_ERR_WORKSPACE, "backward workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const ViewK vk = make_viewk(v);
  const int tiles = vk.tiles_x * vk.tiles_y;
  const Geom g = geom_view((void*)geom, n);
  const TileCfg tc = tile_cfg(v, plan->num_pairs);
  if (tc.T == T32 && v->no_depth_grad != 1)
    return set_error(GR_ERR_INVALID_ARGUMENT, "32-pixel tiles (gr_view.tile = 32): no_depth_grad = 1 only");
  const Bins b = bins_view((void*)bins, 2 * tiles, plan->num_pairs, tc.ch);
  const BwdWs w = bwd_ws(v, n, plan, ws);
  const int64_t cap = item_cap(2 * tiles, plan->num_pairs, tc.ch);
  if (GR_DEBUG_SKIP & 2) return GR_OK;
  prof_mark(PROF_RASTER_BWD, s);
  if (tc.T == T32)
    hipLaunchKernelGGL(k_bwd32, dim3((unsigned)cap), dim3(256), 0, s, vk, n, (const int4*)b.items,
                       (const int*)b.num_items, (const int*)b.pairs, (const float4*)g.rec, (const uint4*)w.UF, w.partials);
  else
  hipLaunchKernelGGL((v->no_depth_grad == 1 ? k_raster_bwd_bf16<false, 2> : k_raster_bwd_bf16<false, 3>), dim3((unsigned)cap),
                     dim3(256), 0, s, vk, n, (const int4*)b.items, (const int*)b.num_items, (const int*)b.pairs,
                     (const float4*)g.rec, (const uint4*)w.UF, w.partials, (float*)nullptr);
  GR_HIP_TRY(hipGetLastError());
  prof_mark(PROF_RASTER_BWD, s);
  return GR_OK;
}

gr_status gr_reduce_views(int num_views, const gr_reduce_view* views, int n, const float* means, const float* scales,
                          const float* colors, int color_dim, const float* opacities, float* d_means, float* d_scales,
                          float* d_colors, float* d_opacities, int accumulate, void* stream) {
  if (num_views < 0 || num_views > GR_REDUCE_MAX_VIEWS)
    return set_error(GR_ERR_INVALID_ARGUMENT, "gr_reduce_views: num_views must be in [0, GR_REDUCE_MAX_VIEWS]");
  if (color_dim != 3 && color_dim != 12 && color_dim != 48)
    return set_error(GR_ERR_INVALID_ARGUMENT, "colors must be (N,3) or SH coeffs (N,4,3) / (N,16,3)");
  if (n < 0) return set_error(GR_ERR_INVALID_ARGUMENT, "n must be >= 0");
  if (n == 0) return GR_OK;
  if (!means || !scales || !colors || !opacities || !d_means || !d_scales || !d_colors || !d_opacities ||
      (num_views > 0 && !views))
    return set_error(GR_ERR_INVALID_ARGUMENT, "null pointer");
  RBatch B;
  B.nv = num_views;
  for (int k = 0; k < num_views; ++k) {
    const gr_reduce_view& rv = views[k];
    gr_status st = check_view(&rv.view);
    if (st != GR_OK) return st;
    if (!rv.view.no_depth_grad)
      return set_error(GR_ERR_INVALID_ARGUMENT, "gr_reduce_views: views must be rendered with no_depth_grad = 1");
    if (rv.plan.num_pairs < 0) return set_error(GR_ERR_OVERFLOW, "pair count overflows int32");
    if (!rv.geom || (rv.plan.num_pairs > 0 && (!rv.bins || !rv.ws)))
      return set_error(GR_ERR_INVALID_ARGUMENT, "gr_reduce_views: null workspace");
    const ViewK vk = make_viewk(&rv.view);
    const Geom g = geom_view((void*)rv.geom, n);
    const Bins b = bins_view((void*)rv.bins, 2 * vk.tiles_x * vk.tiles_y, rv.plan.num_pairs, tile_cfg(&rv.view, rv.plan.num_pairs).ch);
    B.r[k].v = vk;
    B.r[k].offsets = (const Cnt2*)g.offsets;
    B.r[k].pos_of = rv.plan.num_pairs > 0 ? (const int*)b.pos_of : nullptr;
    B.r[k].rows = (const float4*)rv.ws;
  }
  hipStream_t s = (hipStream_t)stream;
  prof_mark(PROF_REDUCE, s);
  const dim3 grid((n + RG - 1) / RG), block(4 * RG);
  if (color_dim == 3)
    hipLaunchKernelGGL(k_reduce_views<3>, grid, block, 0, s, B, n, means, scales, colors, opacities, d_means, d_scales,
                       d_colors, d_opacities, accumulate);
  else if (color_dim == 12)
    hipLaunchKernelGGL(k_reduce_views<12>, grid, block, 0, s, B, n, means, scales, colors, opacities, d_means, d_scales,
                       d_colors, d_opacities, accumulate);
  else
    hipLaunchKernelGGL(k_reduce_views<48>, grid, block, 0, s, B, n, means, scales, colors, opacities, d_means, d_scales,
                       d_colors, d_opacities, accumulate);
  GR_HIP_TRY(hipGetLastError());
  prof_mark(PROF_REDUCE, s);
  return GR_OK;
}

size_t gr_view_sums_floats(int n) { return (size_t)8 * (size_t)(n > 0 ? n : 0); }

gr_status gr_gather_view(const gr_view* v, int n, const gr_plan* plan, const void* geom, const void* bins, const void* ws,
                         float* sums, void* stream) {
  gr_status st = check_view(v);
  if (st != GR_OK) return st;
  if (!v->no_depth_grad)
    return set_error(GR_ERR_INVALID_ARGUMENT, "gr_gather_view: the view must have no_depth_grad = 1 or 2");
  if (!plan) return set_error(GR_ERR_INVALID_ARGUMENT, "plan is null");
  if (plan->num_pairs < 0) return set_error(GR_ERR_OVERFLOW, "pair count overflows int32");
  if (n < 0) return set_error(GR_ERR_INVALID_ARGUMENT, "n must be >= 0");
  if (n == 0) return GR_OK;
  if (!geom || !sums || (plan->num_pairs > 0 && (!bins || !ws)))
    return set_error(GR_ERR_INVALID_ARGUMENT, "gr_gather_view: null pointer");
  hipStream_t s = (hipStream_t)stream;
  if (plan->num_pairs == 0) {  // no pair: every sum is zero
    GR_HIP_TRY(hipMemsetAsync(sums, 0, gr_view_sums_floats(n) * sizeof(float), s));
    return GR_OK;
  }
  const ViewK vk = make_viewk(v);
  const Geom g = geom_view((void*)geom, n);
  const Bins b = bins_view((void*)bins, 2 * vk.tiles_x * vk.tiles_y, plan->num_pairs, tile_cfg(v, plan->num_pairs).ch);
  if (GR_DEBUG_SKIP & 4) return GR_OK;
  prof_mark(PROF_REDUCE, s);
  hipLaunchKernelGGL(k_gather_view<false>, dim3((n + 63) / 64), dim3(256), 0, s, n, (const Cnt2*)g.offsets,
                     (const int*)b.pos_of, (const float4*)ws, (float2*)sums, (const float*)nullptr, (float*)nullptr);
  GR_HIP_TRY(hipGetLastError());
  prof_mark(PROF_REDUCE, s);
  return GR_OK;
}

gr_status gr_reduce_sums(int num_views, const gr_sums_view* views, int n, const float* means, const float* scales,
                         const float* colors, int color_dim, const float* opacities, float* d_means, float* d_scales,
                         float* d_colors, float* d_opacities, int accumulate, void* stream) {
  if (num_views < 0 || num_views > GR_REDUCE_MAX_VIEWS)
    return set_error(GR_ERR_INVALID_ARGUMENT, "gr_reduce_sums: num_views must be in [0, GR_REDUCE_MAX_VIEWS]");
  if (color_dim != 3 && color_dim != 12 && color_dim != 48)
    return set_error(GR_ERR_INVALID_ARGUMENT, "colors must be (N,3) or SH coeffs (N,4,3) / (N,16,3)");
  if (n < 0) return set_error(GR_ERR_INVALID_ARGUMENT, "n must be >= 0");
  if (n == 0) return GR_OK;
  if (!means || !scales || !colors || !opacities || !d_means || !d_scales || !d_colors || !d_opacities ||
      (num_views > 0 && !views))
    return set_error(GR_ERR_INVALID_ARGUMENT, "null pointer");
  SBatch B;
  B.nv = num_views;
  for (int k = 0; k < num_views; ++k) {
    gr_status st = check_view(&views[k].view);
    if (st != GR_OK) return st;
    if (!views[k].sums) return set_error(GR_ERR_INVALID_ARGUMENT, "gr_reduce_sums: null sums");
    B.r[k].v = make_viewk(&views[k].view);
    B.r[k].sums = (const float4*)views[k].sums;
    B.r[k].sums3 = views[k].sums3;
  }
  hipStream_t s = (hipStream_t)stream;
  if (GR_DEBUG_SKIP & 8) return GR_OK;
  prof_mark(PROF_REDUCE, s);
  const int gpb = 64 * (4 / reduce_sums_crw(num_views, color_dim));
  const dim3 grid((n + gpb - 1) / gpb), block(256);
  if (color_dim == 3)
    hipLaunchKernelGGL(k_reduce_sums<3>, grid, block, 0, s, B, n, means, scales, colors, opacities, d_means, d_scales,
                       d_colors, d_opacities, accumulate, (const int*)nullptr);
  else if (color_dim == 12)
    hipLaunchKernelGGL(k_reduce_sums<12>, grid, block, 0, s, B, n, means, scales, colors, opacities, d_means, d_scales,
                       d_colors, d_opacities, accumulate, (const int*)nullptr);
  else
    hipLaunchKernelGGL(k_reduce_sums<48>, grid, block, 0, s, B, n, means, scales, colors, opacities, d_means, d_scales,
                       d_colors, d_opacities, accumulate, (const int*)nullptr);
  GR_HIP_TRY(hipGetLastError());
  prof_mark(PROF_REDUCE, s);
  return GR_OK;
}

gr_status gr_bwd_camera(const gr_view* v, int n, const gr_plan* plan, const float* means, const float* scales,
                        const float* colors, int color_dim, const float* opacities, void* ws, size_t ws_bytes, int depth,
                        float* d_camera, void* stream) {
  gr_status st = check_view(v);
  if (st != GR_OK) return st;
  if (!plan || !d_camera) return set_error(GR_ERR_INVALID_ARGUMENT, "gr_bwd_camera: null plan or output");
  if (plan->num_pairs < 0) return set_error(GR_ERR_OVERFLOW, "pair count overflows int32");
  if (color_dim != 3 && color_dim != 12 && color_dim != 48)
    return set_error(GR_ERR_INVALID_ARGUMENT, "colors must be (N,3) or SH coeffs (N,4,3) / (N,16,3)");
  if (n < 0) return set_error(GR_ERR_INVALID_ARGUMENT, "n must be >= 0");
  if (depth && v->no_depth_grad)
    return set_error(GR_ERR_INVALID_ARGUMENT, "gr_bwd_camera: depth sums of a view rendered with no_depth_grad");
  hipStream_t s = (hipStream_t)stream;
  if (n == 0 || plan->num_pairs == 0) {  // no pair reached the backward: every term is zero
    GR_HIP_TRY(hipMemsetAsync(d_camera, 0, CAM_GRADS * sizeof(float), s));
    return GR_OK;
  }
  if (!means || !scales || !colors || !opacities || !ws) return set_error(GR_ERR_INVALID_ARGUMENT, "null pointer");
  if (ws_bytes < gr_bwd_bytes(v, n, plan)) return set_error(GR_ERR_WORKSPACE, "backward workspace too small");
  const ViewK vk = make_viewk(v);
  const BwdWs w = bwd_ws(v, n, plan, ws);
  const int blocks = blocks_for(n);
  const float4* sums = (const float4*)w.sums;
  const float* sums3 = depth ? (const float*)w.sums3 : nullptr;
  if (color_dim == 3)
    hipLaunchKernelGGL(k_camera_grad<3>, dim3(blocks), dim3(256), 0, s, vk, n, means, scales, colors, opacities, sums, sums3,
                       w.cam_part);
  else if (color_dim == 12)
    hipLaunchKernelGGL(k_camera_grad<12>, dim3(blocks), dim3(256), 0, s, vk, n, means, scales, colors, opacities, sums, sums3,
                       w.cam_part);
  else
    hipLaunchKernelGGL(k_camera_grad<48>, dim3(blocks), dim3(256), 0, s, vk, n, means, scales, colors, opacities, sums, sums3,
                       w.cam_part);
  GR_HIP_TRY(hipGetLastError());
  hipLaunchKernelGGL(k_camera_final, dim3(CAM_GRADS), dim3(64), 0, s, (const double*)w.cam_part, blocks, d_camera);
  GR_HIP_TRY(hipGetLastError());
  return GR_OK;
}

gr_status gr_render_u8(const gr_render_params* p, int n, const float* means, const float* scales, const float* colors,
                       const float* opacities, uint8_t* rgba) {
  if (!p || !rgba) return set_error(GR_ERR_INVALID_ARGUMENT, "null pointer");
  if (p->width <= 0 || p->height <= 0) return set_error(GR_ERR_INVALID_ARGUMENT, "width/height must be positive");
  const size_t HW = (size_t)p->width * p->height;
  if (n <= 0) {
    if (p->force_cpu) {
      // force_cpu selects the CPU renderer (renderer_dispatch.cpp:12-13), whose n <= 0 image is the finalized background
      // with A = 255 in both modes (renderer_cpu.cpp:219-257: zero sums); for n > 0 this path already has its semantics
      uint8_t px[4];
      for (int c = 0; c < 3; ++c) px[c] = (uint8_t)(std::min(std::max(p->background[c], 0.0f), 1.0f) * 255.0f + 0.5f);
      px[3] = 255;
      for (size_t i = 0; i < HW; ++i) std::memcpy(rgba + 4 * i, px, 4);
    } else {
      std::memset(rgba, 0, HW * 4);  // the CUDA renderer's (renderer.cu:279-281)
    }
    return GR_OK;
  }
  if (!means || !scales || !colors || !opacities) return set_error(GR_ERR_INVALID_ARGUMENT, "null pointer");
  gr_view gv{};  // background_dev NULL: the host background of the params
  gv.width = p->width;
  gv.height = p->height;
  std::memcpy(gv.view, p->view, sizeof(gv.view));
  std::memcpy(gv.proj, p->proj, sizeof(gv.proj));
  std::memcpy(gv.background, p->background, sizeof(gv.background));
  gv.cam_pos[0] = gv.cam_pos[1] = gv.cam_pos[2] = 0.f;
  gv.cutoff = 3.0f;
  const ViewK vk = make_viewk(&gv);
  const int tiles = vk.tiles_x * vk.tiles_y;
  const bool sorted = p->enable_depth_sort != 0;
  // One device allocation per call: reentrant (no function-static buffers as renderer.cu:349).
  const size_t nn = (size_t)n;
  size_t o = 0;
  const size_t o_in = o; o = align_up(o + nn * 10 * sizeof(float));
  const size_t o_a = o; o = align_up(o + nn * sizeof(float4));
  const size_t o_c = o; o = align_up(o + nn * sizeof(float4));
  const size_t o_box = o; o = align_up(o + nn * sizeof(int4));
  const size_t o_rect = o; o = align_up(o + nn * sizeof(int4));
  const size_t o_cnt = o; o = align_up(o + (nn + 1) * sizeof(int));
  const size_t o_off = o; o = align_up(o + (nn + 1) * sizeof(int));
  const size_t o_dk = o; o = align_up(o + nn * sizeof(uint32_t));
  const size_t o_img = o; o = align_up(o + HW * 4);
  const size_t o_scan = o; o = align_up(o + scan_tmp_bytes_t<int>(n));
  const size_t o_tot = o; o = align_up(o + sizeof(unsigned long long));
  const size_t fixed = o;
  char* d = nullptr;
  GR_HIP_TRY(hipMalloc(&d, fixed));
  struct Guard {
    void* p;
    ~Guard() { if (p) (void)hipFree(p); }
  } guard{d};
  hipStream_t s = nullptr;
  float* din = (float*)(d + o_in);
  GR_HIP_TRY(hipMemcpy(din, means, nn * 3 * sizeof(float), hipMemcpyHostToDevice));
  GR_HIP_TRY(hipMemcpy(din + 3 * nn, scales, nn * 3 * sizeof(float), hipMemcpyHostToDevice));
  GR_HIP_TRY(hipMemcpy(din + 6 * nn, colors, nn * 3 * sizeof(float), hipMemcpyHostToDevice));
  GR_HIP_TRY(hipMemcpy(din + 9 * nn, opacities, nn * sizeof(float), hipMemcpyHostToDevice));
  LegacyRec lr;
  lr.a = (float4*)(d + o_a);
  lr.c = (float4*)(d + o_c);
  lr.box = (int4*)(d + o_box);
  lr.rect = (int4*)(d + o_rect);
  lr.counts = (int*)(d + o_cnt);
  lr.offsets = (int*)(d + o_off);
  lr.depth_key = (uint32_t*)(d + o_dk);
  hipLaunchKernelGGL(k_preprocess_u8, dim3(blocks_for(n + 1)), dim3(256), 0, s, vk, n, din, din + 3 * nn, din + 6 * nn,
                     din + 9 * nn, lr);
  GR_HIP_TRY(hipGetLastError());
  unsigned long long* tot = (unsigned long long*)(d + o_tot);
  GR_HIP_TRY(hipMemsetAsync(tot, 0, sizeof(*tot), s));
  hipLaunchKernelGGL(k_count_total64, dim3(std::min(blocks_for(n), 1024)), dim3(256), 0, s, n, lr.counts, tot);
  GR_HIP_TRY(hipGetLastError());
  size_t tmp = scan_tmp_bytes_t<int>(n);
  GR_HIP_TRY(hipcub::DeviceScan::ExclusiveSum(d + o_scan, tmp, lr.counts, lr.offsets, n + 1, s));
  unsigned long long K64 = 0;
  GR_HIP_TRY(hipMemcpy(&K64, tot, sizeof(K64), hipMemcpyDeviceToHost));
  if (K64 >= (1ull << 31)) return set_error(GR_ERR_OVERFLOW, "pair count overflows int32");
  const int K = (int)K64;
  // bins: keys_in/out (u32 or u64), ids_in/out, ranges, sort tmp
  const size_t kk = (size_t)(K > 0 ? K : 1);
  const size_t ksz = sorted ? sizeof(uint64_t) : sizeof(uint32_t);
  const int bits = sorted ? 32 + bits_for((uint32_t)tiles) : bits_for((uint32_t)tiles);
  const size_t stmp = sorted ? sort_tmp_bytes<uint64_t>(K, bits) : sort_tmp_bytes<uint32_t>(K, bits);
  size_t q = 0;
  const size_t q_kin = q; q = align_up(q + kk * ksz);
  const size_t q_kout = q; q = align_up(q + kk * ksz);
  const size_t q_iin = q; q = align_up(q + kk * sizeof(int));
  const size_t q_iout = q; q = align_up(q + kk * sizeof(int));
  const size_t q_rg = q; q = align_up(q + (size_t)tiles * sizeof(int2));
  const size_t q_tmp = q; q = align_up(q + stmp);
  char* e = nullptr;
  GR_HIP_TRY(hipMalloc(&e, q));
  Guard guard2{e};
  int2* ranges = (int2*)(e + q_rg);
  GR_HIP_TRY(hipMemsetAsync(ranges, 0, sizeof(int2) * tiles, s));
  if (K > 0) {
    size_t t2 = stmp;
    if (sorted) {
      uint64_t* kin = (uint64_t*)(e + q_kin);
      uint64_t* kout = (uint64_t*)(e + q_kout);
      // low 32 bits = depth key; high bits = tile
      hipLaunchKernelGGL((k_emit<uint64_t, int>), dim3(blocks_for(n)), dim3(256), 0, s, vk, n, (const int4*)lr.rect,
                         (const int*)lr.counts, (const int*)lr.offsets, (const uint64_t*)nullptr,
                         kin, (int*)(e + q_iin));
      GR_HIP_TRY(hipGetLastError());
      hipLaunchKernelGGL(k_patch_depth, dim3(blocks_for(K)), dim3(256), 0, s, (int64_t)K, kin, (const int*)(e + q_iin),
                         (const uint32_t*)lr.depth_key);
      GR_HIP_TRY(hipGetLastError());
      GR_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(e + q_tmp, t2, kin, kout, (int*)(e + q_iin), (int*)(e + q_iout), K, 0,
                                                    bits, s));
      hipLaunchKernelGGL(k_ranges<uint64_t>, dim3(blocks_for(K)), dim3(256), 0, s, (int64_t)K, (const uint64_t*)kout, ranges);
    } else {
      uint32_t* kin = (uint32_t*)(e + q_kin);
      uint32_t* kout = (uint32_t*)(e + q_kout);
      hipLaunchKernelGGL((k_emit<uint32_t, int>), dim3(blocks_for(n)), dim3(256), 0, s, vk, n, (const int4*)lr.rect,
                         (const int*)lr.counts, (const int*)lr.offsets, (const uint32_t*)nullptr,
                         kin, (int*)(e + q_iin));
      GR_HIP_TRY(hipGetLastError());
      GR_HIP_TRY(hipcub::DeviceRadixSort::SortPairs(e + q_tmp, t2, kin, kout, (int*)(e + q_iin), (int*)(e + q_iout), K, 0,
                                                    bits, s));
      hipLaunchKernelGGL(k_ranges<uint32_t>, dim3(blocks_for(K)), dim3(256), 0, s, (int64_t)K, (const uint32_t*)kout, ranges);
    }
    GR_HIP_TRY(hipGetLastError());
  }
  uint8_t* img = (uint8_t*)(d + o_img);
  if (sorted)
    hipLaunchKernelGGL(k_raster_u8<true>, dim3(tiles), dim3(256), 0, s, vk, ranges, (const int*)(e + q_iout), lr.a, lr.c,
                       lr.box, img);
  else
    hipLaunchKernelGGL(k_raster_u8<false>, dim3(tiles), dim3(256), 0, s, vk, ranges, (const int*)(e + q_iout), lr.a, lr.c,
                       lr.box, img);
  GR_HIP_TRY(hipGetLastError());
  GR_HIP_TRY(hipMemcpy(rgba, img, HW * 4, hipMemcpyDeviceToHost));
  return GR_OK;
}

size_t gr_l1_loss_ws_bytes(void) { return (size_t)2 * LOSS_BLOCKS * sizeof(float); }

gr_status gr_l1_loss_fwd(const float* a, const float* b, int64_t n1, const float* c, const float* d, int64_t n2, float w2,
                         float* loss, void* ws, size_t ws_bytes, void* stream) {
  if (n1 <= 0 || n2 < 0 || !a || !b || !loss || (n2 > 0 && (!c || !d)))
    return set_error(GR_ERR_INVALID_ARGUMENT, "gr_l1_loss_fwd: bad arguments");
  if (!ws || ws_bytes < gr_l1_loss_ws_bytes()) return set_error(GR_ERR_WORKSPACE, "gr_l1_loss_fwd: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_l1_partial, dim3(LOSS_BLOCKS, 2), dim3(256), 0, s, a, b, n1, c, d, n2, (float*)ws);
  GR_HIP_TRY(hipGetLastError());
  hipLaunchKernelGGL(k_l1_final, dim3(1), dim3(256), 0, s, (const float*)ws, n1, n2, w2, loss);
  GR_HIP_TRY(hipGetLastError());
  return GR_OK;
}

gr_status gr_fit_param_step(int64_t count, int act, float* param, float* grad, const float* const* accs, int num_accs,
                            float reg, int adam, float* exp_avg, float* exp_avg_sq, float neg_step_size,
                            float bias_correction2_sqrt, double beta1, double beta2, float eps, void* stream) {
  if (count < 0 || act < 0 || act > 2 || !param || (adam && (!exp_avg || !exp_avg_sq)) || (!adam && !grad) ||
      num_accs < 0 || num_accs > GR_FIT_MAX_ACC || (num_accs > 0 && !accs))
    return set_error(GR_ERR_INVALID_ARGUMENT, "gr_fit_param_step: bad arguments");
  if (count == 0) return GR_OK;
  AccList acc;
  acc.n = num_accs;
  for (int a = 0; a < num_accs; ++a) {
    if (!accs[a]) return set_error(GR_ERR_INVALID_ARGUMENT, "gr_fit_param_step: null accumulator");
    acc.p[a] = accs[a];
  }
  const int blocks = (int)std::min<int64_t>((count + 255) / 256, 4096);
  // torch.optim.Adam passes 1 - beta1 (lerp weight) and 1 - beta2 (addcmul value) as Python floats (double)
  const float w1 = (float)(1.0 - beta1), w2 = (float)(1.0 - beta2);
  if (GR_DEBUG_SKIP & 16) return GR_OK;
  hipLaunchKernelGGL(k_fit_param_step, dim3(blocks), dim3(256), 0, (hipStream_t)stream, count, act, param, grad, acc, reg, adam, exp_avg, exp_avg_sq, neg_step_size, bias_correction2_sqrt, w1, (float)beta2, w2, eps);
  GR_HIP_TRY(hipGetLastError());
  return GR_OK;
}

static gr_status param_steps_impl(int num, const gr_param_step* steps, double beta1, double beta2, float eps,
                                  const float* sched, int* step_dev, int* overflow, int* host_flags, void* stream) {
  if (num < 0 || num > GR_FIT_MAX_PARAMS || (num > 0 && !steps))
    return set_error(GR_ERR_INVALID_ARGUMENT, "gr_fit_param_steps: bad arguments");
  ParamSteps P;
  P.num = 0;
  P.first[0] = 0;
  for (int t = 0; t < num; ++t) {
    const gr_param_step& q = steps[t];
    if (q.count < 0 || q.act < 0 || q.act > 2 || !q.param || !q.exp_avg || !q.exp_avg_sq || q.num_accs < 0 ||
        q.num_accs > GR_FIT_MAX_ACC)
      return set_error(GR_ERR_INVALID_ARGUMENT, "gr_fit_param_steps: bad parameter entry");
    for (int a = 0; a < q.num_accs; ++a)
      if (!q.accs[a]) return set_error(GR_ERR_INVALID_ARGUMENT, "gr_fit_param_steps: null accumulator");
    if (q.count == 0) continue;
    auto al = [](const void* a) { return a == nullptr || ((uintptr_t)a & 15u) == 0; };
    bool v4 = q.count % 4 == 0 && al(q.param) && al(q.grad) && al(q.exp_avg) && al(q.exp_avg_sq);
    for (int a = 0; a < q.num_accs; ++a) v4 = v4 && al(q.accs[a]);
    P.s[P.num] = q;
    P.vec4[P.num] = v4 ? 1 : 0;
    // one element (or float4) per thread up to 16384 blocks per tensor: the loads of one pass are all in flight
    P.first[P.num + 1] = P.first[P.num] + (int)std::min<int64_t>(((v4 ? q.count / 4 : q.count) + 255) / 256, 16384);
    ++P.num;
  }
  if (P.num == 0 && !sched) return GR_OK;
  if (GR_DEBUG_SKIP & 16) return GR_OK;
  if (P.num > 0) {
    hipLaunchKernelGGL(k_fit_param_steps, dim3(P.first[P.num]), dim3(256), 0, (hipStream_t)stream, P, (float)(1.0 - beta1),
                       (float)beta2, (float)(1.0 - beta2), eps, sched, (const int*)step_dev, (const int*)overflow);
    GR_HIP_TRY(hipGetLastError());
  }
  if (sched) {
    int* mapped = nullptr;
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, host_flags) == hipSuccess && attr.type == hipMemoryTypeHost && attr.devicePointer)
      mapped = (int*)attr.devicePointer;
    (void)hipGetLastError();
    if (!mapped) return set_error(GR_ERR_INVALID_ARGUMENT, "gr_fit_param_steps_sched: host_flags must be pinned host memory");
    hipLaunchKernelGGL(k_step_advance, dim3(1), dim3(64), 0, (hipStream_t)stream, step_dev, overflow, mapped);
    GR_HIP_TRY(hipGetLastError());
  }
  return GR_OK;
}

size_t gr_fit_activations_ws_bytes(int64_t n) {
  (void)n;
  return 2 * ACT_BLOCKS * sizeof(double) + 256;
}

gr_status gr_fit_activations(int64_t n, const float* scales_raw, const float* opacities_raw, const float* colors_raw,
                             int64_t color_count, float* scales, float* opacities, float* colors, float reg_scale,
                             float reg_opacity, float* reg_out, void* ws, size_t ws_bytes, void* stream) {
  if (n < 0 || color_count < 0) return set_error(GR_ERR_INVALID_ARGUMENT, "gr_fit_activations: negative count");
  if (n > 0 && (!scales_raw || !opacities_raw || !scales || !opacities))
    return set_error(GR_ERR_INVALID_ARGUMENT, "gr_fit_activations: null pointer");
  if (colors_raw && color_count > 0 && !colors) return set_error(GR_ERR_INVALID_ARGUMENT, "gr_fit_activations: null colors");
  if (reg_out && (!ws || ws_bytes < gr_fit_activations_ws_bytes(n)))
    return set_error(GR_ERR_WORKSPACE, "gr_fit_activations: workspace too small");
  if (n == 0) {
    if (reg_out) return set_error(GR_ERR_INVALID_ARGUMENT, "gr_fit_activations: the regulariser of no Gaussians");
    return GR_OK;
  }
  const int64_t most = std::max<int64_t>(3 * n, colors_raw ? color_count : 0);
  const int blocks = (int)std::min<int64_t>(ACT_BLOCKS, (most + 255) / 256);
  double* part = (double*)ws;
  int* ticket = ws ? (int*)((char*)ws + 2 * ACT_BLOCKS * sizeof(double)) : nullptr;
  hipLaunchKernelGGL(k_fit_activations, dim3(blocks), dim3(256), 0, (hipStream_t)stream, n, scales_raw, opacities_raw,
                     colors_raw, colors_raw ? color_count : 0, scales, opacities, colors, reg_scale, reg_opacity, reg_out,
                     part, ticket);
  GR_HIP_TRY(hipGetLastError());
  return GR_OK;
}

gr_status gr_fit_param_steps(int num, const gr_param_step* steps, double beta1, double beta2, float eps, void* stream) {
  return param_steps_impl(num, steps, beta1, beta2, eps, nullptr, nullptr, nullptr, nullptr, stream);
}

gr_status gr_fit_param_steps_sched(int num, const gr_param_step* steps, double beta1, double beta2, float eps,
                                   const float* sched, int* step_dev, int* overflow, int* host_flags, void* stream) {
  if (!sched || !step_dev || !overflow || !host_flags)
    return set_error(GR_ERR_INVALID_ARGUMENT, "gr_fit_param_steps_sched: null schedule, counter, overflow or flags");
  return param_steps_impl(num, steps, beta1, beta2, eps, sched, step_dev, overflow, host_flags, stream);
}

gr_status gr_adam_step(int64_t count, float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                       float neg_step_size, float bias_correction2_sqrt, double beta1, double beta2, float eps, void* stream) {
  if (count < 0 || !param || !grad || !exp_avg || !exp_avg_sq) return set_error(GR_ERR_INVALID_ARGUMENT, "gr_adam_step: bad arguments");
  if (count == 0) return GR_OK;
  const int blocks = (int)std::min<int64_t>((count + 255) / 256, 4096);
  const float w1 = (float)(1.0 - beta1), w2 = (float)(1.0 - beta2);
  hipLaunchKernelGGL(k_adam_step, dim3(blocks), dim3(256), 0, (hipStream_t)stream, count, param, grad, exp_avg, exp_avg_sq,
                     neg_step_size, bias_correction2_sqrt, w1, (float)beta2, w2, eps);
  GR_HIP_TRY(hipGetLastError());
  return GR_OK;
}

gr_status gr_l1_loss_bwd(const float* a, const float* b, int64_t n1, const float* c, const float* d, int64_t n2, float w2,
                         const float* g_loss, float* g_a, float* g_c, void* stream) {
  if (n1 <= 0 || n2 < 0 || !a || !b || !g_loss || !g_a || (n2 > 0 && (!c || !d || !g_c)))
    return set_error(GR_ERR_INVALID_ARGUMENT, "gr_l1_loss_bwd: bad arguments");
  const int64_t nm = n1 > n2 ? n1 : n2;
  hipLaunchKernelGGL(k_l1_grad, dim3(blocks_for(nm)), dim3(256), 0, (hipStream_t)stream, a, b, n1, c, d, n2, w2, g_loss,
                     g_a, g_c);
  GR_HIP_TRY(hipGetLastError());
  return GR_OK;
}

}  // extern "C"
