// gr_fit_exec.cpp — the fit step's per-view schedule as native host code (gr_fit_views, include/gr_hip.h).
//
// The reference fit loop renders its views one after another (fit_multiview_stub.py:277-310).  The
// multi-GPU driver (3dgaussian_amd/fit_multiview.py) runs the same work on several HIP streams with the
// views' preparations ahead on a stream of their own; this file is that schedule in C++, so a step costs
// the host a few microseconds per launch instead of the Python driver's per-view interpreter work
// (the small-view configs and the per-rank share of a multi-GPU step are host-bound in Python).
//
// Only the public C ABI (gr_fwd_prepare_views_async, gr_fwd_render_l1, gr_bwd_splat, gr_gather_view,
// gr_reduce_sums, gr_fwd_render, gr_bwd_fit) and the HIP runtime are used.  Workspaces are the executor's
// own, kept across steps and reused only in stream order: each render stream owns its view workspace
// (bins, forward scratch, backward workspace, saved sums) and a ring of per-view sums for its reduction
// batch; the geoms are a ring of slots written on the preparation stream, a slot being rewritten only
// after the preparation stream has waited for the event recorded behind its last reader.  A buffer that
// must grow is replaced after its stream has drained (rare: the first step, a densify).
// The schedule (streams, preparation groups, reduction batches) is exactly fit_multiview._views_direct's,
// so both give bit-identical losses and gradients (tests/test_fit_exec_gpu.py).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <deque>
#include <string>
#include <vector>

#include "../../include/gr_hip.h"

extern "C" gr_status gr_exec_set_error(gr_status st, const char* msg);  // gr_hip.hip: thread-local message

namespace {

struct Sched {
  int ns;                              // streams used
  std::vector<std::deque<int>> sizes;  // per stream: its reduction batch sizes, in order
};

// fit_multiview._views_direct's batches: stream k's views in near-equal batches of at most reduce_batch,
// the last one reduce_tail views (when 0 < tail < the stream's view count).
Sched schedule(int views, const gr_fit_config& c) {
  Sched s;
  s.ns = std::max(1, std::min(c.num_streams, views));
  s.sizes.resize(s.ns);
  for (int k = 0; k < s.ns; ++k) {
    const int p = views > k ? (views - k + s.ns - 1) / s.ns : 0;
    const int tail = (c.reduce_tail > 0 && c.reduce_tail < p) ? c.reduce_tail : 0;
    const int nb = std::max(1, (p - tail + c.reduce_batch - 1) / c.reduce_batch);
    for (int b = 0; b < nb; ++b) s.sizes[k].push_back((p - tail) / nb + (b < (p - tail) % nb ? 1 : 0));
    if (tail) s.sizes[k].push_back(tail);
  }
  return s;
}

}  // namespace

// A device buffer that grows: replaced (old one freed after `s` has drained) when a request exceeds it.
struct Buf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t fit(size_t bytes, hipStream_t s) {
    if (bytes <= cap) return hipSuccess;
    if (p) {
      hipError_t e = hipStreamSynchronize(s);
      if (e == hipSuccess) e = hipFree(p);
      if (e != hipSuccess) return e;
      p = nullptr;
      cap = 0;
    }
    const size_t want = bytes + bytes / 8 + (1u << 20);  // headroom: pair counts drift from step to step
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

struct StreamWs {  // one render stream's buffers
  Buf bins, scratch, ws, saved;
  std::vector<Buf> sums, sums3;  // one per view of a reduction batch (sums3: the depth-loss path's depth sums)
};

struct GeomSlot {
  Buf buf;
  hipEvent_t free_ev = nullptr;  // recorded behind the slot's last reader
  bool pending = false;          // free_ev recorded and not yet waited for by the preparation stream
};

struct gr_executor {
  int device = 0;
  hipStream_t prep = nullptr;
  std::vector<hipStream_t> side;   // render streams 1..; stream 0 is the caller's
  std::vector<hipEvent_t> groups;  // one event per preparation group (reused across steps)
  hipEvent_t in = nullptr;
  std::vector<hipEvent_t> done;    // side streams' ends
  gr_plan* plans = nullptr;        // pinned, mapped: one plan per view (written by the preparation kernels)
  int plans_cap = 0;
  std::vector<StreamWs> ws;        // per render stream
  std::vector<GeomSlot> geoms;     // ring of geom slots
  std::vector<hipStream_t> last;   // the previous call's render streams 1.. and preparation stream
};

#define GR_EXEC_TRY(expr)                                                            \
  do {                                                                               \
    hipError_t e_ = (expr);                                                          \
    if (e_ != hipSuccess) return gr_exec_set_error(GR_ERR_HIP, hipGetErrorString(e_)); \
  } while (0)
#define GR_EXEC_CALL(expr)          \
  do {                              \
    gr_status s_ = (expr);          \
    if (s_ != GR_OK) return s_;     \
  } while (0)

static gr_status fit_views_on_device(gr_executor* ex, const gr_fit_config* cfg, int num_views, const gr_fit_target* views,
                                     int n, const float* means, const float* scales, const float* colors, int color_dim,
                                     const float* opacities, float w_sil, float w_depth, float g_scale, float* losses,
                                     float* const* acc, void* stream);
static gr_status enqueue_views(gr_executor* ex, const gr_fit_config* cfg, int num_views, const gr_fit_target* views, int n,
                               const float* means, const float* scales, const float* colors, int color_dim,
                               const float* opacities, float w_sil, float w_depth, float g_scale, float* losses,
                               float* const* acc, const Sched& sc, const std::vector<hipStream_t>& st, hipStream_t prep,
                               bool depth, int nslots, int& ngroups);

extern "C" {

gr_status gr_executor_create(int device, gr_executor** out) {
  if (!out) return gr_exec_set_error(GR_ERR_INVALID_ARGUMENT, "gr_executor_create: null output");
  *out = nullptr;
  int cur = 0;
  GR_EXEC_TRY(hipGetDevice(&cur));
  GR_EXEC_TRY(hipSetDevice(device));
  gr_executor* ex = new gr_executor();
  ex->device = device;
  // streams are made on first use, and only when the caller passes none (stream creation order decides the
  // hardware queue each lands on)
  hipError_t e = hipEventCreateWithFlags(&ex->in, hipEventDisableTiming);
  (void)hipSetDevice(cur);
  if (e != hipSuccess) {
    gr_executor_destroy(ex);
    return gr_exec_set_error(GR_ERR_HIP, hipGetErrorString(e));
  }
  *out = ex;
  return GR_OK;
}

void gr_executor_destroy(gr_executor* ex) {
  if (!ex) return;
  if (ex->prep) (void)hipStreamSynchronize(ex->prep);
  for (hipStream_t s : ex->side) {
    (void)hipStreamSynchronize(s);
    (void)hipStreamDestroy(s);
  }
  (void)hipDeviceSynchronize();  // no queued work still uses the executor's buffers
  for (auto& w : ex->ws) {
    w.bins.release();
    w.scratch.release();
    w.ws.release();
    w.saved.release();
    for (auto& b : w.sums) b.release();
    for (auto& b : w.sums3) b.release();
  }
  for (auto& g : ex->geoms) {
    g.buf.release();
    if (g.free_ev) (void)hipEventDestroy(g.free_ev);
  }
  for (hipEvent_t e : ex->groups) (void)hipEventDestroy(e);
  for (hipEvent_t e : ex->done) (void)hipEventDestroy(e);
  if (ex->in) (void)hipEventDestroy(ex->in);
  if (ex->prep) (void)hipStreamDestroy(ex->prep);
  if (ex->plans) (void)hipHostFree(ex->plans);
  delete ex;
}

gr_status gr_fit_views(gr_executor* ex, const gr_fit_config* cfg, int num_views, const gr_fit_target* views, int n,
                       const float* means, const float* scales, const float* colors, int color_dim,
                       const float* opacities, float w_sil, float w_depth, float g_scale, float* losses,
                       float* const* acc, void* stream) {
  if (!ex || !cfg || (num_views > 0 && (!views || !losses || !acc)))
    return gr_exec_set_error(GR_ERR_INVALID_ARGUMENT, "gr_fit_views: null argument");
  // every batch of a stream (its last one holds reduce_tail views) and every preparation group must fit the
  // fixed-size view arrays of gr_reduce_sums / gr_fwd_prepare_views_async (and the per-stream sums ring)
  if (cfg->num_streams < 1 || cfg->prep_ahead < 1 || cfg->prep_group < 1 || cfg->prep_group > GR_PREPARE_MAX_VIEWS ||
      cfg->prep_first < 1 || cfg->prep_first > GR_PREPARE_MAX_VIEWS || cfg->reduce_batch < 1 ||
      cfg->reduce_batch > GR_REDUCE_MAX_VIEWS || cfg->reduce_tail < 0 || cfg->reduce_tail > cfg->reduce_batch)
    return gr_exec_set_error(GR_ERR_INVALID_ARGUMENT, "gr_fit_views: configuration out of range");
  if (num_views == 0 || n <= 0) return GR_OK;
  if (cfg->caps && !cfg->overflow) return gr_exec_set_error(GR_ERR_INVALID_ARGUMENT, "gr_fit_views: caps without overflow");
  const bool depth = views[0].target_depth != nullptr;  // the depth-loss path (one form per call)
  for (int j = 0; j < num_views; ++j) {
    if ((views[j].target_depth != nullptr) != depth)
      return gr_exec_set_error(GR_ERR_INVALID_ARGUMENT, "gr_fit_views: every view or none has a depth target");
    if (!views[j].target_rgb) return gr_exec_set_error(GR_ERR_INVALID_ARGUMENT, "gr_fit_views: null target");
  }
  // the executor's streams, events and buffers belong to its device: make it current for this call
  int prev_dev = 0;
  GR_EXEC_TRY(hipGetDevice(&prev_dev));
  GR_EXEC_TRY(hipSetDevice(ex->device));
  const gr_status st = fit_views_on_device(ex, cfg, num_views, views, n, means, scales, colors, color_dim, opacities, w_sil,
                                           w_depth, g_scale, losses, acc, stream);
  (void)hipSetDevice(prev_dev);
  return st;
}

}  // extern "C"

static gr_status fit_views_on_device(gr_executor* ex, const gr_fit_config* cfg, int num_views, const gr_fit_target* views,
                                     int n, const float* means, const float* scales, const float* colors, int color_dim,
                                     const float* opacities, float w_sil, float w_depth, float g_scale, float* losses,
                                     float* const* acc, void* stream) {
  const bool depth = views[0].target_depth != nullptr;
  const Sched sc = schedule(num_views, *cfg);
  const int ns = sc.ns;
  for (int k = 0; k < ns; ++k)
    for (int q = 0; q < 4; ++q)
      if (!acc[4 * k + q]) return gr_exec_set_error(GR_ERR_INVALID_ARGUMENT, "gr_fit_views: null accumulator");
  hipStream_t main = (hipStream_t)stream;
  // streams, events and the plan array, grown on demand and kept
  while (!cfg->render_streams && (int)ex->side.size() < ns - 1) {
    hipStream_t s;
    GR_EXEC_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    ex->side.push_back(s);
  }
  while ((int)ex->done.size() < ns - 1) {
    hipEvent_t e;
    GR_EXEC_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    ex->done.push_back(e);
  }
  if ((int)ex->ws.size() < ns) ex->ws.resize(ns);
  for (int k = 0; k < ns; ++k)
    if ((int)ex->ws[k].sums.size() < cfg->reduce_batch) {
      ex->ws[k].sums.resize(cfg->reduce_batch);
      ex->ws[k].sums3.resize(cfg->reduce_batch);
    }
  // geom slots: the views prepared ahead, the ones rendering on every stream, and a margin
  const int nslots = cfg->prep_ahead + cfg->prep_group + ns + 2;
  while ((int)ex->geoms.size() < nslots) {
    ex->geoms.emplace_back();
    GR_EXEC_TRY(hipEventCreateWithFlags(&ex->geoms.back().free_ev, hipEventDisableTiming));
  }
  const int max_groups = num_views + 1;
  while ((int)ex->groups.size() < max_groups) {
    hipEvent_t e;
    GR_EXEC_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    ex->groups.push_back(e);
  }
  if (ex->plans_cap < num_views) {
    if (ex->plans) {
      GR_EXEC_TRY(hipDeviceSynchronize());  // no preparation of an earlier step still writes them
      GR_EXEC_TRY(hipHostFree(ex->plans));
    }
    GR_EXEC_TRY(hipHostMalloc((void**)&ex->plans, sizeof(gr_plan) * num_views, hipHostMallocMapped));
    ex->plans_cap = num_views;
  }
  std::vector<hipStream_t> st(ns);
  st[0] = main;
  for (int k = 1; k < ns; ++k) {
    st[k] = cfg->render_streams ? (hipStream_t)cfg->render_streams[k - 1] : ex->side[k - 1];
    if (!st[k]) return gr_exec_set_error(GR_ERR_INVALID_ARGUMENT, "gr_fit_views: null render stream");
  }
  if (!cfg->prep_stream && !ex->prep) GR_EXEC_TRY(hipStreamCreateWithFlags(&ex->prep, hipStreamNonBlocking));
  const hipStream_t prep = cfg->prep_stream ? (hipStream_t)cfg->prep_stream : ex->prep;
  // the workspaces of every render stream (stream 0's on the caller's stream) and the geom slots were last used on
  // the previous call's streams: when any of them changes, those finish first
  std::vector<hipStream_t> now(st.begin(), st.end());
  now.push_back(prep);
  if (!ex->last.empty() && ex->last != now)
    for (hipStream_t s : ex->last) GR_EXEC_TRY(hipStreamSynchronize(s));
  ex->last = now;
  // everything starts after the caller's stream (the activations)
  GR_EXEC_TRY(hipEventRecord(ex->in, main));
  GR_EXEC_TRY(hipStreamWaitEvent(prep, ex->in, 0));
  for (int k = 1; k < ns; ++k) GR_EXEC_TRY(hipStreamWaitEvent(st[k], ex->in, 0));
  // From here work is enqueued on the executor's streams: whatever happens below, the caller's stream is ordered
  // after all of it before this returns (an error part-way must not let the caller free buffers still in use).
  int ngroups = 0;
  auto join = [&]() {
    for (int k = 1; k < ns; ++k)
      if (hipEventRecord(ex->done[k - 1], st[k]) != hipSuccess || hipStreamWaitEvent(main, ex->done[k - 1], 0) != hipSuccess)
        (void)hipStreamSynchronize(st[k]);
    if (hipEventRecord(ex->groups[ngroups], prep) != hipSuccess || hipStreamWaitEvent(main, ex->groups[ngroups], 0) != hipSuccess)
      (void)hipStreamSynchronize(prep);
  };
  const gr_status status = enqueue_views(ex, cfg, num_views, views, n, means, scales, colors, color_dim, opacities, w_sil,
                                         w_depth, g_scale, losses, acc, sc, st, prep, depth, nslots, ngroups);
  join();
  return status;
}

static gr_status enqueue_views(gr_executor* ex, const gr_fit_config* cfg, int num_views, const gr_fit_target* views, int n,
                               const float* means, const float* scales, const float* colors, int color_dim,
                               const float* opacities, float w_sil, float w_depth, float g_scale, float* losses,
                               float* const* acc, const Sched& sc, const std::vector<hipStream_t>& st, hipStream_t prep,
                               bool depth, int nslots, int& ngroups) {
  const int ns = sc.ns;
  const bool sized = cfg->caps != nullptr;  // device-side sizing: the plans are capacities, nothing to wait for
  const size_t geom_bytes = gr_geom_bytes(n);
  std::vector<void*> geom(num_views, nullptr);
  std::vector<int> slot_of(num_views, -1);
  std::vector<int> group_of(num_views, -1);
  int next_prep = 0;
  auto prepare_upto = [&](int j) -> gr_status {  // views [next_prep, j] prepared (whole groups)
    while (next_prep < num_views && next_prep <= j) {
      const int g0 = next_prep, cnt = std::min(num_views - g0, g0 == 0 ? cfg->prep_first : cfg->prep_group);
      gr_view vs[GR_PREPARE_MAX_VIEWS];
      void* gs[GR_PREPARE_MAX_VIEWS];
      gr_plan* ps[GR_PREPARE_MAX_VIEWS];
      for (int q = 0; q < cnt; ++q) {
        const int sl = (g0 + q) % nslots;
        GeomSlot& g = ex->geoms[sl];
        if (g.pending) {  // its previous view's readers first (stream order on the preparation stream)
          GR_EXEC_TRY(hipStreamWaitEvent(prep, g.free_ev, 0));
          g.pending = false;
        }
        GR_EXEC_TRY(g.buf.fit(geom_bytes, prep));
        geom[g0 + q] = g.buf.p;
        slot_of[g0 + q] = sl;
        vs[q] = views[g0 + q].view;
        gs[q] = geom[g0 + q];
        ps[q] = sized ? (cfg->observed ? &cfg->observed[g0 + q] : nullptr) : &ex->plans[g0 + q];
        group_of[g0 + q] = ngroups;
      }
      if (sized)
        GR_EXEC_CALL(gr_fwd_prepare_views_sized(cnt, vs, n, means, scales, colors, color_dim, opacities, gs, geom_bytes,
                                                cfg->caps + g0, ps, cfg->overflow, prep));
      else
        GR_EXEC_CALL(gr_fwd_prepare_views_async(cnt, vs, n, means, scales, colors, color_dim, opacities, gs, geom_bytes, ps,
                                                prep));
      GR_EXEC_TRY(hipEventRecord(ex->groups[ngroups], prep));
      ++ngroups;
      next_prep = g0 + cnt;
    }
    return GR_OK;
  };

  struct Pending {
    gr_view view;
    float* sums;
    float* sums3;  // depth sums (depth-loss path) or null
  };
  // a slot's previous view must have been waited for before the slot is refilled: with nslots > prep_ahead
  // + prep_group + ns the view a slot last held was rendered (and its free event recorded) before the
  // preparation that refills it is enqueued
  std::vector<std::vector<Pending>> pending(ns);
  std::vector<std::deque<int>> sizes = sc.sizes;
  std::vector<int> started(ns, 0);
  const size_t sums_bytes = gr_view_sums_floats(n) * sizeof(float);
  auto reduce_pending = [&](int k) -> gr_status {
    if (pending[k].empty()) return GR_OK;
    gr_sums_view b[GR_REDUCE_MAX_VIEWS];
    const int nb = (int)pending[k].size();
    for (int q = 0; q < nb; ++q) {
      b[q].view = pending[k][q].view;
      b[q].sums = pending[k][q].sums;
      b[q].sums3 = pending[k][q].sums3;
    }
    GR_EXEC_CALL(gr_reduce_sums(nb, b, n, means, scales, colors, color_dim, opacities, acc[4 * k + 0], acc[4 * k + 1],
                                acc[4 * k + 2], acc[4 * k + 3], started[k], st[k]));
    pending[k].clear();
    started[k] = 1;
    return GR_OK;
  };

  // the first two groups, then one more after each render (fit_multiview._prep_groups): the first render is
  // enqueued before the later groups
  GR_EXEC_CALL(prepare_upto(std::min(cfg->prep_first, cfg->prep_ahead - 1)));
  for (int j = 0; j < num_views; ++j) {
    const int k = j % ns;
    hipStream_t s = st[k];
    GR_EXEC_CALL(prepare_upto(j));
    const hipEvent_t ev = ex->groups[group_of[j]];
    GR_EXEC_TRY(hipStreamWaitEvent(s, ev, 0));
    if (!sized) GR_EXEC_TRY(hipEventSynchronize(ev));  // the plan (pair count) sizes this view's workspaces
    const gr_plan plan = sized ? cfg->caps[j] : ex->plans[j];
    if (plan.num_pairs < 0 || plan.num_slots < 0) return gr_exec_set_error(GR_ERR_OVERFLOW, "pair count overflows int32");
    const gr_view& v = views[j].view;
    const size_t bins_bytes = gr_bins_bytes(&v, n, &plan), scratch_bytes = gr_fwd_scratch_bytes(&v, n, &plan);
    const size_t ws_bytes = gr_bwd_bytes(&v, n, &plan);
    StreamWs& W = ex->ws[k];
    GR_EXEC_TRY(W.bins.fit(bins_bytes, s));
    GR_EXEC_TRY(W.scratch.fit(scratch_bytes, s));
    GR_EXEC_TRY(W.ws.fit(ws_bytes, s));
    void *bins = W.bins.p, *scratch = W.scratch.p, *ws = W.ws.p;
    if (!depth) {
      GR_EXEC_CALL(gr_fwd_render_l1(&v, n, &plan, geom[j], bins, W.bins.cap, scratch, W.scratch.cap, views[j].target_rgb,
                                    views[j].target_mask, w_sil, g_scale, losses + j, nullptr, nullptr, ws, W.ws.cap, s));
      GR_EXEC_CALL(gr_bwd_splat(&v, n, &plan, geom[j], bins, ws, W.ws.cap, s));
      Buf& sb = W.sums[pending[k].size()];
      GR_EXEC_TRY(sb.fit(sums_bytes, s));
      GR_EXEC_CALL(gr_gather_view(&v, n, &plan, geom[j], bins, ws, (float*)sb.p, s));
      pending[k].push_back({v, (float*)sb.p, nullptr});
    } else {
      GR_EXEC_TRY(W.saved.fit(gr_saved_floats(&v) * sizeof(float), s));
      GR_EXEC_CALL(gr_fwd_render(&v, n, &plan, geom[j], bins, W.bins.cap, scratch, W.scratch.cap, nullptr, nullptr,
                                 nullptr, (float*)W.saved.p, s));
      Buf& sb = W.sums[pending[k].size()];
      Buf& s3 = W.sums3[pending[k].size()];
      GR_EXEC_TRY(sb.fit(sums_bytes, s));
      GR_EXEC_TRY(s3.fit((size_t)n * sizeof(float), s));
      GR_EXEC_CALL(gr_bwd_fit_gather(&v, n, &plan, geom[j], bins, (const float*)W.saved.p, views[j].target_rgb,
                                     views[j].target_mask, w_sil, views[j].target_depth, w_depth, g_scale, losses + j, ws,
                                     W.ws.cap, (float*)sb.p, (float*)s3.p, s));
      pending[k].push_back({v, (float*)sb.p, (float*)s3.p});
    }
    // the geom slot may be refilled once this stream has passed its last reader
    GeomSlot& gsl = ex->geoms[slot_of[j]];
    GR_EXEC_TRY(hipEventRecord(gsl.free_ev, s));
    gsl.pending = true;
    geom[j] = nullptr;
    GR_EXEC_CALL(prepare_upto(j + cfg->prep_ahead));
    if ((int)pending[k].size() >= sizes[k].front()) {
      GR_EXEC_CALL(reduce_pending(k));
      if (sizes[k].size() > 1) sizes[k].pop_front();
    }
  }
  for (int k = 0; k < ns; ++k) GR_EXEC_CALL(reduce_pending(k));
  return GR_OK;  // the caller joins the streams (fit_views_on_device)
}
