// TEST INFRASTRUCTURE ONLY.  C shim over the reference's own CPU renderer so ctypes can call it.
// Built by oracle/build_ref.sh against /root/reference/src/renderer_cpu.cpp (compiled in place,
// never copied); output goes to oracle/_ref/ (git-ignored).  Used only to pin the oracle's
// uint8 restatement (tests/golden/make_golden.py).
#include <cstdint>
#include <cstring>
#include <vector>

#include "gr/gaussian_types.h"
#include "gr/renderer.h"

extern "C" int ref_render_u8(int width, int height, const float* view, const float* proj, const float* bg,
                             int enable_depth_sort, int n, const float* means, const float* scales,
                             const float* colors, const float* opac, uint8_t* rgba) {
  gr::RenderParams p;
  p.width = width;
  p.height = height;
  std::memcpy(p.view, view, sizeof(float) * 16);
  std::memcpy(p.proj, proj, sizeof(float) * 16);
  std::memcpy(p.background, bg, sizeof(float) * 3);
  p.enable_depth_sort = enable_depth_sort;
  p.force_cpu = 1;
  std::vector<std::uint8_t> out = gr::render_gaussians_cpu(means, scales, colors, opac, n, p);
  std::memcpy(rgba, out.data(), out.size());
  return 0;
}
