// Host-side launch planners of the native kernels (csrc/include/apex_amd/launch_plan.h, the
// header the .hip launchers call), built with AddressSanitizer + UBSan on the host (tools/host_sanitize.sh; SURVEY.md 5.2 -- GPU ASan / xnack+ runs are not available on this
// pool).  These planners turn tensor shapes into grids, split counts and workspace sizes; a wrong
// value becomes an out-of-bounds access on the GPU, so they are swept over the ResNet / transformer
// shapes and adversarial edges and their invariants asserted here, where signed overflow and
// out-of-bounds host reads are caught by the sanitizers.
#include "apex_amd/launch_plan.h"

#include <cstdio>
#include <vector>

namespace {

namespace plan = apex_amd::plan;

int g_failures = 0;
int64_t g_checks = 0;

#define CHECK(cond, ...)                                      \
  do {                                                        \
    ++g_checks;                                               \
    if (!(cond)) {                                            \
      ++g_failures;                                           \
      std::fprintf(stderr, "FAIL %s:%d: %s: ", __FILE__, __LINE__, #cond); \
      std::fprintf(stderr, __VA_ARGS__);                      \
      std::fprintf(stderr, "\n");                             \
    }                                                         \
  } while (0)

apex_amd::ConvTapArgs conv_args(int n, int h, int w, int c, int kout, int k, int stride) {
  apex_amd::ConvTapArgs a{};
  a.n = n; a.ih = h; a.iw = w; a.c = c; a.kout = kout;
  a.oh = (h + 2 * (k / 2) - k) / stride + 1;
  a.ow = (w + 2 * (k / 2) - k) / stride + 1;
  a.oht = a.oh; a.owt = a.ow; a.ish = stride; a.isw = stride; a.osh = 1; a.osw = 1;
  a.ntaps = k * k;
  for (int t = 0; t < a.ntaps; ++t) {
    a.dh[t] = t / k - k / 2;
    a.dw[t] = t % k - k / 2;
  }
  return a;
}

void check_conv() {
  const int cus = 256;
  struct S { int c, kout, k, stride, h; };
  std::vector<S> shapes = {{64, 64, 3, 1, 56},    {128, 128, 3, 2, 56}, {128, 128, 3, 1, 28},
                           {256, 256, 3, 2, 28},  {256, 256, 3, 1, 14}, {512, 512, 3, 2, 14},
                           {512, 512, 3, 1, 7},   {64, 256, 1, 1, 56},  {1024, 2048, 1, 2, 14},
                           {2048, 512, 1, 1, 7},  {64, 64, 3, 1, 1},    {64, 128, 3, 1, 3}};
  for (int n : {1, 3, 64, 256, 1024}) {
    for (const S& s : shapes) {
      const apex_amd::ConvTapArgs a = conv_args(n, s.h, s.h, s.c, s.kout, s.k, s.stride);
      const int64_t m = (int64_t)a.n * a.oh * a.ow;
      // fprop: every forced or chosen tile width divides kout, the grid fits the launch's unsigned x
      for (int forced = -1; forced <= plan::kConvCfgs; ++forced) {
        const int cfg = plan::conv_fprop_cfg(a, cus, forced);
        const int bn = plan::conv_fprop_bn(cfg), bm = plan::conv_fprop_bm(cfg);
        CHECK(cfg >= 0 && cfg < plan::kConvCfgs && a.kout % bn == 0, "cfg %d kout %d", cfg, a.kout);
        CHECK(cfg < 7 || plan::conv_fprop2_ok(a), "fprop2 cfg %d with > 2 GiB operands", cfg);
        const int64_t grid = (m + bm - 1) / bm * (a.kout / bn);
        CHECK(grid > 0 && grid < (1ll << 32), "grid %lld", (long long)grid);
      }
      // wgrad: the pixel splits cover [0, m) exactly once, chunks are whole K-steps, every split
      // has work, the output tiling covers kout x ntaps*c
      for (int v = 0; v < plan::kWgradVariants; ++v) {
        const plan::WgPlan p = plan::conv_wgrad(a, cus, v);
        CHECK(p.chunk % plan::kWgradBK == 0 && p.chunk > 0, "chunk %d", p.chunk);
        CHECK((int64_t)p.splits * p.chunk >= m && (int64_t)(p.splits - 1) * p.chunk < m,
              "splits %d chunk %d m %lld", p.splits, p.chunk, (long long)m);
        CHECK(a.kout % p.bm == 0 && (a.ntaps * a.c) % p.bn == 0, "tile %dx%d", p.bm, p.bn);
        CHECK(p.tiles == (a.kout / p.bm) * (a.ntaps * a.c / p.bn), "tiles %d", p.tiles);
        CHECK(!plan::conv_wgrad_variant_ok(a, v) || v == 0 || a.c % p.bn == 0, "tile crosses a tap");
        CHECK((int64_t)p.splits * a.kout * a.ntaps * a.c < (1ll << 40), "workspace");
      }
    }
  }
}

void check_gemm() {
  const int cus = 256;
  std::vector<int64_t> ms = {1, 7, 64, 255, 256, 1000, 1024, 4096, 16384, 50257};
  std::vector<int64_t> ks = {64, 128, 1024, 2048, 3072, 4096, 8192, 16384, 65536};
  for (int64_t m : ms)
    for (int64_t n : {8, 256, 1024, 3072, 4096})
      for (int64_t k : ks) {
        apex_amd::GemmArgs g{};
        g.m = (int)m; g.n = (int)n; g.k = (int)k;
        g.epilogue = apex_amd::kEpiNone;
        int chunk = 0;
        const int parts = plan::gemm_splitk_parts(g, cus, &chunk);
        CHECK(parts >= 1 && chunk > 0, "parts %d chunk %d", parts, chunk);
        if (parts > 1) {
          CHECK(chunk % plan::kGemmBK == 0, "chunk %d", chunk);
          CHECK((int64_t)parts * chunk >= k && (int64_t)(parts - 1) * chunk < k, "parts %d chunk %d k %lld", parts,
                chunk, (long long)k);
        } else {
          CHECK(chunk == k, "unsplit chunk %d k %lld", chunk, (long long)k);
        }
        const int cp = plan::colsum_parts(m, (int)n, cus);
        CHECK(cp >= 1 && cp <= (m + 7) / 8, "colsum parts %d m %lld", cp, (long long)m);
      }
}

void check_norm() {
  for (int64_t groups : {0ll, 1ll, 5ll, 511ll, 512ll, 513ll, 1ll << 20, 1ll << 40}) {
    const int g = plan::ln_bwd_grid(groups, 256);
    CHECK(g >= 1 && g <= 512, "grid %d for %lld groups", g, (long long)groups);
  }
}

}  // namespace

int main() {
  check_conv();
  check_gemm();
  check_norm();
  std::printf("host_checks: %lld checks, %d failures\n", (long long)g_checks, g_failures);
  return g_failures ? 1 : 0;
}
