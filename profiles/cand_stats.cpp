// profiles/cand_stats.cpp -- candidate-list statistics of the binned locator on a synthetic
// grid (host build, irt_debug_scene_*): for random points in the shell, the number of
// candidates the sub-cell mask admits in the point's bin (what a one-hop "test every
// admitted candidate" scan would gather) against the number the serial scan tests before
// its first hit.  Build: make -C profiles cand_stats (links the product library's host part).
//   ./cand_stats bisections levels terrainHeight npoints
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <random>
#include <vector>

#include "icon_rt_hip.h"
#include "icon_rt_hip_debug.h"
#include "irt_build.h"

using namespace irt;

int main(int argc, char **argv) {
  const int bis = argc > 1 ? atoi(argv[1]) : 5, levels = argc > 2 ? atoi(argv[2]) : 90;
  const float terrain = argc > 3 ? (float)atof(argv[3]) : 0.f;
  const long npts = argc > 4 ? atol(argv[4]) : 200000;
  const float top = 75000.f;
  size_t n = 0;
  irt_synth_grid_terrain(2, bis, levels, top, 0.f, 1u, terrain, nullptr, 0, &n);
  std::vector<irt_icon_cell> cells(n);
  if (irt_synth_grid_terrain(2, bis, levels, top, 0.f, 1u, terrain, cells.data(), n, &n)) return 1;
  irt_debug_scene *s = nullptr;
  if (irt_debug_scene_build(cells.data(), n, &s)) return 1;
  size_t hb = 0, fb = 0;
  irt_debug_scene_array(s, IRT_DEBUG_ARRAY_BIN_HDR, nullptr, 0, &hb);
  irt_debug_scene_array(s, IRT_DEBUG_ARRAY_FAT, nullptr, 0, &fb);
  std::vector<uint32_t> H(hb / 4);
  std::vector<float> F(fb / 4);
  irt_debug_scene_array(s, IRT_DEBUG_ARRAY_BIN_HDR, H.data(), hb, &hb);
  irt_debug_scene_array(s, IRT_DEBUG_ARRAY_FAT, F.data(), fb, &fb);
  const int G = (int)llround(sqrt((double)(H.size() / kBinHdrWords) / 6.0));
  std::mt19937_64 rng(7);
  std::uniform_real_distribution<double> U(0.0, 1.0);
  const float R = 6371229.f;
  long found = 0, hist[17] = {0}, tested = 0, admitted = 0, firstPass = 0;
  long failRadial = 0, failPlane = 0, testedHalf = 0, admittedHalf = 0, binFirst = 0, quadFirst = 0, secondPass = 0, secondSame = 0, needThird = 0;
  for (long i = 0; i < npts; ++i) {
    const double z = 2 * U(rng) - 1, ph = 2 * M_PI * U(rng), rr = sqrt(1 - z * z);
    const float r0 = R + (float)(U(rng) * top);
    const float px = (float)(r0 * rr * cos(ph)), py = (float)(r0 * rr * sin(ph)), pz = (float)(r0 * z);
    const float r = sqrtf(px * px + py * py + pz * pz);
    uint32_t sub = 0;
    const uint32_t cell = cubemap_cell_sub(px, py, pz, G, sub);
    const uint32_t *h = &H[(size_t)cell * kBinHdrWords];
    const int b = bin_of(r, u2f(h[0]), u2f(h[1]), u2f(h[2]));
    const uint32_t beg = h[3] + (b ? h[4 + b - 1] : 0), end = h[3] + h[4 + b];
    const uint32_t mask = (h[8 + sub] >> (8 * b)) & 0xFFu;
    // a radial half mask: the bin split at the midpoint of its entries' radial extent (clipped
    // to the bin); below it only candidates with h0 < mid, above only those with hN >= mid
    float lo = INFINITY, hi = -INFINITY;
    for (uint32_t q = beg; q < end; ++q) {
      lo = fminf(lo, F[(size_t)q * 16 + 12]);
      hi = fmaxf(hi, F[(size_t)q * 16 + 13]);
    }
    if (b > 0) lo = fmaxf(lo, u2f(h[b - 1]));
    if (b < 3) hi = fminf(hi, u2f(h[b]));
    const float mid = 0.5f * (lo + hi);
    int adm = 0, t = 0, hit = -1, admH = 0, tH = 0, hitH = -1;
    // the union of the masks of the sub-cell's 2 x 2 quad (kSub = 4: quads of sub-cells)
    const uint32_t si = sub % kSub, sj = sub / kSub, q0 = (sj & ~1u) * kSub + (si & ~1u);
    const uint32_t qmask = ((h[8 + q0] | h[8 + q0 + 1] | h[8 + q0 + kSub] | h[8 + q0 + kSub + 1]) >> (8 * b)) & 0xFFu;
    int qj = -1;  // the quad's first admitted candidate
    const float *e1st = nullptr;
    for (uint32_t j = 0; beg + j < end && qj < 0; ++j)
      if (j >= (uint32_t)kMaskCand || ((qmask >> j) & 1u)) qj = (int)j;
    for (uint32_t j = 0; beg + j < end; ++j) {
      if (j < (uint32_t)kMaskCand && !((mask >> j) & 1u)) continue;
      ++adm;
      const float *e = &F[(size_t)(beg + j) * 16];
      const bool rad = !(r < e[12] || r > e[13]);
      bool ok = rad;
      for (int k = 0; ok && k < 3; ++k)
        if (eval_plane(e + 4 * k, px, py, pz) > 0.f) ok = false;
      if (hit < 0) {
        ++t;
        if (!ok) ++(rad ? failPlane : failRadial);
        if (ok) hit = adm;
      }
      if (j == 0 && ok) ++binFirst;
      if ((int)j == qj && ok) ++quadFirst;
      if (adm == 1) e1st = e;
      if (adm == 2 && t == 2) {  // the first admitted failed: is the second like it?
        if (e[12] == e1st[12] && e[13] == e1st[13] && e[15] == e1st[15]) ++secondSame;
      }  // the bin's first candidate (unmasked) is the answer
      const bool half = j >= (uint32_t)kMaskCand || (r < mid ? e[12] < mid : e[13] >= mid);
      if (half) {
        ++admH;
        if (hitH < 0) {
          ++tH;
          if (ok) hitH = admH;
        }
      }
    }
    if (hit < 0) continue;
    ++found;
    if (hit == 2) ++secondPass;
    if (hit > 2) ++needThird;
    if (hitH < 0) {
      printf("half mask lost a hit\n");
      return 1;
    }
    tested += t;
    testedHalf += tH;
    admittedHalf += admH;
    admitted += adm;
    firstPass += hit == 1;
    ++hist[adm < 16 ? adm : 16];
  }
  printf("R2B%02d x %d terrain %.0f: G %d, %zu records, %zu entries, %ld/%ld located\n", bis, levels,
         terrain, G, n, F.size() / 16, found, npts);
  printf("tested per sample %.3f, admitted per sample %.3f, first admitted passes %.3f\n",
         (double)tested / found, (double)admitted / found, (double)firstPass / found);
  printf("failed tests per sample: radial %.3f, planes %.3f; with a radial half mask: tested %.3f, admitted %.3f\n",
         (double)failRadial / found, (double)failPlane / found, (double)testedHalf / found,
         (double)admittedHalf / found);
  printf("the second admitted answers %.3f (its radial range and meta equal the first's when the first fails: %.3f); a third or later %.3f\n",
         (double)secondPass / found, (double)secondSame / found, (double)needThird / found);
  printf("the bin's first candidate is the answer: %.3f; the 2x2 quad's first admitted: %.3f\n",
         (double)binFirst / found, (double)quadFirst / found);
  printf("admitted histogram:");
  for (int k = 0; k <= 16; ++k)
    if (hist[k]) printf(" %d:%.4f", k, (double)hist[k] / found);
  printf("\n");
  irt_debug_scene_free(s);
  return 0;
}
