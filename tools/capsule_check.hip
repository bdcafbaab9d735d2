// capsule_check.hip -- GPU check of the capsule-prism separation distance
// (tool, not shipped): bb_bodycon.h:capsule_prism_apart (9 edge pairs + 10
// face projections) against the minimum over the prism's 8 boundary
// triangles (seg_tri, the oracle's form) on 1M random segment/prism pairs,
// relief and flat prisms.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I openballbot-rl_amd/csrc \
//       tools/capsule_check.hip -o tools/_build/capsule_check
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <random>
#include <vector>

#include "bb_bodycon.h"

using namespace bb;

struct Case { double Tp[3][3], c[3], a[3], hh, r; };
struct Res { int h1, h2; double d1, d2, n1[3], n2[3], p1[3], p2[3]; };

// the triangle form: separation distance as the minimum over the 8 triangles
__device__ bool apart_tri(const Seg<double>& g, const PrismG<double>& P, const double* p0, const double* p1,
                          double& dist, double* n, double* pos) {
  const int tri[8][3] = {{0, 1, 2}, {3, 4, 5}, {0, 1, 4}, {0, 4, 3}, {1, 2, 5}, {1, 5, 4}, {2, 0, 3}, {2, 3, 5}};
  double best = 1e30, bp[3] = {0, 0, 0}, bq[3] = {0, 0, 0};
  for (int f = 0; f < 8; f++) {
    double cp[3], cq[3];
    const double d = seg_tri(p0, p1, P.V[tri[f][0]], P.V[tri[f][1]], P.V[tri[f][2]], cp, cq);
    if (d < best) { best = d; for (int i = 0; i < 3; i++) { bp[i] = cp[i]; bq[i] = cq[i]; } }
  }
  if (best >= g.r) return false;
  if (best > 1e-12) { for (int i = 0; i < 3; i++) n[i] = (bp[i] - bq[i]) / best; }
  else { n[0] = P.pn[0][0]; n[1] = P.pn[0][1]; n[2] = P.pn[0][2]; }
  dist = best - g.r;
  for (int i = 0; i < 3; i++) pos[i] = bp[i] - n[i] * (g.r + dist * 0.5);
  return true;
}

__global__ void check(const Case* cs, Res* rs, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Case& C = cs[i];
  PrismG<double> P;
  prism_build(P, C.Tp, -0.1);
  Seg<double> g;
  for (int j = 0; j < 3; j++) { g.c[j] = C.c[j]; g.a[j] = C.a[j]; }
  g.hh = C.hh; g.r = C.r;
  double p0[3], p1[3];
  seg_ends(g, p0, p1);
  Res R{};
  // only segments that miss the prism (capsule_prism's !inter branch)
  double t0 = 0, t1 = 1;
  bool inter = true;
  for (int f = 0; f < 5; f++) {
    const double dir[3] = {p1[0] - p0[0], p1[1] - p0[1], p1[2] - p0[2]};
    const double a0 = dot3(P.pn[f], p0) - P.pd[f], ad = dot3(P.pn[f], dir);
    if (fabs(ad) < 1e-30) { if (a0 > 0) inter = false; }
    else { const double t = -a0 / ad; if (ad > 0) t1 = fmin(t1, t); else t0 = fmax(t0, t); }
  }
  if (t0 > t1) inter = false;
  if (!inter) {
    R.h1 = capsule_prism_apart(g, P, p0, p1, R.d1, R.n1, R.p1);
    R.h2 = apart_tri(g, P, p0, p1, R.d2, R.n2, R.p2);
  }
  rs[i] = R;
}

int main() {
  const int N = 1 << 20;
  std::vector<Case> cs(N);
  std::mt19937_64 rng(1);
  std::uniform_real_distribution<double> U(-1, 1);
  for (int it = 0; it < N; it++) {
    Case& C = cs[it];
    const double s = 0.03425, x0 = U(rng) * 0.1, y0 = U(rng) * 0.1;  // one hfield cell
    double px[3] = {x0, x0, x0 + s}, py[3] = {y0, y0 + s, y0};
    if (it & 1) { px[0] = x0; py[0] = y0 + s; px[1] = x0 + s; py[1] = y0; px[2] = x0 + s; py[2] = y0 + s; }
    const bool flat = it & 2;
    for (int i = 0; i < 3; i++) { C.Tp[i][0] = px[i]; C.Tp[i][1] = py[i]; C.Tp[i][2] = flat ? 0.0 : 0.05 + 0.02 * U(rng); }
    for (int i = 0; i < 3; i++)
      C.c[i] = i < 2 ? x0 + s / 2 + U(rng) * 0.06 : (flat ? 0.02 + 0.01 * U(rng) : 0.06 + U(rng) * 0.06);
    double a[3] = {U(rng), U(rng), U(rng)};
    const double al = sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
    for (int i = 0; i < 3; i++) C.a[i] = a[i] / al;
    C.hh = 0.02 + 0.05 * (U(rng) + 1);
    C.r = 0.025;
  }
  Case* dc;
  Res* dr;
  if (hipMalloc(&dc, N * sizeof(Case)) != hipSuccess || hipMalloc(&dr, N * sizeof(Res)) != hipSuccess) return 2;
  if (hipMemcpy(dc, cs.data(), N * sizeof(Case), hipMemcpyHostToDevice) != hipSuccess) return 2;
  check<<<N / 64, 64>>>(dc, dr, N);
  std::vector<Res> rs(N);
  if (hipMemcpy(rs.data(), dr, N * sizeof(Res), hipMemcpyDeviceToHost) != hipSuccess) return 2;
  int mism = 0, hits = 0;
  double worst = 0;
  for (int i = 0; i < N; i++) {
    const Res& R = rs[i];
    if (R.h1 != R.h2) { mism++; continue; }
    if (!R.h1) continue;
    hits++;
    double e = fabs(R.d1 - R.d2);
    for (int j = 0; j < 3; j++) e = fmax(e, fmax(fabs(R.n1[j] - R.n2[j]), fabs(R.p1[j] - R.p2[j])));
    worst = fmax(worst, e);
  }
  printf("{\"cases\": %d, \"separated_contacts\": %d, \"contact_decision_mismatches\": %d, \"max_abs_diff\": %.3e}\n", N, hits,
         mism, worst);
  return mism ? 1 : 0;
}
