// bb_bodycon.h -- contact geometry of the dynamic (contype/conaffinity) pairs
// of ballbot.xml besides ball-wheel and ball-hfield:
//   hfield x {tower cylinder, cam sticks, wheel capsules}   (mjc_ConvexHField)
//   ball   x {tower cylinder, cam sticks}                   (sphere-cylinder / sphere-capsule)
// (ballast: contype 0; cam cone meshes: asset absent from the reference).
// Per prism the minimum-translation penetration by the separating-axis
// theorem: exact for capsule-prism (prism face normals + segment x edges),
// cylinder-prism adds the cylinder axis, axis x edges and vertex radials
// (exact except rim-edge contacts).  Same algorithm as the oracle
// (oracle/bb_oracle.c: capsule_prism, cylinder_prism, sphere_cylinder).
#pragma once

#include "bb_physics.h"

namespace bb {

template <typename T>
struct Seg {       // capsule / cylinder: centre, unit axis, half-length, radius
  T c[3], a[3], hh, r;
};

template <typename T>
struct PrismG {    // triangular prism: 6 vertices, 5 outward planes n.x <= d
  T V[6][3], pn[5][3], pd[5];
};

template <typename T>
BB_HD void prism_build(PrismG<T>& P, const T (&Tp)[3][3], T zb) {
#pragma unroll
  for (int i = 0; i < 3; i++) {
    P.V[i][0] = Tp[i][0]; P.V[i][1] = Tp[i][1]; P.V[i][2] = Tp[i][2];
    P.V[3 + i][0] = Tp[i][0]; P.V[3 + i][1] = Tp[i][1]; P.V[3 + i][2] = zb;
  }
  T e1[3] = {Tp[1][0] - Tp[0][0], Tp[1][1] - Tp[0][1], Tp[1][2] - Tp[0][2]};
  T e2[3] = {Tp[2][0] - Tp[0][0], Tp[2][1] - Tp[0][1], Tp[2][2] - Tp[0][2]};
  T nt[3];
  cross3(nt, e1, e2);
  if (nt[2] < 0) { nt[0] = -nt[0]; nt[1] = -nt[1]; nt[2] = -nt[2]; }
  const T il = T(1) / sqrt(dot3(nt, nt));
  P.pn[0][0] = nt[0] * il; P.pn[0][1] = nt[1] * il; P.pn[0][2] = nt[2] * il;
  P.pd[0] = dot3(P.pn[0], Tp[0]);
  P.pn[1][0] = 0; P.pn[1][1] = 0; P.pn[1][2] = -1; P.pd[1] = -zb;
  const T area = (Tp[1][0] - Tp[0][0]) * (Tp[2][1] - Tp[0][1]) - (Tp[2][0] - Tp[0][0]) * (Tp[1][1] - Tp[0][1]);
  const T sgn = area > 0 ? T(1) : T(-1);
#pragma unroll
  for (int i = 0; i < 3; i++) {
    const int j = (i + 1) % 3;
    const T ex = Tp[j][0] - Tp[i][0], ey = Tp[j][1] - Tp[i][1];
    const T nx = ey * sgn, ny = -ex * sgn, nl = sqrt(nx * nx + ny * ny);
    P.pn[2 + i][0] = nx / nl; P.pn[2 + i][1] = ny / nl; P.pn[2 + i][2] = 0;
    P.pd[2 + i] = dot3(P.pn[2 + i], Tp[i]);
  }
}

template <typename T>
BB_HD T prism_support(const PrismG<T>& P, const T* n) {
  T m = dot3(n, P.V[0]);
#pragma unroll
  for (int i = 1; i < 6; i++) m = maxT(m, dot3(n, P.V[i]));
  return m;
}

// max and min of n . V over the prism's vertices (support along n and -n)
template <typename T>
BB_HD void prism_extent(const PrismG<T>& P, const T* n, T& mx, T& mn) {
  mx = mn = dot3(n, P.V[0]);
#pragma unroll
  for (int i = 1; i < 6; i++) {
    const T d = dot3(n, P.V[i]);
    mx = maxT(mx, d);
    mn = minT(mn, d);
  }
}

// closest points of segments p0p1 and q0q1 (Ericson 5.1.9); squared distance
template <typename T>
BB_HD T seg_seg2(const T* p0, const T* p1, const T* q0, const T* q1, T* cp, T* cq) {
  T d1[3] = {p1[0] - p0[0], p1[1] - p0[1], p1[2] - p0[2]};
  T d2[3] = {q1[0] - q0[0], q1[1] - q0[1], q1[2] - q0[2]};
  T r[3] = {p0[0] - q0[0], p0[1] - q0[1], p0[2] - q0[2]};
  const T a = dot3(d1, d1), e = dot3(d2, d2), f = dot3(d2, r);
  T s, t;
  if (a <= T(1e-30) && e <= T(1e-30)) { s = t = 0; }
  else if (a <= T(1e-30)) { s = 0; t = clampT(f / e, T(0), T(1)); }
  else {
    const T c = dot3(d1, r);
    if (e <= T(1e-30)) { t = 0; s = clampT(-c / a, T(0), T(1)); }
    else {
      const T b = dot3(d1, d2), den = a * e - b * b;
      s = den > 0 ? clampT((b * f - c * e) / den, T(0), T(1)) : T(0);
      t = (b * s + f) / e;
      if (t < 0) { t = 0; s = clampT(-c / a, T(0), T(1)); }
      else if (t > 1) { t = 1; s = clampT((b - c) / a, T(0), T(1)); }
    }
  }
#pragma unroll
  for (int i = 0; i < 3; i++) { cp[i] = p0[i] + s * d1[i]; cq[i] = q0[i] + t * d2[i]; }
  T d[3] = {cp[0] - cq[0], cp[1] - cq[1], cp[2] - cq[2]};
  return dot3(d, d);
}

template <typename T>
BB_HD T seg_seg(const T* p0, const T* p1, const T* q0, const T* q1, T* cp, T* cq) {
  return sqrt(seg_seg2(p0, p1, q0, q1, cp, cq));
}

// distance of segment p0p1 to triangle abc (0 if they intersect)
template <typename T>
BB_HD T seg_tri(const T* p0, const T* p1, const T* a, const T* b, const T* c, T* cp, T* ct) {
  T e1[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]}, e2[3] = {c[0] - a[0], c[1] - a[1], c[2] - a[2]}, n[3];
  cross3(n, e1, e2);
  T d[3] = {p1[0] - p0[0], p1[1] - p0[1], p1[2] - p0[2]};
  const T den = dot3(n, d);
  if (fabs(den) > T(1e-30)) {
    T ap[3] = {a[0] - p0[0], a[1] - p0[1], a[2] - p0[2]};
    const T t = dot3(n, ap) / den;
    if (t >= 0 && t <= 1) {
      T x[3] = {p0[0] + t * d[0], p0[1] + t * d[1], p0[2] + t * d[2]}, q[3];
      closest_pt_tri(q, x, a, b, c);
      T dd[3] = {x[0] - q[0], x[1] - q[1], x[2] - q[2]};
      if (dot3(dd, dd) < T(1e-28)) {
#pragma unroll
        for (int i = 0; i < 3; i++) { cp[i] = x[i]; ct[i] = x[i]; }
        return 0;
      }
    }
  }
  T best = T(1e30), q[3], x1[3], x2[3];
  const T* ends[2] = {p0, p1};
#pragma unroll
  for (int k = 0; k < 2; k++) {
    closest_pt_tri(q, ends[k], a, b, c);
    T dd[3] = {ends[k][0] - q[0], ends[k][1] - q[1], ends[k][2] - q[2]};
    const T dist = sqrt(dot3(dd, dd));
    if (dist < best) {
      best = dist;
#pragma unroll
      for (int i = 0; i < 3; i++) { cp[i] = ends[k][i]; ct[i] = q[i]; }
    }
  }
  const T* E[3][2] = {{a, b}, {b, c}, {c, a}};
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const T dist = seg_seg(p0, p1, E[k][0], E[k][1], x1, x2);
    if (dist < best) {
      best = dist;
#pragma unroll
      for (int i = 0; i < 3; i++) { cp[i] = x1[i]; ct[i] = x2[i]; }
    }
  }
  return best;
}

template <typename T>
BB_HD void seg_ends(const Seg<T>& g, T* p0, T* p1) {
#pragma unroll
  for (int i = 0; i < 3; i++) { p0[i] = g.c[i] - g.hh * g.a[i]; p1[i] = g.c[i] + g.hh * g.a[i]; }
}

template <typename T>
BB_HD void prism_centroid(const PrismG<T>& P, T* cen) {
  cen[0] = cen[1] = cen[2] = 0;
#pragma unroll
  for (int v = 0; v < 6; v++)
#pragma unroll
    for (int i = 0; i < 3; i++) cen[i] += P.V[v][i] * T(1.0 / 6);
}

// capsule_prism when the axis segment misses the prism: the separation
// distance and closest pair.  The closest pair is an endpoint and a face
// interior point (the endpoint in front of the face, its projection inside
// every other face plane), or a point of the segment and one of the 9 prism
// edges: the minimum over the 8 boundary triangles (the oracle's seg_tri
// loop) from 9 segment pairs and 10 projections instead of 16 point-triangle
// and 24 segment pairs.
template <typename T>
BB_HD inline bool capsule_prism_apart(const Seg<T>& g, const PrismG<T>& P, const T* p0, const T* p1, T& dist, T* n,
                                      T* pos) {
  T best2 = T(1e30), bp[3] = {0, 0, 0}, bq[3] = {0, 0, 0};
  T h0[5], h1[5];
#pragma unroll
  for (int f = 0; f < 5; f++) { h0[f] = dot3(P.pn[f], p0) - P.pd[f]; h1[f] = dot3(P.pn[f], p1) - P.pd[f]; }
#pragma unroll
  for (int f = 0; f < 5; f++) {
#pragma unroll
    for (int k = 0; k < 2; k++) {
      const T* x = k ? p1 : p0;
      const T hf = k ? h1[f] : h0[f];
      bool inside = hf > 0;
#pragma unroll
      for (int g2 = 0; g2 < 5; g2++)
        if (g2 != f) inside = inside && (k ? h1[g2] : h0[g2]) - hf * dot3(P.pn[g2], P.pn[f]) <= T(1e-12);
      if (inside && hf * hf < best2) {
        best2 = hf * hf;
#pragma unroll
        for (int i = 0; i < 3; i++) { bp[i] = x[i]; bq[i] = x[i] - hf * P.pn[f][i]; }
      }
    }
  }
  const int E[9][2] = {{0, 1}, {1, 2}, {2, 0}, {3, 4}, {4, 5}, {5, 3}, {0, 3}, {1, 4}, {2, 5}};
  // the bottom edges (3-5) are at least the segment's height above the prism's bottom away: when
  // that is >= r they cannot make a contact, and when a contact exists they are not the closest
  // feature -- skipping them changes no result (a capsule near the surface is far above it)
  const bool bottom = minT(p0[2], p1[2]) - P.V[3][2] < g.r;
#pragma unroll
  for (int e = 0; e < 9; e++) {
    if (e >= 3 && e <= 5 && !bottom) continue;
    T cp[3], cq[3];
    const T d2 = seg_seg2(p0, p1, P.V[E[e][0]], P.V[E[e][1]], cp, cq);
    if (d2 < best2) {
      best2 = d2;
#pragma unroll
      for (int i = 0; i < 3; i++) { bp[i] = cp[i]; bq[i] = cq[i]; }
    }
  }
  const T best = sqrt(best2);
  if (best >= g.r) return false;
  if (best > T(1e-12)) {
    const T ib = T(1) / best;
#pragma unroll
    for (int i = 0; i < 3; i++) n[i] = (bp[i] - bq[i]) * ib;
  } else {
    n[0] = P.pn[0][0]; n[1] = P.pn[0][1]; n[2] = P.pn[0][2];
  }
  dist = best - g.r;
#pragma unroll
  for (int i = 0; i < 3; i++) pos[i] = bp[i] - n[i] * (g.r + dist * T(0.5));
  return true;
}

#ifdef __HIP_DEVICE_COMPILE__
// On the GPU capsule_prism_apart runs as a call: inlined into the base-tree
// collision it costs that code its registers (§6b).  The call takes its inputs
// by value -- the segment ends, the radius, the prism's top triangle and bottom
// -- and returns its outputs by value (14 dwords, in registers), so nothing
// goes through the stack: with the prism and the segment passed by reference
// every call wrote ~470 B per lane to scratch (the relief kernels' write
// traffic).  The prism is rebuilt from the same inputs by the same code, so it
// is bit for bit the caller's.  dist = 1e30 when there is no contact.
template <typename T>
struct ApartOut {
  T dist, n[3], pos[3];
};
template <typename T>
__attribute__((noinline)) __device__ ApartOut<T> capsule_prism_apart_call(T p00, T p01, T p02, T p10, T p11, T p12, T r,
                                                                          T v00, T v01, T v02, T v10, T v11, T v12,
                                                                          T v20, T v21, T v22, T zb) {
  const T Tp[3][3] = {{v00, v01, v02}, {v10, v11, v12}, {v20, v21, v22}};
  PrismG<T> P;
  prism_build(P, Tp, zb);
  Seg<T> g;  // capsule_prism_apart reads only the radius
  g.r = r;
  const T p0[3] = {p00, p01, p02}, p1[3] = {p10, p11, p12};
  ApartOut<T> o;
  T d = T(0);
  o.dist = capsule_prism_apart(g, P, p0, p1, d, o.n, o.pos) ? d : T(1e30);
  return o;
}
#endif

#ifdef BB_PHASE_CLOCKS
// (diagnostic) which way capsule_prism goes: 0 the face early-out, 1 the intersecting segment's
// SAT, 2 the separated segment's distance (capsule_prism_apart); the same tests, in its order
template <typename T>
BB_HD int capsule_prism_path(const Seg<T>& g, const PrismG<T>& P) {
  T p0[3], p1[3];
  seg_ends(g, p0, p1);
  T dir[3] = {p1[0] - p0[0], p1[1] - p0[1], p1[2] - p0[2]};
  for (int f = 0; f < 5; f++) {
    const T d0 = dot3(P.pn[f], p0) - P.pd[f], d1 = dot3(P.pn[f], p1) - P.pd[f];
    if (d0 >= g.r && d1 >= g.r) return 0;
  }
  T t0 = 0, t1 = 1;
  bool inter = true;
  for (int f = 0; f < 5; f++) {
    const T a0 = dot3(P.pn[f], p0) - P.pd[f], ad = dot3(P.pn[f], dir);
    if (fabs(ad) < T(1e-30)) {
      if (a0 > 0) inter = false;
    } else {
      const T t = -a0 / ad;
      if (ad > 0) t1 = minT(t1, t); else t0 = maxT(t0, t);
    }
  }
  if (t0 > t1) inter = false;
  return inter ? 1 : 2;
}
#endif

// capsule vs prism; normal from prism to capsule.  Returns 1 on contact.
template <typename T>
BB_HD bool capsule_prism(const Seg<T>& g, const PrismG<T>& P, T& dist, T* n, T* pos) {
  T p0[3], p1[3];
  seg_ends(g, p0, p1);
  T dir[3] = {p1[0] - p0[0], p1[1] - p0[1], p1[2] - p0[2]};
  // separated by more than r along a face normal: no contact (cheap early out)
#pragma unroll
  for (int f = 0; f < 5; f++) {
    const T d0 = dot3(P.pn[f], p0) - P.pd[f], d1 = dot3(P.pn[f], p1) - P.pd[f];
    if (d0 >= g.r && d1 >= g.r) return false;
  }
  T t0 = 0, t1 = 1;
  bool inter = true;
#pragma unroll
  for (int f = 0; f < 5; f++) {
    const T a0 = dot3(P.pn[f], p0) - P.pd[f], ad = dot3(P.pn[f], dir);
    if (fabs(ad) < T(1e-30)) {
      if (a0 > 0) inter = false;
    } else {
      const T t = -a0 / ad;
      if (ad > 0) t1 = minT(t1, t); else t0 = maxT(t0, t);
    }
  }
  if (t0 > t1) inter = false;
  if (!inter) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(BB_CAPSULE_INLINE)
#ifdef BB_EXP_DUP_APART  // timing experiment (tools/lib_bench): the separated-segment distance twice
    {
      const ApartOut<T> o2 = capsule_prism_apart_call(p0[0], p0[1], p0[2], p1[0], p1[1], p1[2], g.r, P.V[0][0],
                                                      P.V[0][1], P.V[0][2], P.V[1][0], P.V[1][1], P.V[1][2],
                                                      P.V[2][0], P.V[2][1], P.V[2][2], P.V[3][2]);
      asm volatile("" :: "v"(o2.dist), "v"(o2.n[0]), "v"(o2.pos[0]) : "memory");
    }
#endif
    const ApartOut<T> o = capsule_prism_apart_call(p0[0], p0[1], p0[2], p1[0], p1[1], p1[2], g.r, P.V[0][0], P.V[0][1],
                                                   P.V[0][2], P.V[1][0], P.V[1][1], P.V[1][2], P.V[2][0], P.V[2][1],
                                                   P.V[2][2], P.V[3][2]);
    if (o.dist == T(1e30)) return false;  // (a NaN distance is a contact, as in capsule_prism_apart)
    dist = o.dist;
#pragma unroll
    for (int i = 0; i < 3; i++) { n[i] = o.n[i]; pos[i] = o.pos[i]; }
    return true;
#else
    return capsule_prism_apart(g, P, p0, p1, dist, n, pos);
#endif
  }
  // intersecting: minimum over the separating-axis candidates
  T bestd = T(1e30), bn[3] = {0, 0, 1};
  // both signs of an axis from one set of dot products: support(-a) =
  // -min(a.V), min(-a.p) = -max(a.p) (negation is exact: same values as
  // evaluating -a directly)
  auto test = [&](const T* ax) {
    T mx, mn;
    prism_extent(P, ax, mx, mn);
    const T e0 = dot3(ax, p0), e1 = dot3(ax, p1);
    const T dp = mx - minT(e0, e1), dm = -mn + maxT(e0, e1);
    if (dp < bestd) { bestd = dp; bn[0] = ax[0]; bn[1] = ax[1]; bn[2] = ax[2]; }
    if (dm < bestd) { bestd = dm; bn[0] = -ax[0]; bn[1] = -ax[1]; bn[2] = -ax[2]; }
  };
#pragma unroll
  for (int f = 0; f < 5; f++) test(P.pn[f]);
#pragma unroll
  for (int k = 0; k < 4; k++) {
    T e[3] = {0, 0, 1};
    if (k > 0) { const int i = k - 1, j = k % 3; e[0] = P.V[j][0] - P.V[i][0]; e[1] = P.V[j][1] - P.V[i][1]; e[2] = P.V[j][2] - P.V[i][2]; }
    T x[3];
    cross3(x, dir, e);
    const T xl = sqrt(dot3(x, x));
    if (xl > T(1e-12) * (sqrt(dot3(dir, dir)) * sqrt(dot3(e, e)) + T(1e-30))) {
      x[0] /= xl; x[1] /= xl; x[2] /= xl;
      test(x);
    }
  }
  n[0] = bn[0]; n[1] = bn[1]; n[2] = bn[2];
  dist = -bestd - g.r;
  const T e0 = dot3(n, p0), e1 = dot3(n, p1);
  T xd[3];
  if (fabs(e0 - e1) < T(1e-12)) {
    T cen[3];
    prism_centroid(P, cen);
    const T dd = dot3(dir, dir);
    T cp0[3] = {cen[0] - p0[0], cen[1] - p0[1], cen[2] - p0[2]};
    const T t = clampT(dd > 0 ? dot3(cp0, dir) / dd : T(0), t0, t1);
#pragma unroll
    for (int i = 0; i < 3; i++) xd[i] = p0[i] + t * dir[i];
  } else {
#pragma unroll
    for (int i = 0; i < 3; i++) xd[i] = e0 < e1 ? p0[i] : p1[i];
  }
#pragma unroll
  for (int i = 0; i < 3; i++) pos[i] = xd[i] - n[i] * (g.r + dist * T(0.5));
  return true;
}

template <typename T>
BB_HD T cyl_support(const Seg<T>& g, const T* n) {
  const T na = dot3(n, g.a);
  const T rad = T(1) - na * na;
  return dot3(n, g.c) + g.hh * fabs(na) + g.r * sqrt(rad > 0 ? rad : T(0));
}

// cylinder vs prism; normal from prism to cylinder.  Returns 1 on contact.
template <typename T>
BB_HD bool cylinder_prism(const Seg<T>& g, const PrismG<T>& P, T& dist, T* n, T* pos) {
  T bestd = T(1e30), bn[3] = {0, 0, 1};
  bool sep = false;
  // both signs of an axis from one set of dot products (see capsule_prism):
  // cyl_support(-a) = -a.c + hh |a.u| + r sqrt(1 - (a.u)^2)
  auto test = [&](const T* ax) {
    T mx, mn;
    prism_extent(P, ax, mx, mn);
    const T na = dot3(ax, g.a);
    const T rad = T(1) - na * na;
    const T sr = sqrt(rad > 0 ? rad : T(0));
    const T ac = dot3(ax, g.c);
    const T csm = -ac + g.hh * fabs(na) + g.r * sr, csp = ac + g.hh * fabs(na) + g.r * sr;  // cyl_support(-a), (a)
    const T dp = mx + csm, dm = -mn + csp;
    if (dp <= 0) sep = true;
    if (dp < bestd) { bestd = dp; bn[0] = ax[0]; bn[1] = ax[1]; bn[2] = ax[2]; }
    if (dm <= 0) sep = true;
    if (dm < bestd) { bestd = dm; bn[0] = -ax[0]; bn[1] = -ax[1]; bn[2] = -ax[2]; }
  };
  // a separating axis decides the result (no contact) whatever the later axes give: leave at
  // the first group that finds one (the face normals, most often the top face's, for a tower
  // above the terrain), so most non-touching candidates skip the other eleven axes
  test(P.pn[0]);  // the top face first: it separates most non-touching candidates by itself
  if (sep) return false;
#pragma unroll
  for (int f = 1; f < 5; f++) test(P.pn[f]);
  test(g.a);
  if (sep) return false;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    T e[3] = {0, 0, 1};
    if (k > 0) { const int i = k - 1, j = k % 3; e[0] = P.V[j][0] - P.V[i][0]; e[1] = P.V[j][1] - P.V[i][1]; e[2] = P.V[j][2] - P.V[i][2]; }
    T x[3];
    cross3(x, g.a, e);
    const T xl = sqrt(dot3(x, x));
    if (xl > T(1e-12) * (sqrt(dot3(e, e)) + T(1e-30))) { x[0] /= xl; x[1] /= xl; x[2] /= xl; test(x); }
  }
  if (sep) return false;
#pragma unroll
  for (int v = 0; v < 6; v++) {
    T d[3] = {P.V[v][0] - g.c[0], P.V[v][1] - g.c[1], P.V[v][2] - g.c[2]};
    const T t = dot3(d, g.a);
    T x[3] = {d[0] - t * g.a[0], d[1] - t * g.a[1], d[2] - t * g.a[2]};
    const T xl = sqrt(dot3(x, x));
    if (xl > T(1e-12)) { x[0] /= xl; x[1] /= xl; x[2] /= xl; test(x); }
  }
  if (sep) return false;
  n[0] = bn[0]; n[1] = bn[1]; n[2] = bn[2];
  dist = -bestd;
  // deepest cylinder point along -n (degenerate sets: nearest the prism centroid)
  T cen[3], dc[3];
  prism_centroid(P, cen);
  dc[0] = cen[0] - g.c[0]; dc[1] = cen[1] - g.c[1]; dc[2] = cen[2] - g.c[2];
  const T na2 = dot3(n, g.a);
  T rad[3] = {n[0] - na2 * g.a[0], n[1] - na2 * g.a[1], n[2] - na2 * g.a[2]};
  const T rl = sqrt(dot3(rad, rad));
  const T along = fabs(na2) > T(1e-9) ? (na2 > 0 ? -g.hh : g.hh) : clampT(dot3(dc, g.a), -g.hh, g.hh);
  T sp[3] = {g.c[0] + along * g.a[0], g.c[1] + along * g.a[1], g.c[2] + along * g.a[2]};
  if (rl > T(1e-9)) {
#pragma unroll
    for (int k = 0; k < 3; k++) sp[k] -= g.r * rad[k] / rl;
  } else {
    const T t = dot3(dc, g.a);
    T pr[3] = {dc[0] - t * g.a[0], dc[1] - t * g.a[1], dc[2] - t * g.a[2]};
    const T pl = sqrt(dot3(pr, pr));
    const T sc = pl > g.r ? g.r / pl : T(1);
#pragma unroll
    for (int k = 0; k < 3; k++) sp[k] += pr[k] * sc;
  }
#pragma unroll
  for (int k = 0; k < 3; k++) pos[k] = sp[k] - n[k] * (dist * T(0.5));
  return true;
}

#if defined(__HIP_DEVICE_COMPILE__) && defined(BB_EXP_DUP_CYL)
// timing experiment: cylinder_prism from scalars, as a call (bb_team16.h BB_EXP_DUP_CYL)
template <typename T>
__attribute__((noinline)) __device__ T cylinder_prism_dup_call(T c0, T c1, T c2, T a0, T a1, T a2, T hh, T r, T v00,
                                                             T v01, T v02, T v10, T v11, T v12, T v20, T v21, T v22,
                                                             T zb) {
  const T Tp[3][3] = {{v00, v01, v02}, {v10, v11, v12}, {v20, v21, v22}};
  PrismG<T> P;
  prism_build(P, Tp, zb);
  Seg<T> g;
  g.c[0] = c0; g.c[1] = c1; g.c[2] = c2; g.a[0] = a0; g.a[1] = a1; g.a[2] = a2; g.hh = hh; g.r = r;
  T d = 0, n[3], pos[3];
  return cylinder_prism(g, P, d, n, pos) ? d : T(1e30);
}
#endif

// sphere (geom1) vs cylinder (geom2); normal from sphere to cylinder
template <typename T>
BB_HD bool sphere_cylinder(const T* c, T r, const Seg<T>& g, T& dist, T* n, T* pos) {
  T d[3] = {c[0] - g.c[0], c[1] - g.c[1], c[2] - g.c[2]};
  const T z = dot3(d, g.a);
  T rv[3] = {d[0] - z * g.a[0], d[1] - z * g.a[1], d[2] - z * g.a[2]};
  const T rho = sqrt(dot3(rv, rv));
  T u[3] = {0, 0, 0};
  if (rho > T(1e-12)) { u[0] = rv[0] / rho; u[1] = rv[1] / rho; u[2] = rv[2] / rho; }
  const bool inside = fabs(z) <= g.hh && rho <= g.r;
  if (!inside) {
    const T zc = clampT(z, -g.hh, g.hh), rc = minT(rho, g.r);
    T q[3] = {g.c[0] + zc * g.a[0] + rc * u[0], g.c[1] + zc * g.a[1] + rc * u[1], g.c[2] + zc * g.a[2] + rc * u[2]};
    T dq[3] = {q[0] - c[0], q[1] - c[1], q[2] - c[2]};
    const T dd = sqrt(dot3(dq, dq));
    if (dd >= r) return false;
    dist = dd - r;
    if (dd > T(1e-12)) { n[0] = dq[0] / dd; n[1] = dq[1] / dd; n[2] = dq[2] / dd; }
    else { n[0] = g.a[0]; n[1] = g.a[1]; n[2] = g.a[2]; }
  } else {
    const T ds = g.r - rho, dcap = g.hh - fabs(z);
    if (ds < dcap) {
      n[0] = -u[0]; n[1] = -u[1]; n[2] = -u[2];
      dist = -ds - r;
    } else {
      const T sg = z >= 0 ? T(1) : T(-1);
      n[0] = -sg * g.a[0]; n[1] = -sg * g.a[1]; n[2] = -sg * g.a[2];
      dist = -dcap - r;
    }
  }
#pragma unroll
  for (int k = 0; k < 3; k++) pos[k] = c[k] + n[k] * (r + dist * T(0.5));
  return true;
}

// sphere (geom1) vs capsule (geom2): mjraw_SphereCapsule; normal sphere -> capsule
template <typename T>
BB_HD bool sphere_capsule(const T* c, T r, const Seg<T>& g, T& dist, T* n, T* pos) {
  T p0[3], p1[3], cp[3], cq[3];
  seg_ends(g, p0, p1);
  const T d = seg_seg(c, c, p0, p1, cp, cq);
  dist = d - r - g.r;
  if (dist > 0) return false;
  if (d > 0) { n[0] = (cq[0] - c[0]) / d; n[1] = (cq[1] - c[1]) / d; n[2] = (cq[2] - c[2]) / d; }
  else { n[0] = 1; n[1] = 0; n[2] = 0; }
#pragma unroll
  for (int k = 0; k < 3; k++) pos[k] = c[k] + n[k] * (r + dist * T(0.5));
  return true;
}

// World poses of the base-tree geoms: 0 tower (cylinder), 1-2 cam sticks,
// 3-5 wheels (capsules); body ids 1, 2, 3, 4, 5, 6.
template <typename T>
BB_HD void body_geom(const ModelT<T>& m, const Kin<T>& k, int gidx, Seg<T>& g) {
  T t[3];
  if (gidx == 0) {
    mv3(t, k.Rb, m.tower_c);
    g.c[0] = k.pb[0] + t[0]; g.c[1] = k.pb[1] + t[1]; g.c[2] = k.pb[2] + t[2];
    g.a[0] = k.Rb[2]; g.a[1] = k.Rb[5]; g.a[2] = k.Rb[8];
    g.hh = m.tower_hh; g.r = m.tower_r;
  } else if (gidx <= 2) {
    const int s = gidx - 1;
    mv3(t, k.Rb, m.stick_c[s]);
    g.c[0] = k.pb[0] + t[0]; g.c[1] = k.pb[1] + t[1]; g.c[2] = k.pb[2] + t[2];
    mv3(g.a, k.Rb, m.stick_a[s]);
    g.hh = m.stick_hh; g.r = m.stick_r;
  } else {
    const int w = gidx - 3;
    mv3(t, k.Rb, k.wc[w]);
    g.c[0] = k.pb[0] + t[0]; g.c[1] = k.pb[1] + t[1]; g.c[2] = k.pb[2] + t[2];
    T al[3];
    mv3(al, k.Rw[w], m.gz);
    mv3(g.a, k.Rb, al);
    g.hh = m.wheel_hh; g.r = m.wheel_r;
  }
}

}  // namespace bb
