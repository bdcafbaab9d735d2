// bb_pairmap.h -- which workgroup of the one-launch relief pair (relief_pair1_kernel,
// bb_kernels.hip) runs which loop.  Host and device: tests/hostcheck checks the map.
#pragma once
#include <hip/hip_runtime.h>

namespace bb {

constexpr int NXCD = 8;  // XCDs of an MI355X; the dispatcher deals workgroup b to XCD b % 8

// Block b of the one-launch pair -> its kind (0 fast, 1 full; -1: idle) and its index among
// that kind's workgroups.  Whole groups of NXCD consecutive blocks share a kind, one block per
// XCD label (b % NXCD); group 0 is fast, group 1 full, and the remaining groups are dealt to the
// kinds in proportion (centred Bresenham).  So every prefix of the grid that the dispatcher seats holds
// both kinds on every label, and the launch makes progress even when the chip is shared and
// only part of the grid is resident (the rest then finds every env done and exits).  nf and ns
// are multiples of NXCD with at least one group each (bb_create, pair_adapt_kernel).
__host__ __device__ inline int pair_kind_of(int b, int nf, int ns, int* wg) {
  const int Gs = ns / NXCD, G = nf / NXCD + Gs, g = b / NXCD, x = b % NXCD;
  if (g >= G) return -1;
  int kind, idx;
  if (g < 2) {
    kind = g;
    idx = 0;
  } else {
    const int R = G - 2, S = Gs - 1, gp = g - 2;
    // full groups among the first x of the rest: floor(x S / R + 1/2) (Bresenham, centred)
    const int lo = int((2LL * gp * S + R) / (2LL * R)), hi = int((2LL * (gp + 1) * S + R) / (2LL * R));
    kind = hi > lo ? 1 : 0;
    idx = kind ? 1 + lo : 1 + gp - lo;
  }
  *wg = idx * NXCD + x;
  return kind;
}

}  // namespace bb
