// bb_pair.hip -- the relief pair's kernels and launch (bb_step_multi on relief
// banks) as their own translation unit: bb_kernels.hip compiled
// with BB_PAIR_TU (everything but the C-ABI) and, in the build,
// -mllvm -disable-machine-licm (see bb_pair_launch_tu in bb_kernels.hip).
#define BB_PAIR_TU
#include "bb_kernels.hip"
