// bb_kernels.hip -- gfx950 kernels and the C-ABI boundary (include/ballbot_mi355x.h).
//
// Layout in HBM (per handle, n envs, T = float or double):
//   qpos  T[17][n]   qvel T[15][n]   warm T[15][n]     SoA: lane e reads
//   steps int[n]     terrain int[n]  episodes int[n]   element i at [i*n + e]
//   bank  float[n_terrains][293*293], size_z float[nt], offset float[nt]
// One env per TEAM of L lanes (L = 16 by default: 4 envs per 64-lane wave,
// one wave per workgroup, 4096 envs -> 1024 waves = one per SIMD).  Each team
// owns an EnvWork (bb_solve.h) in LDS holding the mass blocks, contact
// Jacobians, ground-contact store, Hessian/Cholesky factor and phase-local
// scratch; the constraint solve is team-parallel, the per-env state is
// replicated in the team's registers and stored by the team's lane 0.
//
// FMA contraction per source expression only (a * b + c written as one
// expression): the backend's contraction of separate multiplies and adds
// depends on the inlining context, so two kernels inlining the same step
// (bb_step's, bb_step_multi's, the relief pair's, the rollout's) could round
// differently.  With contraction fixed by the source, every kernel computes
// each env's step bit for bit the same.
#if defined(BB_FP_CONTRACT_OFF)  // variant builds (tools/lib_bench.py): no contraction at all
#pragma clang fp contract(off)
#elif !defined(BB_FP_CONTRACT_FAST)  // ... or the compiler default (fast, backend-decided)
#pragma clang fp contract(on)
#endif
#include <hip/hip_runtime.h>

#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <climits>
#include <vector>

#include "../../include/ballbot_mi355x.h"
#include "bb_model.h"
#include "bb_step.h"
#include "bb_terrain.h"
#include "bb_rollout.h"
#include "bb_render.h"
#include "bb_ppo.h"
#include "bb_mlp.h"
#include "bb_encoder.h"
#include "bb_pairmap.h"

using namespace bb;

#ifdef BB_PHASE_CLOCKS
// (in bb_pair.hip the name is bb_phase_cycles_pair, renamed there: not read back)
namespace bb { __device__ unsigned long long bb_phase_cycles[100]; }
#endif

namespace {

constexpr int WAVE = 64;
constexpr int TEAM = 16;  // lanes per env == one DPP row
char g_err[512] = "";

int fail(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
  return -1;
}
#define HIPCHK(x)                                                                   \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) return fail("%s: %s", #x, hipGetErrorString(e_));         \
  } while (0)

// per-team EnvWork stride in LDS (16-byte aligned)
template <typename T>
__host__ __device__ constexpr size_t work_stride() { return (sizeof(EnvWork<T>) + 15) / 16 * 16; }
template <typename T>
size_t lds_bytes(int epw) { return work_stride<T>() * epw; }
template <typename T>
__device__ __forceinline__ EnvWork<T>& team_work(unsigned char* smem, int team) {
  return *reinterpret_cast<EnvWork<T>*>(smem + size_t(team) * work_stride<T>());
}

// the terrain-draw configuration (Dev.tsrc; one per handle, in device memory)
struct TerrainSrc {
  const int* tstream;         // [n_streams][tlen] bank slot of draw k (bb_set_terrain_stream); NULL: none
  const int* env_stream;      // [n] stream of each env; NULL: stream 0
  int tlen;
  unsigned long long* rng;    // [5][n] per-env PCG64 (bb_set_terrain_rng): state hi/lo, inc hi/lo, 32-bit buffer
  const int* seed_slot;       // [TERRAIN_SEEDS] bank slot holding each terrain seed (-1: not resident); NULL: slot == seed
};

struct Dev {
  int n;
  void* qpos;
  void* qvel;
  void* warm;
  int* steps;
  int* terrain;
  int* pending_terrain;       // >= 0: terrain pinned by bb_assign_terrain; < 0: draw from the stream
  int* episodes;              // terrain-stream draws made by each env so far
  // Where a reset's terrain comes from: a device record that bb_set_terrain_rng /
  // bb_set_terrain_stream rewrite in place.  Dev is captured by value in HIP graphs, so it holds
  // only this record's address, which never changes: a graph captured before a re-seed draws
  // from the new generators (or the new table) at replay.
  const struct TerrainSrc* tsrc;
  int* tseed;                 // [n] terrain seed of each env's last device draw (-1: none)
  const float* bank;
  const float* size_z;
  const float* offset;
  const float* hmax;  // per terrain: max(hfield) (the top height is hmax * size_z)
  int n_terrains;
  unsigned long long* stats;  // resets, diverged, overflow, slow-path env-steps, iters, draws past the stream table, spill
  int* slow_list;             // envs the fast kernel handed to the full kernel this step
  int* slow_count;            // [0] fast list size, [1] predicted-slow list size, [2] hand-overs
  int* park;                  // bb_step_multi (two launches): the step each env was parked at, K when done
  int* fast_envs;             // this step's fast-kernel env list (ascending)
  int* pred_envs;             // envs predicted to need base-tree contacts (full kernel, concurrent)
  uint8_t* pred_mark;
  void* body_spill;           // T[n][MAXB - MAXB_LDS][NBF]: base-tree contacts past the LDS slots
  void* hand;                 // relief pair: T[n][HAND] env state between holds (qpos, qvel, warm, step), per env
  int* perm;                  // relief_multi_kernel: env of each workgroup slot (balance_kernel), NULL: identity
  unsigned long long* ring;   // relief pair: [NRINGS][ring_len] ticket rings of envs ready for a step (pair_ring)
  int* rctr;                  // relief pair: [NRINGS][2] ring head / tail
  int ring_len;               // an XCD's envs + its resident teams: an entry is never overwritten before it is taken
  unsigned long long* pair_env;  // relief_pair_kernel, last launch, per env: [n] cycles stepped, [n] wall tick of its last step
  unsigned long long* pair_busy;  // relief_pair_kernel, last launch: [2] team-cycles stepping, [2] team lifetimes
                                  // in shader cycles, [2] in wall-clock ticks (fast, full)
  unsigned long long* cost;   // relief_multi_kernel: shader cycles each env's steps took in the last launch
  int* fault;                 // host-mapped sticky error word (bb_check): a relief-pair launch hit its budget
};

// env e's spill block for base-tree contacts MAXB_LDS..MAXB-1
template <typename T>
__device__ __forceinline__ T* body_spill_of(const Dev& d, int e) {
  return reinterpret_cast<T*>(d.body_spill) + size_t(e) * ((MAXB - MAXB_LDS) * NBF);
}

// Device-coherent (agent-scope) loads and stores: `sc1` accesses, which the
// per-XCD L2s do not serve stale nor hold dirty.  Data that moves between
// workgroups on different XCDs inside one launch (the relief pair's env
// hand-over) goes through these instead of __threadfence(), which on gfx950 is
// buffer_wbl2 + buffer_inv of the WHOLE L2 of the XCD: every hand-over then
// cost every wave on that XCD its cached lines (kernel code included).
template <typename V>
__device__ __forceinline__ V ld_coh(const V* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename V>
__device__ __forceinline__ void st_coh(V* p, V v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// the wave's earlier stores complete (device-coherent ones are then visible to
// every XCD) before its later memory operations: the release of a hand-over
// whose data went through st_coh
__device__ __forceinline__ void stores_done() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// COH: through ld_coh / st_coh (the relief pair's hand-over)
template <typename T, bool COH = false>
__device__ __forceinline__ void load_state(const Dev& d, int e, T* q, T* v, T* w, int& step) {
  const T* Q = (const T*)d.qpos;
  const T* V = (const T*)d.qvel;
  const T* W = (const T*)d.warm;
  if constexpr (COH) {
#pragma unroll
    for (int i = 0; i < NQ; i++) q[i] = ld_coh(Q + i * d.n + e);
#pragma unroll
    for (int i = 0; i < NV; i++) { v[i] = ld_coh(V + i * d.n + e); w[i] = ld_coh(W + i * d.n + e); }
    step = ld_coh(d.steps + e);
  } else {
#pragma unroll
    for (int i = 0; i < NQ; i++) q[i] = Q[i * d.n + e];
#pragma unroll
    for (int i = 0; i < NV; i++) { v[i] = V[i * d.n + e]; w[i] = W[i * d.n + e]; }
    step = d.steps[e];
  }
}
template <typename T, bool COH = false>
__device__ __forceinline__ void store_state(const Dev& d, int e, const T* q, const T* v, const T* w, int step) {
  // e opaque here: otherwise the 47 per-element addresses of load_state are
  // kept live (94 VGPRs) across the whole step and spill to scratch
  asm volatile("" : "+v"(e));
  T* Q = (T*)d.qpos;
  T* V = (T*)d.qvel;
  T* W = (T*)d.warm;
  if constexpr (COH) {
#pragma unroll
    for (int i = 0; i < NQ; i++) st_coh(Q + i * d.n + e, q[i]);
#pragma unroll
    for (int i = 0; i < NV; i++) { st_coh(V + i * d.n + e, v[i]); st_coh(W + i * d.n + e, w[i]); }
    st_coh(d.steps + e, step);
  } else {
#pragma unroll
    for (int i = 0; i < NQ; i++) Q[i * d.n + e] = q[i];
#pragma unroll
    for (int i = 0; i < NV; i++) { V[i * d.n + e] = v[i]; W[i * d.n + e] = w[i]; }
    d.steps[e] = step;
  }
}

// numpy's PCG64 (the bit generator of gymnasium's np_random, Generator(PCG64(
// SeedSequence(seed)))): a 128-bit LCG, state = state * M + inc, output
// XSL-RR of the new state.  Generator.integers(0, 10000) takes 32-bit draws
// (the bit generator buffers the high half of each 64-bit output for the next
// one) through Lemire's bounded multiply with rejection.  Integer work,
// bit-exact against numpy (tests/test_host_config.py restates it on the host,
// tests/test_gpu_terrain_stream.py checks the device draws).
struct Pcg64 {
  unsigned long long sh, sl, ih, il, buf;  // state, increment (hi, lo); buf: bit 32 = has_uint32, low 32 = uinteger
};
constexpr int TERRAIN_SEEDS = 10000;  // ballbot_env.py:505-510 integers(0, 10000)

__device__ __forceinline__ unsigned long long pcg64_next64(Pcg64& g) {
  constexpr unsigned long long MH = 0x2360ED051FC65DA4ull, ML = 0x4385DF649FCCF645ull;
  const unsigned long long lo = g.sl * ML;
  unsigned long long hi = __umul64hi(g.sl, ML) + g.sl * MH + g.sh * ML;
  const unsigned long long lo2 = lo + g.il;
  hi += g.ih + (lo2 < lo ? 1ull : 0ull);
  g.sl = lo2;
  g.sh = hi;
  const unsigned rot = unsigned(hi >> 58);
  const unsigned long long x = hi ^ lo2;
  return (x >> rot) | (x << ((64u - rot) & 63u));
}
__device__ __forceinline__ unsigned pcg64_next32(Pcg64& g) {
  if (g.buf >> 32) {  // the buffered half; numpy clears has_uint32 and keeps the value
    const unsigned u = unsigned(g.buf);
    g.buf = u;
    return u;
  }
  const unsigned long long x = pcg64_next64(g);
  g.buf = (1ull << 32) | (x >> 32);
  return unsigned(x);
}
// Generator.integers(0, 10000): buffered_bounded_lemire_uint32 with rng = 9999
__device__ __forceinline__ int pcg64_terrain_seed(Pcg64& g) {
  constexpr unsigned EXCL = TERRAIN_SEEDS;
  unsigned long long m = (unsigned long long)pcg64_next32(g) * EXCL;
  unsigned left = unsigned(m);
  if (left < EXCL) {
    constexpr unsigned THRESHOLD = (0xFFFFFFFFu - (EXCL - 1u)) % EXCL;
    while (left < THRESHOLD) {
      m = (unsigned long long)pcg64_next32(g) * EXCL;
      left = unsigned(m);
    }
  }
  return int(m >> 32);
}

// The terrain of env e's next episode.  The reference draws
// r_seed = _np_random.integers(0, 10000) at every reset (ballbot_env.py:505-510)
// from the env's own generator: SB3 seeds training env i with reset(seed=seed+i)
// (VecEnv.seed, then the first reset of learn(); gymnasium's Env.reset(seed)
// replaces _np_random, :596), an eval env keeps np_random(seed + N_ENVS + i) from
// construction (:378-384, train.py:90-97).  With bb_set_terrain_rng each env runs
// that generator here (unbounded, exact); the drawn seed's bank slot comes from
// seed_slot (a draw whose seed is not resident is counted in stats[5] and takes
// slot seed % n_terrains).  Otherwise the host's precomputed draws per stream
// (bb_set_terrain_stream): draw episodes[e] of the table.  A pinned terrain
// (bb_assign_terrain) takes no draw.  Called by one lane per env.  The env's
// generator and counters go through ld_coh / st_coh: in the relief pair the
// env's next reset may run on another XCD within the same launch.
__device__ __forceinline__ int next_terrain(const Dev& d, int e) {
  const int pin = d.pending_terrain[e];
  if (pin >= 0) return pin;
  const TerrainSrc src = *d.tsrc;
  if (src.rng) {
    const size_t n = size_t(d.n);
    unsigned long long* rng = src.rng;
    Pcg64 g{ld_coh(rng + e), ld_coh(rng + n + e), ld_coh(rng + 2 * n + e), ld_coh(rng + 3 * n + e),
            ld_coh(rng + 4 * n + e)};
    const int s = pcg64_terrain_seed(g);
    st_coh(rng + e, g.sh); st_coh(rng + n + e, g.sl); st_coh(rng + 4 * n + e, g.buf);
    st_coh(d.episodes + e, ld_coh(d.episodes + e) + 1);
    st_coh(d.tseed + e, s);
    int slot = src.seed_slot ? src.seed_slot[s] : s;
    if (unsigned(slot) >= unsigned(d.n_terrains)) {
      atomicAdd(&d.stats[5], 1ull);
      slot = s % d.n_terrains;
    }
    return slot;
  }
  if (!src.tstream) return 0;
  int k = ld_coh(d.episodes + e);
  st_coh(d.episodes + e, k + 1);
  if (k >= src.tlen) {  // past the resident draws: reuse them (counted)
    atomicAdd(&d.stats[5], 1ull);
    k %= src.tlen;
  }
  const int st = src.env_stream ? src.env_stream[e] : 0;
  return src.tstream[size_t(st) * src.tlen + k];
}

template <typename T>
__device__ __forceinline__ void reset_lane(const ModelT<T>& m, const Dev& d, int e, T* q, T* v, T* w, int& step) {
  const int tid = next_terrain(d, e);
  d.terrain[e] = tid;
  reset_state(m, T(d.offset[tid]), q, v, w);
  step = 0;
}

// BODY = false: the fast kernel (no base-tree contact support compiled in;
// envs that may touch a base-tree geom are appended to d.slow_list and left
// untouched).  BODY = true: the full kernel over d.slow_list.
template <typename T, bool BODY>
__global__ __launch_bounds__(64) void step_kernel(ModelT<T> mg, EnvCfg cfg, Dev d, const float* __restrict__ act,
                                                  float* __restrict__ obs, float* __restrict__ rew,
                                                  uint8_t* __restrict__ done, float* __restrict__ tobs,
                                                  float* __restrict__ pos2d, int auto_reset, int L, int epw,
                                                  const int* __restrict__ elist, const int* __restrict__ ecount) {
  // epw teams of L lanes per 64-lane wave (teams >= epw idle)
  extern __shared__ __align__(16) unsigned char smem[];
  // list launches are sized for every env; workgroups past the list end leave
  // before touching LDS (on flat terrain the full-kernel lists are empty)
  // XCD-aware workgroup order: the dispatcher deals workgroups round-robin over
  // the 8 XCDs (workgroup b runs on XCD b % 8), so give each XCD a contiguous
  // range of env groups.  A 128-B line of SoA state holds 16 fp64 envs, i.e.
  // four 4-env workgroups: in launch order those sat on four XCDs and the line
  // was fetched into four L2s.  Any permutation is exact (envs are independent).
  // List launches are sized for every env but only the first na = ceil(count /
  // epw) workgroups have work: the permutation is taken over those (rounded up
  // to a multiple of 8), so the active groups spread over all eight XCDs
  // instead of piling onto the first few.
  const int nwg = int(gridDim.x), b = int(blockIdx.x);
  int g;
  // list launches: the count is clamped to the list's size (n), so a count that
  // was not reset cannot send a workgroup past the list
  const int ecnt = elist ? min(*ecount, d.n) : 0;
  if (elist) {
    const int na = (ecnt + epw - 1) / epw, nb = (na + 7) & ~7;
    if (nb > nwg) {
      g = b;  // too few workgroups in the grid for the rounded-up permutation
    } else {
      if (b >= nb) return;
      g = (b & 7) * (nb >> 3) + (b >> 3);
    }
    if (g >= na) return;
  } else {
    g = (nwg & 7) ? b : (b & 7) * (nwg >> 3) + (b >> 3);
  }
  // model constants staged in LDS once per workgroup: uniform-address LDS
  // reads broadcast, and ~150 uniform doubles no longer overflow the SGPRs
  __shared__ ModelT<T> ms;
  if (threadIdx.x == 0) ms = mg;
  __syncthreads();
  const ModelT<T>& m = ms;
  const Team tm{L, int(threadIdx.x) & (L - 1)};
  const int team = threadIdx.x / L;
  if (team >= epw) return;
  int e = g * epw + team;
  if (elist) {  // env list of this launch (ascending env ids)
    if (e >= ecnt) return;
    e = elist[e];
  }
  if (unsigned(e) >= unsigned(d.n)) return;
  const bool lead = tm.tl == 0;
#ifdef BB_PHASE_CLOCKS
  const unsigned long long t_env0 = clock64();
#endif
  EnvWork<T>& W = team_work<T>(smem, team);
#ifdef BB_PHASE_CLOCKS
  if (lead) W.dbg_nb = 0;
#endif
  if (BODY && lead) W.bspill = body_spill_of<T>(d, e);  // read after the forward's first team_sync
  // the env state lives in the team's workspace (every lane writes the same
  // values): 47 values held in registers across four solves would spill
  T* q = W.qn;
  T* v = W.vn;
  T* w = W.wn;
  int step;
  load_state(d, e, q, v, w, step);
  float a[3] = {act[3 * e], act[3 * e + 1], act[3 * e + 2]};
  const int tid = d.terrain[e];
  const float* hf = d.bank + size_t(tid) * (HF_N * HF_N);
  float o[15], r, p2[2];
  int iters = 0;
  const TerrainRef<T> tr{hf, T(d.size_z[tid]), T(d.hmax[tid]) * T(d.size_z[tid])};
  int fl = env_step<T, BODY>(m, cfg, q, v, w, step, a, tr, W, o, r, p2, &iters, tm);
  if (!BODY && (fl & F_SLOWPATH)) {
    if (lead) {
      const int at = atomicAdd(d.slow_count + 2, 1);
      if (at < d.n) d.slow_list[at] = e;  // never past the list, whatever the count holds
    }
    return;
  }
  if (!lead) return;
  if (BODY) atomicAdd(&d.stats[3], 1ull);  // env-steps through the full kernel
  if (tobs) {
#pragma unroll
    for (int i = 0; i < 15; i++) tobs[15 * e + i] = o[i];
  }
  if (pos2d) { pos2d[2 * e] = p2[0]; pos2d[2 * e + 1] = p2[1]; }
  // SB3 VecEnv auto-reset of a terminated episode; a MuJoCo divergence reset
  // (F_DIVERGED) already happened inside the step and ends nothing
  const bool reset = auto_reset && (fl & F_TERMINATED);
  if (reset) {
    reset_lane(m, d, e, q, v, w, step);
#pragma unroll
    for (int i = 0; i < 15; i++) o[i] = 0.f;  // reset obs: identity quat, zero velocities, zero action
  }
#pragma unroll
  for (int i = 0; i < 15; i++) obs[15 * e + i] = o[i];
  rew[e] = r;
  done[e] = uint8_t(fl);
  store_state(d, e, q, v, w, step);
  // counters (wave-aggregated by the compiler)
  if (reset) atomicAdd(&d.stats[0], 1ull);
  if (fl & F_DIVERGED) atomicAdd(&d.stats[1], 1ull);
  if (fl & F_OVERFLOW) atomicAdd(&d.stats[2], 1ull);
  if (fl & F_SPILL) atomicAdd(&d.stats[6], 1ull);
  atomicAdd(&d.stats[4], (unsigned long long)iters);
#ifdef BB_PHASE_CLOCKS
  {  // per-env step duration: max, sum and count per kernel (full 34-36, fast 37-39)
    const unsigned long long dt = clock64() - t_env0;
    atomicMax(&bb_phase_cycles[BODY ? 34 : 37], dt);
    atomicAdd(&bb_phase_cycles[BODY ? 35 : 38], dt);
    atomicAdd(&bb_phase_cycles[BODY ? 36 : 39], 1ull);
    // full kernel: step-duration histogram (bins of 2^20 cycles) with the base-tree
    // contacts and Newton iterations of the envs in each bin
    if (BODY) {
      const int bin = int(dt >> 20) < 9 ? int(dt >> 20) : 9;
      atomicAdd(&bb_phase_cycles[40 + bin], 1ull);
      atomicAdd(&bb_phase_cycles[50 + bin], (unsigned long long)W.dbg_nb);
      atomicAdd(&bb_phase_cycles[60 + bin], (unsigned long long)iters);
      atomicMax(&bb_phase_cycles[70 + bin], (unsigned long long)W.dbg_nb);
    }
  }
#endif
}

// The full env step of multi_step_kernel's hand-overs.  Inlined (BB_MULTI_MODE
// 1): as a separate function (0) the call costs the fast path its registers
// (512 VGPRs + 2.4 KB scratch; 6.33 M against 7.91 M env-steps/s at 4096 flat
// fp64, 16 steps per launch).  2: full step for every env, 3: no hand-over
// (timing variants only: 3 is wrong when a hand-over occurs).
#ifndef BB_MULTI_MODE
#define BB_MULTI_MODE 1
#endif
template <typename T>
__device__
#if BB_MULTI_MODE == 0
__noinline__
#else
__forceinline__
#endif
int full_env_step(const ModelT<T>& m, const EnvCfg& cfg, T* q, T* v, T* w, int& step,
                                          const float* a, const TerrainRef<T>& tr, EnvWork<T>& W, float* o,
                                          float& r, float* p2, int* iters, const Team& tm) {
  return env_step<T, true>(m, cfg, q, v, w, step, a, tr, W, o, r, p2, iters, tm);
}

// One env step of a team inside a multi-step launch (multi_step_kernel,
// rollout_kernel): the fast path first; an env it hands over (F_SLOWPATH: a
// base-tree geom may touch the terrain) is restored from the team's LDS copy
// bk of the step's start state and takes the full step inline.  Auto-reset,
// terrain draw and counters as step_kernel.  tobs_row / p2_row (may be NULL):
// this step's terminal obs and pos2d.  On return o holds the obs after any
// reset; the flags are the step's.  full: the predictor routed the env to the
// full step (relief_multi_kernel): the fast path is not tried.
// HO = false (multi_step_kernel's first launch): the full step is not compiled
// in; an env the fast path hands over is restored to the step's start state
// and F_PARKED returned, without counting the attempt -- the finish launch
// redoes that step through the hand-over and counts it there.
constexpr int F_PARKED = 1 << 17;  // internal: never in a done byte

// bb_step_multi on relief banks, adaptive form (slow_count slots): SC_ROUTE holds
// the next launch's form (0: the work queue, ROUTE_PARK: the parked multi-step
// launches), SC_TOUCHED counts the envs of the last launch that needed a full step
constexpr int SC_ROUTE = 8, SC_TOUCHED = 10, ROUTE_PARK = 1;

// stores of the step's output rows (obs, reward, done, terminal obs, pos2d): -DBB_OUT_NT makes
// them nontemporal, -DBB_OUT_SKIP=mask drops some of them in the relief pair (1 obs, 2 reward,
// 4 done, 8 terminal obs, 16 pos2d): diagnostics of the pair's output write-backs,
// never in the product build
#ifndef BB_OUT_SKIP
#define BB_OUT_SKIP 0
#endif
template <typename V>
__device__ __forceinline__ void out_st(V* p, V v) {
#ifdef BB_OUT_NT
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}

template <typename T, bool HO = true, bool FULLONLY = false>
__device__ __forceinline__ int team_step(const ModelT<T>& m, const EnvCfg& cfg, const Dev& d, int e, int& tid,
                                         T* q, T* v, T* w, int& step, T* bk, const float* a, EnvWork<T>& W, float* o,
                                         float& r, float* tobs_row, float* p2_row, int auto_reset, const Team& tm,
                                         unsigned* cnt, bool full = false) {
  // FULLONLY (relief_pair_kernel<T, true>): the full step only -- the fast path is
  // not compiled in, so the launch keeps the full step's registers
  const int L = tm.L;
  const bool lead = tm.tl == 0;
  if constexpr (!FULLONLY) {
    team_sync();
    for (int i = tm.tl; i < NQ + 2 * NV; i += L) bk[i] = q[i];
    team_sync();
  }
  const float* hf = d.bank + size_t(tid) * (HF_N * HF_N);
  float p2[2];
  int iters = 0;
  const TerrainRef<T> tr{hf, T(d.size_z[tid]), T(d.hmax[tid]) * T(d.size_z[tid])};
  const int step0 = step;
  int fl;
#if BB_MULTI_MODE == 2
  fl = F_SLOWPATH;
#else
  if constexpr (FULLONLY) fl = F_SLOWPATH;
  else fl = full ? F_SLOWPATH : env_step<T, false>(m, cfg, q, v, w, step, a, tr, W, o, r, p2, &iters, tm);
#endif
  const bool slow = (fl & F_SLOWPATH) != 0;  // team-uniform
#if BB_MULTI_MODE == 3
  if (false) {
#else
  if (slow) {
#endif
    if constexpr (!FULLONLY) {
      team_sync();
      for (int i = tm.tl; i < NQ + 2 * NV; i += L) q[i] = bk[i];
      team_sync();
      step = step0;
    }
    if constexpr (!HO) return F_PARKED;
    else fl = full_env_step<T>(m, cfg, q, v, w, step, a, tr, W, o, r, p2, &iters, tm);
  }
  const bool reset = auto_reset && (fl & F_TERMINATED);
  if (lead) {
    cnt[3] += slow;
    if (tobs_row && !(BB_OUT_SKIP & 8)) {
#pragma unroll
      for (int i = 0; i < 15; i++) out_st(tobs_row + i, o[i]);
    }
    if (p2_row && !(BB_OUT_SKIP & 16)) { out_st(p2_row, p2[0]); out_st(p2_row + 1, p2[1]); }
    if (reset) {
      tid = next_terrain(d, e);
      st_coh(d.terrain + e, tid);
    }
  }
  if (reset) {
    tid = __shfl(tid, team_shift_of(L));  // the lead's draw
    team_sync();
    reset_state(m, T(d.offset[tid]), q, v, w);  // every lane writes the same values
    step = 0;
#pragma unroll
    for (int i = 0; i < 15; i++) o[i] = 0.f;
  }
  if (lead) {
    cnt[0] += reset;
    cnt[1] += (fl & F_DIVERGED) != 0;
    cnt[2] += (fl & F_OVERFLOW) != 0;
    cnt[6] += (fl & F_SPILL) != 0;
    cnt[4] += unsigned(iters);
  }
  return fl;
}

// A multi-step launch's counters: team_step adds to the team's (or env slot's)
// LDS row cnt[8] (indices as Dev::stats; 5, the stream wraps, is counted in
// next_terrain), and the row goes to d.stats once at the end of the launch --
// not one same-address device atomic per env-step, whose completion every
// later vector-memory wait of the step would also wait for.
__device__ __forceinline__ void counts_clear(unsigned* cnt) {
#pragma unroll
  for (int i = 0; i < 8; i++) cnt[i] = 0u;
}
__device__ __forceinline__ void counts_flush(const Dev& d, const unsigned* cnt) {
#pragma unroll
  for (int i = 0; i < 8; i++)
    if (i != 5 && cnt[i]) atomicAdd(&d.stats[i], (unsigned long long)cnt[i]);
}

// K env steps of every env in one launch (bb_step_multi): actions [K][n][3]
// known in advance (open-loop: benchmarks, replayed action sequences).  Each
// team steps its env K times back to back (team_step); no env waits for the
// slowest env of the chip at every step, only for the slowest of its wave.
// Per step k the outputs, counters, auto-reset and terrain draws are exactly
// those of the k-th bb_step call under the serial route.
//
// Two launches (park != NULL): HO = false steps every env until done or until
// the fast path hands a step over (a base-tree geom may touch the terrain);
// that env is parked at its step k (park[e] = k, K when done) with the step's
// start state stored.  HO = true then resumes the parked envs from park[e]
// with the full step inline and exits at once for the others.  The first
// launch carries no full step, so it keeps the fast kernel's registers: the
// full step inlined beside it costs 157-196 spilled VGPRs (scratch traffic on
// every step, hand-over or not).  park == NULL: one launch, hand-overs inline.
// variant builds (tools/lib_bench.py): tell the compiler a SIMD holds one wave of the kernel
// (4096 envs fill the chip at one wave per SIMD whatever the registers), so that it schedules
// for latency instead of an occupancy it cannot reach
#ifdef BB_WPE1
#define BB_WPE __attribute__((amdgpu_waves_per_eu(1, 1)))
#else
#define BB_WPE
#endif
template <typename T, bool HO>
__global__ BB_WPE __launch_bounds__(64) void multi_step_kernel(ModelT<T> mg, EnvCfg cfg, Dev d, const float* __restrict__ act,
                                                        int K, float* __restrict__ obs, float* __restrict__ rew,
                                                        uint8_t* __restrict__ done, float* __restrict__ tobs,
                                                        float* __restrict__ pos2d, int auto_reset, int L, int epw,
                                                        int* __restrict__ park, const int* __restrict__ gate) {
  // gate (relief banks, adaptive form): run only when the device flag selects the
  // parked launches (ROUTE_PARK); workgroup-uniform, before any barrier
  if (gate && *gate != ROUTE_PARK) return;
  extern __shared__ __align__(16) unsigned char smem[];
  const int nwg = int(gridDim.x), b = int(blockIdx.x);
  const int g = (nwg & 7) ? b : (b & 7) * (nwg >> 3) + (b >> 3);  // XCD-aware order, as step_kernel
  __shared__ ModelT<T> ms;
  if (threadIdx.x == 0) ms = mg;
  __syncthreads();
  const ModelT<T>& m = ms;
  const Team tm{L, int(threadIdx.x) & (L - 1)};
  const int team = threadIdx.x / L;
  if (team >= epw) return;
  const int e = g * epw + team;
  if (unsigned(e) >= unsigned(d.n)) return;
  int k0 = 0;
  if (HO && park) {  // the finish launch: only parked envs, from their parked step
    k0 = park[e];
    if (k0 >= K) return;  // team-uniform
  }
  const bool lead = tm.tl == 0;
  EnvWork<T>& W = team_work<T>(smem, team);
  // the step's start state (qn, vn, wn are contiguous: 47 values), for a hand-over
  T* bk = reinterpret_cast<T*>(smem + size_t(epw) * work_stride<T>()) + team * (NQ + 2 * NV);
  __shared__ unsigned s_cnt[WAVE / TEAM][8];
  unsigned* cnt = s_cnt[team];
  if (lead) {
    W.bspill = body_spill_of<T>(d, e);
    counts_clear(cnt);
  }
  T* q = W.qn;
  T* v = W.vn;
  T* w = W.wn;
  int step;
  load_state(d, e, q, v, w, step);
  int tid = d.terrain[e];
  const size_t n = size_t(d.n);
  int parked = K;
#pragma unroll 1
  for (int k = k0; k < K; k++) {
    const size_t row = size_t(k) * n + e;
    const float* ak = act + 3 * row;
    const float a[3] = {ak[0], ak[1], ak[2]};
    float o[15], r;
    const int fl = team_step<T, HO>(m, cfg, d, e, tid, q, v, w, step, bk, a, W, o, r, tobs ? tobs + 15 * row : nullptr,
                                    pos2d ? pos2d + 2 * row : nullptr, auto_reset, tm, cnt);
    if (!HO && (fl & F_PARKED)) {  // team-uniform
      parked = k;
      break;
    }
    if (lead) {
#pragma unroll
      for (int i = 0; i < 15; i++) obs[15 * row + i] = o[i];
      rew[row] = r;
      done[row] = uint8_t(fl);
    }
  }
  team_sync();
  if (lead) {
    store_state(d, e, q, v, w, step);
    counts_flush(d, cnt);
    if (!HO) park[e] = parked;
    if (!HO && gate && parked < K) atomicAdd(d.slow_count + SC_TOUCHED, 1);  // adaptive: an env that needed a full step
  }
}

// The rollout's policy step for one env on its team: SB3
// ActorCriticPolicy.forward of the reference's proprio MLP (pi = vf = 4 x 128
// LeakyReLU trunks over the 15 sorted-key obs; mean = action_net(h_pi), value =
// value_net(h_vf)), fp32.  The trunk weights come INPUT-major (W^T: [in][128],
// bb_rollout_args), so for each input k the team's 16 lanes read one
// contiguous 512-B row slice: lane tl owns units 4 tl + c and 64 + 4 tl + c
// (c < 4) as two float4s, and every fetched cache line is used whole (the
// output-major rows cost 4x the L2 traffic: 16 lines per load, 16 B used of
// each).  Each unit is a k-ordered fmaf chain from the layer input in LDS.
// (bb_ppo_mlp_act's MFMA tiles sum in another order: the two agree to fp32
// rounding, tests/test_gpu_rollout.py.)
__device__ __forceinline__ float leaky_f(float z) { return z > 0.f ? z : z * 0.01f; }
__device__ __forceinline__ void team_policy(const float* __restrict__ P, const int* __restrict__ off, const float* x,
                                            float* hA, float* hB, const Team& tm, float mu[3], float& val) {
  constexpr int HIDN = 128, IN = 15;
  const int u0 = 4 * tm.tl;  // this lane's units: u0 + c, 64 + u0 + c
#pragma unroll 1
  for (int tr = 0; tr < 2; tr++) {
    const int wb = tr ? MLP_VF_W0 : MLP_PI_W0, bb_ = tr ? MLP_VF_B0 : MLP_PI_B0;
    float* hin = hA;
    float* hout = hB;
#pragma unroll 1
    for (int l = 0; l < 4; l++) {
      const float* WT = P + off[wb + l];  // [K][128]
      const float* bl = P + off[bb_ + l];
      const float* in = l ? hin : x;
      const int K = l ? HIDN : IN;
      float4 a0 = *reinterpret_cast<const float4*>(bl + u0);
      float4 a1 = *reinterpret_cast<const float4*>(bl + 64 + u0);
#ifdef BB_POLICY_UNROLL
#pragma unroll BB_POLICY_UNROLL
#else
#pragma unroll 8
#endif
      for (int k = 0; k < K; k++) {
        const float hk = in[k];
        const float4 w0 = *reinterpret_cast<const float4*>(WT + k * HIDN + u0);
        const float4 w1 = *reinterpret_cast<const float4*>(WT + k * HIDN + 64 + u0);
        a0.x = fmaf(hk, w0.x, a0.x); a0.y = fmaf(hk, w0.y, a0.y);
        a0.z = fmaf(hk, w0.z, a0.z); a0.w = fmaf(hk, w0.w, a0.w);
        a1.x = fmaf(hk, w1.x, a1.x); a1.y = fmaf(hk, w1.y, a1.y);
        a1.z = fmaf(hk, w1.z, a1.z); a1.w = fmaf(hk, w1.w, a1.w);
      }
      float* out = l ? hout : hin;  // layer 0 writes hA; later layers alternate
      *reinterpret_cast<float4*>(out + u0) = make_float4(leaky_f(a0.x), leaky_f(a0.y), leaky_f(a0.z), leaky_f(a0.w));
      *reinterpret_cast<float4*>(out + 64 + u0) =
          make_float4(leaky_f(a1.x), leaky_f(a1.y), leaky_f(a1.z), leaky_f(a1.w));
      team_sync();
      if (l) { float* t_ = hin; hin = hout; hout = t_; }
    }
    // heads on h4 (hin, output-major Wa/Wv): lane partial sums over its 8 units, then the team sum
    const float4 h0 = *reinterpret_cast<const float4*>(hin + u0);
    const float4 h1 = *reinterpret_cast<const float4*>(hin + 64 + u0);
    auto dot8 = [&](const float* w) {
      const float4 w0 = *reinterpret_cast<const float4*>(w + u0);
      const float4 w1 = *reinterpret_cast<const float4*>(w + 64 + u0);
      float s = 0.f;
      s = fmaf(h0.x, w0.x, s); s = fmaf(h0.y, w0.y, s); s = fmaf(h0.z, w0.z, s); s = fmaf(h0.w, w0.w, s);
      s = fmaf(h1.x, w1.x, s); s = fmaf(h1.y, w1.y, s); s = fmaf(h1.z, w1.z, s); s = fmaf(h1.w, w1.w, s);
      return s;
    };
    if (tr == 0) {
      const float* Wa = P + off[MLP_WA];
#pragma unroll
      for (int c = 0; c < 3; c++) mu[c] = team_sum(tm, dot8(Wa + c * HIDN)) + P[off[MLP_BA] + c];
    } else {
      val = team_sum(tm, dot8(P + off[MLP_WV])) + P[off[MLP_BV]];
    }
    team_sync();
  }
}

struct RolloutDev {
  const float* P;
  int off[MLP_NSLOTS];
  const float* noise;      // [T][n][3]
  int T;
  float* obs;              // [n][15] in/out
  uint8_t* last_starts;    // [n] in/out
  double* ep_ret;          // [n] in/out
  long long* ep_len;       // [n] in/out
  float* b_obs;            // [T][n][15]
  float* b_act;            // [T][n][3]
  float* b_val;            // [T][n]
  float* b_logp;           // [T][n]
  float* b_rew;            // [T][n]
  uint8_t* b_starts;       // [T][n]
  double* ep_r;            // [T][n]
  long long* ep_l;         // [T][n]
};

// One whole PPO rollout (SB3 OnPolicyAlgorithm.collect_rollouts + Monitor) in
// ONE launch (bb_rollout): every env runs its T steps of (policy, sample,
// clip, env step, bookkeeping) back to back on its team -- the policy's
// parameters are fixed during a rollout, and envs are independent, so no step
// needs a grid-wide barrier.  Per step the rollout buffer gets the obs, the
// unclipped action, value, log-probability, reward and episode start; finished
// episodes their (float64 return, length).  The step itself is team_step
// (fast path, inline full-step hand-over, auto-reset).
// Two launches (park != NULL), as multi_step_kernel: HO = false parks an env
// at the step the fast path hands over (its state, observation and episode
// counters as before that step; the policy rows it wrote are rewritten
// identically), and HO = true resumes the parked envs from park[e] -- the
// policy is fixed during a rollout, so an env's remaining steps need nothing
// from the other envs.
template <typename T, bool HO>
__global__ __launch_bounds__(64) void rollout_kernel(ModelT<T> mg, EnvCfg cfg, Dev d, RolloutDev ro, int L, int epw,
                                                     int* __restrict__ park) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int nwg = int(gridDim.x), b = int(blockIdx.x);
  const int g = (nwg & 7) ? b : (b & 7) * (nwg >> 3) + (b >> 3);
  __shared__ ModelT<T> ms;
  if (threadIdx.x == 0) ms = mg;
  __syncthreads();
  const ModelT<T>& m = ms;
  const Team tm{L, int(threadIdx.x) & (L - 1)};
  const int team = threadIdx.x / L;
  if (team >= epw) return;
  const int e = g * epw + team;
  if (unsigned(e) >= unsigned(d.n)) return;
  int t0 = 0;
  if (HO && park) {  // the finish launch: only parked envs, from their parked step
    t0 = park[e];
    if (t0 >= ro.T) return;  // team-uniform
  }
  const bool lead = tm.tl == 0;
  EnvWork<T>& W = team_work<T>(smem, team);
  T* bk = reinterpret_cast<T*>(smem + size_t(epw) * work_stride<T>()) + team * (NQ + 2 * NV);
  // policy scratch x[16], hA[128], hB[128] in the team's contact stores (g, then
  // bc): they only hold data inside a step.  (A separate LDS block pushed a
  // workgroup past 40 KB: 3 instead of 4 workgroups per CU, a quarter of the
  // waves in a second round.)
  static_assert(offsetof(EnvWork<T>, bc) == offsetof(EnvWork<T>, g) + sizeof(W.g) &&
                    sizeof(W.g) + sizeof(W.bc) >= 272 * sizeof(float),
                "policy scratch must fit in EnvWork::g + bc");
  float* pol = reinterpret_cast<float*>(W.g);
  float* x = pol;
  float* hA = pol + 16;
  float* hB = pol + 144;
  __shared__ unsigned s_cnt[WAVE / TEAM][8];
  unsigned* cnt = s_cnt[team];
  if (lead) {
    W.bspill = body_spill_of<T>(d, e);
    counts_clear(cnt);
  }
  T* q = W.qn;
  T* v = W.vn;
  T* w = W.wn;
  int step;
  load_state(d, e, q, v, w, step);
  int tid = d.terrain[e];
  const size_t n = size_t(d.n);
  float o[15];
#pragma unroll
  for (int i = 0; i < 15; i++) o[i] = ro.obs[15 * size_t(e) + i];
  uint8_t start = ro.last_starts[e];
  double ret = ro.ep_ret[e];
  long long len = ro.ep_len[e];
  const float* ls = ro.P + ro.off[MLP_LS];
  constexpr float HL2PI = 0.91893853320467274f;
  int parked = ro.T;
#pragma unroll 1
  for (int t = t0; t < ro.T; t++) {
    const size_t row = size_t(t) * n + e;
    team_sync();
    if (tm.tl < 15) x[tm.tl] = o[tm.tl];
    team_sync();
    float mu[3] = {0.f, 0.f, 0.f}, val = 0.f;
#ifndef BB_ROLLOUT_NO_POLICY
    team_policy(ro.P, ro.off, x, hA, hB, tm, mu, val);
#endif
    // SB3 DiagGaussian (bb_ppo_mlp_act's arithmetic): a = mean + eps * exp(log_std)
    float a[3], ac[3], lp = 0.f;
#pragma unroll
    for (int j = 0; j < 3; j++) {
      const float ls_j = ls[j];
      a[j] = __fadd_rn(mu[j], __fmul_rn(ro.noise[3 * row + j], expf(ls_j)));
      const float z = __fmul_rn(__fsub_rn(a[j], mu[j]), expf(-ls_j));
      lp += -0.5f * z * z - ls_j - 0.5f * (2.f * HL2PI);
      ac[j] = fminf(fmaxf(a[j], -1.f), 1.f);
    }
    if (lead) {
#pragma unroll
      for (int i = 0; i < 15; i++) ro.b_obs[15 * row + i] = o[i];
#pragma unroll
      for (int j = 0; j < 3; j++) ro.b_act[3 * row + j] = a[j];
      ro.b_val[row] = val;
      ro.b_logp[row] = lp;
      ro.b_starts[row] = start;
    }
    float r, o_prev[15];
    if (!HO) {
#pragma unroll
      for (int i = 0; i < 15; i++) o_prev[i] = o[i];
    }
    const int fl = team_step<T, HO>(m, cfg, d, e, tid, q, v, w, step, bk, ac, W, o, r, nullptr, nullptr, 1, tm, cnt);
    if (!HO && (fl & F_PARKED)) {  // team-uniform: the env resumes at step t in the finish launch
#pragma unroll
      for (int i = 0; i < 15; i++) o[i] = o_prev[i];
      parked = t;
      break;
    }
    // collect_rollouts + Monitor bookkeeping (bb_rollout_track): done = terminated
    const bool dn = (fl & F_TERMINATED) != 0;
    ret += double(r);
    len += 1;
    if (lead) {
      ro.b_rew[row] = r;
      ro.ep_r[row] = dn ? ret : __builtin_nan("");
      ro.ep_l[row] = dn ? len : 0;
    }
    ret = dn ? 0.0 : ret;
    len = dn ? 0 : len;
    start = dn ? 1 : 0;
  }
  team_sync();
  if (lead) {
    store_state(d, e, q, v, w, step);
    counts_flush(d, cnt);
    if (!HO) park[e] = parked;
#pragma unroll
    for (int i = 0; i < 15; i++) ro.obs[15 * size_t(e) + i] = o[i];
    ro.last_starts[e] = start;
    ro.ep_ret[e] = ret;
    ro.ep_len[e] = len;
  }
}

template <typename T>
__global__ __launch_bounds__(64) void reset_kernel(ModelT<T> m, Dev d, const uint8_t* mask, float* obs) {
  const int e = blockIdx.x * WAVE + threadIdx.x;
  // a full reset gives every env a valid state again: it clears the relief pair's sticky fault
  if (!mask && e == 0 && d.fault) __hip_atomic_store(d.fault, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (e >= d.n) return;
  if (mask && !mask[e]) return;
  T q[NQ], v[NV], w[NV];
  int step;
  reset_lane(m, d, e, q, v, w, step);
  store_state(d, e, q, v, w, step);
  if (obs) {
#pragma unroll
    for (int i = 0; i < 15; i++) obs[15 * e + i] = 0.f;
  }
}

template <typename T>
__global__ __launch_bounds__(64) void forward_kernel(ModelT<T> mg, Dev d, const double* ctrl, double* qacc, int* ncon,
                                                     int L, int epw) {
  extern __shared__ __align__(16) unsigned char smem[];
  __shared__ ModelT<T> ms;
  if (threadIdx.x == 0) ms = mg;
  __syncthreads();
  const ModelT<T>& m = ms;
  const Team tm{L, int(threadIdx.x) & (L - 1)};
  const int team = threadIdx.x / L;
  if (team >= epw) return;
  const int e = blockIdx.x * epw + team;
  if (e >= d.n) return;
  EnvWork<T>& W = team_work<T>(smem, team);
  if (tm.tl == 0) W.bspill = body_spill_of<T>(d, e);
  T q[NQ], v[NV], w[NV], c[3];
  int step;
  load_state(d, e, q, v, w, step);
  for (int i = 0; i < 3; i++) c[i] = T(ctrl[3 * e + i]);
  const int tid = d.terrain[e];
  StageOut<T> so;
  const TerrainRef<T> tr{d.bank + size_t(tid) * (HF_N * HF_N), T(d.size_z[tid]), T(d.hmax[tid]) * T(d.size_z[tid])};
  forward<T, true>(m, q, v, c, w, tr, W, &so, tm);
  if (tm.tl != 0) return;
  for (int i = 0; i < NV; i++) qacc[NV * e + i] = double(w[i]);
  if (ncon) { ncon[2 * e] = so.ng; ncon[2 * e + 1] = so.nb; }
}

// The predictor's test for one env (a 16-lane team, lane tl; team_shift = the
// team's first lane in the wave): may a base-tree geom come within one step's
// reach of the ball or of a heightfield prism under it?  Team-uniform result.
template <typename T>
__device__ __forceinline__ bool predict_env(const ModelT<T>& m, const Dev& d, int tid, const T* Qe, const T* Ve,
                                            int tl, int team_shift) {
  constexpr int PL = 16;
  T pb[3], qb[4], pB[3], qB[4];
#pragma unroll
  for (int i = 0; i < 3; i++) { pb[i] = Qe[i]; pB[i] = Qe[10 + i]; }
#pragma unroll
  for (int i = 0; i < 4; i++) { qb[i] = Qe[3 + i]; qB[i] = Qe[13 + i]; }
  qnormalize(qb);
  qnormalize(qB);
  T Rb[9], RB[9];
  q2mat(Rb, qb);
  q2mat(RB, qB);
  T vb = 0, wb = 0;
#pragma unroll
  for (int i = 0; i < 3; i++) {
    const T a = Ve[i], b = Ve[3 + i];
    vb += a * a; wb += b * b;
  }
  // one step's reach of any geom point (|v| + 0.5 m |w|) h, x3, + 1 cm
  const T margin = T(3) * m.h * (sqrt(vb) + T(0.5) * sqrt(wb)) + T(0.01);
  const T cB[3] = {pB[0] + RB[2] * m.dz, pB[1] + RB[5] * m.dz, pB[2] + RB[8] * m.dz};  // ball centre
  const float* hf = d.bank + size_t(tid) * (HF_N * HF_N);
  const T size_z = T(d.size_z[tid]), hz = T(d.hmax[tid]) * size_z;
  bool slow = false;
  for (int gi = 0; gi < 6 && !slow; gi++) {
    // geom gi as a segment (base frame): tower axis, stick, wheel capsule
    // (axis = hinge axis; centre at zero hinge angle, +1 mm for its 0.3 mm offset)
    T cl[3], al[3], hh, gr;
    if (gi == 0) {
      cl[0] = m.tower_c[0]; cl[1] = m.tower_c[1]; cl[2] = m.tower_c[2];
      al[0] = 0; al[1] = 0; al[2] = 1;
      hh = m.tower_hh; gr = m.tower_r;
    } else if (gi <= 2) {
#pragma unroll
      for (int i = 0; i < 3; i++) { cl[i] = m.stick_c[gi - 1][i]; al[i] = m.stick_a[gi - 1][i]; }
      hh = m.stick_hh; gr = m.stick_r;
    } else {
      const int w = gi - 3;
      T R[9], t[3];
      q2mat(R, m.wq[w]);
      const T dd[3] = {m.cw[0] - m.jpos[0], m.cw[1] - m.jpos[1], m.cw[2] - m.jpos[2]};
      mv3(t, R, dd);
      cl[0] = m.anchor[0] + t[0]; cl[1] = m.anchor[1] + t[1]; cl[2] = m.anchor[2] + t[2];
      al[0] = m.u[w][0]; al[1] = m.u[w][1]; al[2] = m.u[w][2];
      hh = m.wheel_hh; gr = m.wheel_r + T(0.001);
    }
    T cw[3], aw[3];
    mv3(cw, Rb, cl);
    cw[0] += pb[0]; cw[1] += pb[1]; cw[2] += pb[2];
    mv3(aw, Rb, al);
    T p0[3], p1[3];
#pragma unroll
    for (int i = 0; i < 3; i++) { p0[i] = cw[i] - hh * aw[i]; p1[i] = cw[i] + hh * aw[i]; }
    if (gi == 0) {  // ball x tower: distance to the cylinder
      const T dd[3] = {cB[0] - cw[0], cB[1] - cw[1], cB[2] - cw[2]};
      const T z = dot3(dd, aw);
      const T rv[3] = {dd[0] - z * aw[0], dd[1] - z * aw[1], dd[2] - z * aw[2]};
      const T ez = maxT(fabs(z) - hh, T(0)), er = maxT(sqrt(dot3(rv, rv)) - gr, T(0));
      slow = sqrt(ez * ez + er * er) < m.ball_r + margin;
    } else if (gi < 3) {  // ball x sticks
      T cp[3], cq[3];
      slow = seg_seg(cB, cB, p0, p1, cp, cq) < m.ball_r + gr + margin;
    }
    // capsule-hull AABB of the geom, grown by the margin
    const T ext = gr + margin;
    const T lo = minT(p0[2], p1[2]) - ext;
    if (slow || !(lo <= hz)) continue;
    const T x0 = minT(p0[0], p1[0]) - ext, x1 = maxT(p0[0], p1[0]) + ext;
    const T y0 = minT(p0[1], p1[1]) - ext, y1 = maxT(p0[1], p1[1]) + ext;
    const T sx = m.hf_sx, sy = m.hf_sy;
    const int N1 = HF_N - 1;
    // written so that a NaN pose (a diverged state before mj_checkPos resets
    // it in the step) skips the geom: no cell index is formed from it
    if (!(x0 <= sx && x1 >= -sx && y0 <= sy && y1 >= -sy)) continue;
    int cmin = (int)floor((x0 + sx) / (2 * sx) * N1), cmax = (int)ceil((x1 + sx) / (2 * sx) * N1);
    int rmin = (int)floor((y0 + sy) / (2 * sy) * N1), rmax = (int)ceil((y1 + sy) / (2 * sy) * N1);
    cmin = cmin < 0 ? 0 : cmin; cmax = cmax > N1 ? N1 : cmax;
    rmin = rmin < 0 ? 0 : rmin; rmax = rmax > N1 ? N1 : rmax;
    // the kernels' prisms (cells [rmin, rmax) x [cmin, cmax)) that the grown
    // geom could reach this step (the same conservative test the kernels prune with)
    Seg<T> sg;
#pragma unroll
    for (int i = 0; i < 3; i++) { sg.c[i] = cw[i]; sg.a[i] = aw[i]; }
    sg.hh = hh;
    sg.r = ext;
    const T dx = 2 * sx / N1, dy = 2 * sy / N1;
#ifdef __HIP_DEVICE_COMPILE__
    t16::Reach<T> sr;
    t16::make_reach(sg, sr);
#endif
    const int nc = cmax - cmin, total = (rmax - rmin) * nc;
    bool hit = false;
    // cell i's four heights; the next cell's are loaded while this one is tested
    auto cellz = [&](int i, float (&z)[4]) {
      if (i < total) {
        const int r = rmin + i / nc, c = cmin + i % nc;
        z[0] = hf[r * HF_N + c]; z[1] = hf[(r + 1) * HF_N + c];
        z[2] = hf[r * HF_N + c + 1]; z[3] = hf[(r + 1) * HF_N + c + 1];
      }
    };
    float znext[4] = {0.f, 0.f, 0.f, 0.f};
    cellz(tl, znext);
    for (int i = tl; i < total && !hit; i += PL) {  // cell i of the sub-grid, row-major
      const float zc[4] = {znext[0], znext[1], znext[2], znext[3]};
      cellz(i + PL, znext);
      const int r = rmin + i / nc, c = cmin + i % nc;
      const T x0 = dx * c - sx, x1 = dx * (c + 1) - sx, y0 = dy * r - sy, y1 = dy * (r + 1) - sy;
      const T z00 = T(zc[0]) * size_z, z10 = T(zc[1]) * size_z;
      const T z01 = T(zc[2]) * size_z, z11 = T(zc[3]) * size_z;
      if (maxT(maxT(z00, z10), maxT(z01, z11)) < lo) continue;
      const T A[3][3] = {{x0, y0, z00}, {x0, y1, z10}, {x1, y0, z01}};
      const T B[3][3] = {{x0, y1, z10}, {x1, y0, z01}, {x1, y1, z11}};
#ifdef __HIP_DEVICE_COMPILE__
      hit = t16::prism_may_hit(sr, A) || t16::prism_may_hit(sr, B);
#else
      (void)A; (void)B; hit = true;  // host pass of the kernel: never run
#endif
    }
#ifdef __HIP_DEVICE_COMPILE__
    slow = ((__ballot(hit) >> team_shift) & 0xFFFFull) != 0;  // team-uniform
#else
    (void)team_shift; slow = hit;
#endif
  }
  return slow;
}

// Which envs should take the full kernel this step: a base-tree geom within a
// margin of the ball or of a heightfield vertex under it (the fast kernel's
// exact per-stage test stays the arbiter; this only routes work).  One
// 16-lane team per env (4 per wave): the per-geom setup is replicated, the
// cells under each geom's grown AABB are dealt over the lanes and the hits
// reduced with a ballot.  (One lane per env was 64 waves walking ~230 cells
// each: 93 us per step on perlin, on the critical path of the full kernel.)
template <typename T>
__global__ __launch_bounds__(64) void predict_kernel(ModelT<T> mg, Dev d) {
  __shared__ ModelT<T> ms;
  if (threadIdx.x == 0) ms = mg;
  __syncthreads();
  const ModelT<T>& m = ms;
  constexpr int PL = 16;
  const int tl = int(threadIdx.x) & (PL - 1), team_shift = team_shift_of(PL);
  const int e = blockIdx.x * (WAVE / PL) + int(threadIdx.x) / PL;
  if (e >= d.n) return;  // team-uniform
  const T* Q = (const T*)d.qpos;
  const T* V = (const T*)d.qvel;
  T Qe[NQ], Ve[6];
#pragma unroll
  for (int i = 0; i < NQ; i++) Qe[i] = Q[i * d.n + e];
#pragma unroll
  for (int i = 0; i < 6; i++) Ve[i] = V[i * d.n + e];
  const bool slow = predict_env<T>(m, d, d.terrain[e], Qe, Ve, tl, team_shift);
  if (tl == 0) d.pred_mark[e] = slow ? 1 : 0;
}

// K steps of every env in one launch on relief banks (bb_step_multi, route 0):
// a work queue inside each workgroup.  A workgroup of QW waves owns QENV envs
// (their EnvWork in its LDS).  Each wave repeatedly claims up to 4 envs whose
// next step is due and that the predictor routes the same way -- all fast or
// all full -- and steps them, so a wave never runs the fast and the full
// step one after the other for different teams (the divergence that costs
// multi_step_kernel its gain on relief).  Per env the result is route 0's:
// predicted envs take the full step, the others the fast path with the
// hand-over.  The claims are under an LDS spin lock held by one lane of the
// claiming wave; a workgroup ends when its QENV x K env-steps are done, which
// every wave observes.
constexpr int QW = 4, QENV = 4 * QW;

// RO: the whole PPO rollout (bb_rollout) instead of open-loop steps: each
// claimed env runs one (policy, sample, clip, step, bookkeeping) step as
// rollout_kernel does; its observation and episode counters wait in LDS
// between claims.
template <typename T, bool RO>
__global__ __launch_bounds__(64 * QW) void relief_multi_kernel(ModelT<T> mg, EnvCfg cfg, Dev d,
                                                               const float* __restrict__ act, int K,
                                                               float* __restrict__ obs, float* __restrict__ rew,
                                                               uint8_t* __restrict__ done, float* __restrict__ tobs,
                                                               float* __restrict__ pos2d, int auto_reset, RolloutDev ro,
                                                               const int* __restrict__ gate) {
  if (gate && *gate == ROUTE_PARK) return;  // adaptive form: the parked launches run instead
  extern __shared__ __align__(16) unsigned char smem[];
  __shared__ ModelT<T> ms;
  __shared__ int s_k[QENV], s_busy[QENV], s_kind[QENV], s_tid[QENV], s_step[QENV], s_env[QENV];
  __shared__ int s_claim[QW][4], s_fin[QW];
  __shared__ int s_lock, s_left;
  __shared__ unsigned s_cnt[QENV][8];  // per env slot (team_step's counters)
  // RO: per env the observation, episode start and Monitor counters between claims
  __shared__ float s_obs[RO ? QENV : 1][15];
  __shared__ int s_start[RO ? QENV : 1];
  __shared__ double s_ret[RO ? QENV : 1];
  __shared__ long long s_len[RO ? QENV : 1];
  const int nwg = int(gridDim.x), b = int(blockIdx.x);
  const int g = (nwg & 7) ? b : (b & 7) * (nwg >> 3) + (b >> 3);
  const int e0 = g * QENV;
  const int nloc = min(QENV, d.n - e0);
  if (nloc <= 0) return;  // workgroup-uniform
  const int wave = int(threadIdx.x) >> 6, lane = int(threadIdx.x) & 63;
  const Team tm{16, lane & 15};
  const int team = lane >> 4;
  const bool lead = tm.tl == 0;
  const size_t n = size_t(d.n);
  T* bk0 = reinterpret_cast<T*>(smem + size_t(QENV) * work_stride<T>());
  if (threadIdx.x == 0) {
    ms = mg;
    s_lock = 0;
    s_left = nloc * K;
  }
  if (int(threadIdx.x) < nloc) {
    const int i = int(threadIdx.x), e = d.perm ? d.perm[e0 + i] : e0 + i;
    EnvWork<T>& W = team_work<T>(smem, i);
    int step;
    load_state(d, e, W.qn, W.vn, W.wn, step);
    W.bspill = body_spill_of<T>(d, e);
    s_env[i] = e;
    counts_clear(s_cnt[i]);
    s_k[i] = 0;
    s_busy[i] = 0;
    s_tid[i] = d.terrain[e];
    s_step[i] = step;
    if (RO) {
#pragma unroll
      for (int j = 0; j < 15; j++) s_obs[i][j] = ro.obs[15 * size_t(e) + j];
      s_start[i] = ro.last_starts[e];
      s_ret[i] = ro.ep_ret[e];
      s_len[i] = ro.ep_len[e];
    }
  }
  __syncthreads();
  const ModelT<T>& m = ms;
  {  // the first step's routes: wave w predicts envs 4w .. 4w + 3
    const int i = 4 * wave + team;
    if (i < nloc) {
      EnvWork<T>& W = team_work<T>(smem, i);
      const bool sl = predict_env<T>(m, d, s_tid[i], W.qn, W.vn, tm.tl, team_shift_of(16));
      if (lead) s_kind[i] = sl ? 1 : 0;
    }
  }
  __syncthreads();
#pragma unroll 1
  for (;;) {
    if (lane == 0) {
      while (atomicCAS(&s_lock, 0, 1) != 0) __builtin_amdgcn_s_sleep(1);
      int nf = 0, ns = 0;
      for (int i = 0; i < nloc; i++)
        if (!s_busy[i] && s_k[i] < K) (s_kind[i] ? ns : nf)++;
      // full steps first when a whole wave of them is due (they are the long
      // ones), else whole waves of fast steps, else the larger group
      const int kind = ns >= 4 ? 1 : (nf >= 4 ? 0 : (ns >= nf ? 1 : 0));
      int c = 0;
      for (int i = 0; i < nloc && c < 4; i++)
        if (!s_busy[i] && s_k[i] < K && s_kind[i] == kind) { s_busy[i] = 1; s_claim[wave][c++] = i; }
      for (; c < 4; c++) s_claim[wave][c] = -1;
      s_fin[wave] = s_left == 0;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      atomicExch(&s_lock, 0);
    }
    team_sync();  // the wave's lanes see lane 0's claims
    if (s_fin[wave]) break;
    const int i = s_claim[wave][team];
    if (s_claim[wave][0] < 0) {  // nothing due that is not being stepped (wave-uniform)
      __builtin_amdgcn_s_sleep(2);
      continue;
    }
    if (i >= 0) {
      EnvWork<T>& W = team_work<T>(smem, i);
      T* bk = bk0 + i * (NQ + 2 * NV);
      const int e = s_env[i], k = s_k[i];
      const size_t row = size_t(k) * n + e;
      int tid = s_tid[i], step = s_step[i];
      const bool full = s_kind[i] != 0;
      const unsigned long long c0 = clock64();
      float a[3], o[15], r;
      if (RO) {
        // the policy step of rollout_kernel (scratch: the env's contact stores)
        float* x = reinterpret_cast<float*>(W.g);
        if (tm.tl < 15) x[tm.tl] = s_obs[i][tm.tl];
        team_sync();
        float mu[3] = {0.f, 0.f, 0.f}, val = 0.f;
        team_policy(ro.P, ro.off, x, x + 16, x + 144, tm, mu, val);
        const float* ls = ro.P + ro.off[MLP_LS];
        float lp = 0.f, araw[3];
#pragma unroll
        for (int j = 0; j < 3; j++) {
          const float ls_j = ls[j];
          araw[j] = __fadd_rn(mu[j], __fmul_rn(ro.noise[3 * row + j], expf(ls_j)));
          const float z = __fmul_rn(__fsub_rn(araw[j], mu[j]), expf(-ls_j));
          lp += -0.5f * z * z - ls_j - 0.5f * (2.f * 0.91893853320467274f);
          a[j] = fminf(fmaxf(araw[j], -1.f), 1.f);
        }
        if (lead) {
#pragma unroll
          for (int j = 0; j < 15; j++) ro.b_obs[15 * row + j] = s_obs[i][j];
#pragma unroll
          for (int j = 0; j < 3; j++) ro.b_act[3 * row + j] = araw[j];
          ro.b_val[row] = val;
          ro.b_logp[row] = lp;
          ro.b_starts[row] = uint8_t(s_start[i]);
        }
      } else {
        const float* ak = act + 3 * row;
        a[0] = ak[0]; a[1] = ak[1]; a[2] = ak[2];
      }
      const int fl = team_step<T>(m, cfg, d, e, tid, W.qn, W.vn, W.wn, step, bk, a, W, o, r,
                                  (!RO && tobs) ? tobs + 15 * row : nullptr, (!RO && pos2d) ? pos2d + 2 * row : nullptr,
                                  RO ? 1 : auto_reset, tm, s_cnt[i], full);
      if (lead) {
        if (RO) {  // collect_rollouts + Monitor bookkeeping (bb_rollout_track)
          const bool dn = (fl & F_TERMINATED) != 0;
          const double ret = s_ret[i] + double(r);
          const long long len = s_len[i] + 1;
          ro.b_rew[row] = r;
          ro.ep_r[row] = dn ? ret : __builtin_nan("");
          ro.ep_l[row] = dn ? len : 0;
          s_ret[i] = dn ? 0.0 : ret;
          s_len[i] = dn ? 0 : len;
          s_start[i] = dn ? 1 : 0;
#pragma unroll
          for (int j = 0; j < 15; j++) s_obs[i][j] = o[j];
        } else {
#pragma unroll
          for (int j = 0; j < 15; j++) obs[15 * row + j] = o[j];
          rew[row] = r;
          done[row] = uint8_t(fl);
        }
      }
      const bool next = k + 1 < K && predict_env<T>(m, d, tid, W.qn, W.vn, tm.tl, team_shift_of(16));
      team_sync();
      if (lead) {
        if (d.cost) d.cost[e] += clock64() - c0;  // this env's cost, for the next launch's balance
        s_tid[i] = tid;
        s_step[i] = step;
        s_kind[i] = next ? 1 : 0;
        s_k[i] = k + 1;
        atomicSub(&s_left, 1);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        s_busy[i] = 0;
      }
    }
  }
  __syncthreads();
  if (int(threadIdx.x) < nloc) {
    const int i = int(threadIdx.x), e = s_env[i];
    EnvWork<T>& W = team_work<T>(smem, i);
    store_state(d, e, W.qn, W.vn, W.wn, s_step[i]);
    counts_flush(d, s_cnt[i]);
    if (!RO && gate && s_cnt[i][3]) atomicAdd(d.slow_count + SC_TOUCHED, 1);  // adaptive: an env that took a full step
    if (RO) {
#pragma unroll
      for (int j = 0; j < 15; j++) ro.obs[15 * size_t(e) + j] = s_obs[i][j];
      ro.last_starts[e] = uint8_t(s_start[i]);
      ro.ep_ret[e] = s_ret[i];
      ro.ep_len[e] = s_len[i];
    }
  }
}

// ---- bb_step_multi on relief banks: the relief pair --------------------------
// relief_multi_kernel holds both steps, and the union of their registers spills
// (512 VGPRs, ~1 KB of scratch per lane, 21.5 GB of HBM traffic per 256-step
// launch on perlin).  The pair runs them as two PERSISTENT launches at the same
// time, on two streams: relief_pair_kernel<T, false> takes the steps the
// predictor routes to the fast path (only the fast step compiled in: no
// scratch) and relief_pair_kernel<T, true> the full steps (only the full step).
// An env moves between them through two FIFO rings of env ids in HBM (d.ring:
// fast, full; head/tail counters in slow_count) with its state in HBM; d.park[e]
// counts its steps.  Per env the steps are route 0's, as in relief_multi_kernel
// and bb_step (bit-identical): a predicted env takes the full step, the others
// the fast path, and an env the fast path hands over goes to the full launch,
// which redoes that step.  A team holds an env for at most `seg` steps and
// requeues it, so every env progresses evenly and the launch ends within a
// few segments of its last env.  Of each launch's grid of pair_cap one-wave
// workgroups (the chip's resident capacity) the first SC_ACTIVE[kind] work and
// the rest exit at once; the two counts add up to pair_cap, so the working
// workgroups of both launches are resident together and neither waits for the
// other to be scheduled.  pair_adapt_kernel moves workgroups between the kinds
// after each launch from the idle time each kind measured.  A wall-clock budget
// ends both launches with an error flag (stats[7]) should a launch ever wait
// for work that cannot come -- no hang.
constexpr int SC_RHEAD = 16, SC_RTAIL = 18, SC_DONE = 20, SC_ERR = 21, SC_ACTIVE = 22, SC_IDLE = 24;
// diagnostics of the last launch (bb_pair_counters): claims [2], completed steps [2], fast-path hand-overs
constexpr int SC_CLAIMS = 32, SC_STEPS = 34, SC_PARKED = 36;
// Between two holds within a launch an env's state lives in d.hand, one contiguous record per env
// (3 cache lines at fp64), written and read by the team's 16 lanes: in the SoA arrays the same
// 48 values sit in 48 lines, and each write-through (sc1) store of one value is its own memory
// request.  park[e] carries PARK_HAND once the record holds the env's state; the SoA arrays
// hold it at the launch's start and get it back when the env's K steps are done.
constexpr int HAND = NQ + 2 * NV + 1, PARK_HAND = 1 << 30;
// solo waves: ring 2 (the heavy envs' full steps) counters, the solo workgroup count, the heavy
// marks of this launch (reset by pair_rings_kernel, which keeps the count in SC_HEAVY_LAST)
constexpr int SC_SOLO = 42, SC_HEAVY = 43, SC_HEAVY_LAST = 44;
// Rings per XCD: the fast and full rings are sharded 8 ways by env block, env e belonging to
// XCD label (e >> 5) & 7 (32 envs: one 128-B line of a [K][n] float output), and a team takes
// envs from the rings of its workgroup's label, blockIdx & 7 -- the XCD the dispatcher deals
// that workgroup to.  So an env's steps run on one XCD's L2: the partial output lines of
// neighbouring envs merge there instead of being written back piecemeal from eight L2s, and
// its terrain cells stay cached.  The label is only a placement hint: any mapping is correct,
// since every label has fast and full workgroups (each kind keeps >= pair_cap / 8 >= 8).  The
// heavy envs' solo ring (kind 2) is one ring: the solo workgroups may cover fewer than 8 labels.
constexpr int NRINGS = 2 * NXCD + 1;  // NXCD: bb_pairmap.h
__device__ __forceinline__ int env_xcd(int e) { return (e >> 5) & (NXCD - 1); }
__device__ __forceinline__ int pair_ring(int kind, int x) { return kind < 2 ? kind * NXCD + x : 2 * NXCD; }

__device__ __forceinline__ int ld_agent(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The rings are ticket queues.  A team without an env takes a ticket (one
// atomicAdd on the ring's head: no compare-and-swap retries between the ~2000
// teams of a kind) and, at each later pass of its wave's loop, looks whether
// the entry of that ticket has arrived; a release appends its env with one
// atomicAdd on the tail.  Entries carry their ticket (ticket << 32 | env), so a
// slot needs no clearing and a look never takes an older lap's entry; the ring
// is longer than the envs plus the resident teams, so an entry is never
// overwritten before its ticket's holder took it.
__device__ __forceinline__ unsigned long long ring_entry(int ticket, int e) {
  return (static_cast<unsigned long long>(unsigned(ticket)) << 32) | unsigned(e);
}
__device__ __forceinline__ int ring_ticket(const Dev& d, int r) { return atomicAdd(d.rctr + 2 * r, 1); }
// the env of `ticket` in ring `kind`, or -1 while it has not been appended
__device__ __forceinline__ int ring_look(const Dev& d, int r, int ticket) {
  const unsigned long long v = ld_coh(d.ring + size_t(r) * d.ring_len + (unsigned(ticket) % unsigned(d.ring_len)));
  return unsigned(v >> 32) == unsigned(ticket) ? int(unsigned(v)) : -1;
}
// append env e to ring `kind` (lead lane; the env's state is stored and released)
__device__ __forceinline__ void ring_push(const Dev& d, int kind, int e) {
  const int r = pair_ring(kind, env_xcd(e));
  const int t = atomicAdd(d.rctr + 2 * r + 1, 1);
  st_coh(d.ring + size_t(r) * d.ring_len + (unsigned(t) % unsigned(d.ring_len)), ring_entry(t, e));
}

// A rollout's per-env carry between steps (ROLL): the observation the policy sees next, the
// episode-start flag and the Monitor's running return and length.  In LDS while a team holds
// the env; in RolloutDev's [n] arrays (device-coherent) between holds and at the ends.
struct RollCarry {
  float o[16];
  double ret;
  long long len;
  int start;
};

// one team loop of the relief pair (FULL: the full launch's; wg: this workgroup's index among
// its kind's working workgroups; the caller checked the gate and the active count).  ROLL: a
// PPO rollout (bb_rollout) instead of bb_step_multi's open-loop actions -- per step the team
// runs the policy on the env's observation (team_policy), samples and clips the action, steps,
// and keeps the rollout buffer and the Monitor's episode statistics (rollout_kernel's body);
// K is the rollout length, act and the [K][n] outputs are unused.
template <typename T, bool FULL, bool ROLL>
__device__ __forceinline__ void pair_loop(const ModelT<T>& mg, const EnvCfg& cfg, const Dev& d, const float* __restrict__ act,
                                          int K, float* __restrict__ obs, float* __restrict__ rew,
                                          uint8_t* __restrict__ done, float* __restrict__ tobs,
                                          float* __restrict__ pos2d, int auto_reset, int seg,
                                          unsigned long long budget, const int* __restrict__ gate, int wg,
                                          unsigned char* smem, ModelT<T>& ms, unsigned (*s_cnt)[8], int (*s_diag)[3],
                                          const RolloutDev& ro, RollCarry* s_roll) {
  int* sc = d.slow_count;
  if (threadIdx.x == 0) ms = mg;
  if (threadIdx.x < 32) s_cnt[threadIdx.x >> 3][threadIdx.x & 7] = 0u;
  __syncthreads();
  const ModelT<T>& m = ms;
  const Team tm{TEAM, int(threadIdx.x) & (TEAM - 1)};
  const int team = int(threadIdx.x) / TEAM;
  const bool lead = tm.tl == 0;
  const int n = d.n;
  EnvWork<T>& W = team_work<T>(smem, team);
  T* bk = reinterpret_cast<T*>(smem + size_t(WAVE / TEAM) * work_stride<T>()) + team * (NQ + 2 * NV);
  unsigned* cnt = s_cnt[team];
  if (lead) { s_diag[team][0] = 0; s_diag[team][1] = 0; s_diag[team][2] = 0; }
  const int kind = FULL ? 1 : 0;
  // solo waves (full launch, the first sc[SC_SOLO] workgroups): team 0 alone steps the envs
  // marked heavy (ring 2), so a heavy env's step never waits for wave-mates' divergent work
  const bool solo = FULL && wg < sc[SC_SOLO];
  const int rkind = solo ? 2 : kind;
  const int myring = pair_ring(rkind, int(blockIdx.x) & (NXCD - 1));  // this team's ring (see env_xcd)
  const unsigned long long t0 = wall_clock64(), c_start = clock64();
  unsigned long long tw = t0;  // when this team last became idle: the budget bounds a wait, not the team's life
  int e = -1, k = 0, tid = 0, step = 0, held = 0, ticket = -1;  // ticket: the lead's, -1 when none
  unsigned idle = 0;
  unsigned long long busy = 0;  // this team's cycles stepping envs (the split of the next launch)
  unsigned long long held_busy = 0;  // ... the held env's, since the claim
  for (;;) {
    // a team without an env takes the next one of its kind (the rest of the wave
    // skips this block); stop when every env has done its K steps
    int stop = 0;
    if (e < 0) {
      int got = -1;
      if (lead) {
        if (ld_agent(sc + SC_DONE) >= n || ld_agent(sc + SC_ERR) || (solo && team > 0)) {
          got = -2;
        } else {
          if (ticket < 0) ticket = ring_ticket(d, myring);
          got = ring_look(d, myring, ticket);
          if (got >= 0) ticket = -1;
          else if (wall_clock64() - tw > budget) {
            // no env came for `budget` ticks: end the launch for every team, count it, and
            // raise the handle's sticky fault (host-mapped: bb_check / the next call reports it)
            if (atomicExch(sc + SC_ERR, 1) == 0) {
              atomicAdd(&d.stats[7], 1ull);
              if (d.fault) __hip_atomic_store(d.fault, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            got = -2;
          }
        }
      }
      got = __shfl(got, team_shift_of(TEAM));
      if (got == -2) {
        stop = 1;
      } else if (got >= 0) {
        // acquire: the releasing team's device-coherent stores, read device-coherently
        // (their addresses depend on the popped id, so they issue after it)
        e = got;
        const int pk = ld_coh(d.park + e);
        k = pk & (PARK_HAND - 1);
        if (pk & PARK_HAND) {  // the record (qn, vn, wn are contiguous in EnvWork)
          const T* hr = reinterpret_cast<const T*>(d.hand) + size_t(e) * HAND;
          for (int i = tm.tl; i < HAND - 1; i += TEAM) W.qn[i] = ld_coh(hr + i);
          step = int(ld_coh(hr + HAND - 1));
          team_sync();
        } else {
          load_state<T, true>(d, e, W.qn, W.vn, W.wn, step);
        }
        tid = ld_coh(d.terrain + e);
        held = 0;
        held_busy = 0;
        if (lead) { W.bspill = body_spill_of<T>(d, e); s_diag[team][0]++; }
        if constexpr (ROLL) {  // the env's rollout carry
          RollCarry& c = s_roll[team];
          if (tm.tl < 15) c.o[tm.tl] = ld_coh(ro.obs + 15 * size_t(e) + tm.tl);
          if (lead) {
            c.start = int(ld_coh(ro.last_starts + e));
            c.ret = ld_coh(ro.ep_ret + e);
            c.len = ld_coh(ro.ep_len + e);
          }
        }
        team_sync();
      }
    }
    if (stop) break;
    if (e >= 0) {
      const unsigned long long c0 = clock64();
      const size_t row = size_t(k) * n + e;
      float a[3];
      if constexpr (ROLL) {
        // SB3 policy step on the carried observation (rollout_kernel's arithmetic); a step the
        // fast path hands over is redone by the full loop from the same observation and noise,
        // so its buffer rows are rewritten with the same values
        RollCarry& c = s_roll[team];
        float* pol = reinterpret_cast<float*>(W.g);  // x[16], hA[128], hB[128]: contact stores, dead between steps
        team_sync();
        if (tm.tl < 15) pol[tm.tl] = c.o[tm.tl];
        team_sync();
        float mu[3] = {0.f, 0.f, 0.f}, val = 0.f;
        team_policy(ro.P, ro.off, pol, pol + 16, pol + 144, tm, mu, val);
        const float* ls = ro.P + ro.off[MLP_LS];
        constexpr float HL2PI = 0.91893853320467274f;
        float araw[3], lp = 0.f;
#pragma unroll
        for (int j = 0; j < 3; j++) {
          const float ls_j = ls[j];
          araw[j] = __fadd_rn(mu[j], __fmul_rn(ro.noise[3 * row + j], expf(ls_j)));
          const float z = __fmul_rn(__fsub_rn(araw[j], mu[j]), expf(-ls_j));
          lp += -0.5f * z * z - ls_j - 0.5f * (2.f * HL2PI);
          a[j] = fminf(fmaxf(araw[j], -1.f), 1.f);
        }
        if (lead) {
#pragma unroll
          for (int i = 0; i < 15; i++) ro.b_obs[15 * row + i] = c.o[i];
#pragma unroll
          for (int j = 0; j < 3; j++) ro.b_act[3 * row + j] = araw[j];
          ro.b_val[row] = val;
          ro.b_logp[row] = lp;
          ro.b_starts[row] = uint8_t(c.start);
        }
      } else {
        const float* ak = act + 3 * row;
        a[0] = ak[0]; a[1] = ak[1]; a[2] = ak[2];
      }
      float o[15], r;
      const int fl = team_step<T, FULL, FULL>(m, cfg, d, e, tid, W.qn, W.vn, W.wn, step, bk, a, W, o, r,
                                               tobs ? tobs + 15 * row : nullptr, pos2d ? pos2d + 2 * row : nullptr,
                                               auto_reset, tm, cnt);
      int next = kind;
      if (!FULL && (fl & F_PARKED)) {  // the fast path handed the step over: the full launch redoes it
        next = 1;
        if (lead) s_diag[team][2]++;
      } else if constexpr (ROLL) {  // collect_rollouts + Monitor bookkeeping (bb_rollout_track)
        RollCarry& c = s_roll[team];
        const bool dn = (fl & F_TERMINATED) != 0;
        if (lead) {
          s_diag[team][1]++;
          const double ret = c.ret + double(r);
          const long long len = c.len + 1;
          ro.b_rew[row] = r;
          ro.ep_r[row] = dn ? ret : __builtin_nan("");
          ro.ep_l[row] = dn ? len : 0;
          c.ret = dn ? 0.0 : ret;
          c.len = dn ? 0 : len;
          c.start = dn ? 1 : 0;
        }
        if (tm.tl < 15) c.o[tm.tl] = o[tm.tl];
        k++;
        held++;
        if (k < K) next = predict_env<T>(m, d, tid, W.qn, W.vn, tm.tl, team_shift_of(TEAM)) ? 1 : 0;
      } else {
        if (lead) {
          s_diag[team][1]++;
          if (!(BB_OUT_SKIP & 1)) {
#pragma unroll
            for (int i = 0; i < 15; i++) out_st(obs + 15 * row + i, o[i]);
          }
          if (!(BB_OUT_SKIP & 2)) out_st(rew + row, r);
          if (!(BB_OUT_SKIP & 4)) out_st(done + row, uint8_t(fl));
        }
        k++;
        held++;
        if (k < K) next = predict_env<T>(m, d, tid, W.qn, W.vn, tm.tl, team_shift_of(TEAM)) ? 1 : 0;
      }
      const unsigned long long dc = clock64() - c0;
      busy += dc;
      held_busy += dc;
      if (k >= K || next != kind || held >= seg) {  // release the env (team-uniform)
        team_sync();
        if (k < K) {  // the record, spread over the team's lanes
          T* hr = reinterpret_cast<T*>(d.hand) + size_t(e) * HAND;
          for (int i = tm.tl; i < HAND - 1; i += TEAM) st_coh(hr + i, W.qn[i]);
          if (lead) st_coh(hr + HAND - 1, T(step));
        }
        if constexpr (ROLL) {  // the carry, for the next holder (or the caller, after the last step)
          const RollCarry& c = s_roll[team];
          if (tm.tl < 15) st_coh(ro.obs + 15 * size_t(e) + tm.tl, c.o[tm.tl]);
          if (lead) {
            st_coh(ro.last_starts + e, uint8_t(c.start));
            st_coh(ro.ep_ret + e, c.ret);
            st_coh(ro.ep_len + e, c.len);
          }
        }
        if (lead) {
          if (k >= K) store_state<T, true>(d, e, W.qn, W.vn, W.wn, step);
          st_coh(d.park + e, k < K ? k | PARK_HAND : k);
          st_coh(d.pair_env + e, ld_coh(d.pair_env + e) + held_busy);
          if (k >= K) st_coh(d.pair_env + n + e, static_cast<unsigned long long>(wall_clock64()));
          stores_done();  // release: the state (and a reset's draw) before the ring entry
          if (k >= K) atomicAdd(sc + SC_DONE, 1);
          else ring_push(d, next == 1 && (d.pred_mark[e] & 2) ? 2 : next, e);
          if (FULL && gate) atomicAdd(sc + SC_TOUCHED, 1);  // adaptive route: an env took full steps
          tw = wall_clock64();
        }
        e = -1;
      }
    } else {
      idle++;
    }
    // the wave sleeps only when none of its teams holds an env
    if (__ballot(e >= 0) == 0ull) __builtin_amdgcn_s_sleep(8);
  }
  team_sync();
  if (lead) {
    counts_flush(d, cnt);
    if (idle) atomicAdd(sc + SC_IDLE + kind, int(idle > 1000000u ? 1000000u : idle));
    if (busy) atomicAdd(d.pair_busy + kind, busy);
    atomicAdd(d.pair_busy + 2 + kind, clock64() - c_start);
    atomicAdd(d.pair_busy + 4 + kind, wall_clock64() - t0);
    atomicAdd(sc + SC_CLAIMS + kind, s_diag[team][0]);
    atomicAdd(sc + SC_STEPS + kind, s_diag[team][1]);
    if (!FULL) atomicAdd(sc + SC_PARKED, s_diag[team][2]);
  }
}

// the pair as two launches (on two streams)
template <typename T, bool FULL>
__global__ __launch_bounds__(64) void relief_pair_kernel(ModelT<T> mg, EnvCfg cfg, Dev d, const float* __restrict__ act,
                                                         int K, float* __restrict__ obs, float* __restrict__ rew,
                                                         uint8_t* __restrict__ done, float* __restrict__ tobs,
                                                         float* __restrict__ pos2d, int auto_reset, int seg,
                                                         unsigned long long budget, const int* __restrict__ gate) {
  // adaptive form: the parked launches run instead; else only the active workgroups
  // (workgroup-uniform, before any barrier)
  if ((gate && *gate == ROUTE_PARK) || int(blockIdx.x) >= d.slow_count[SC_ACTIVE + FULL]) return;
  extern __shared__ __align__(16) unsigned char smem[];
  __shared__ ModelT<T> ms;
  __shared__ unsigned s_cnt[WAVE / TEAM][8];
  __shared__ int s_diag[WAVE / TEAM][3];  // claims, completed steps, fast-path hand-overs
  pair_loop<T, FULL, false>(mg, cfg, d, act, K, obs, rew, done, tobs, pos2d, auto_reset, seg, budget, gate,
                            int(blockIdx.x), smem, ms, s_cnt, s_diag, RolloutDev{}, nullptr);
}

// the pair as ONE launch: SC_ACTIVE[0] workgroups run the fast loop and SC_ACTIVE[1] the full
// loop, interleaved by groups of NXCD blocks (pair_kind_of); the two loops are disjoint regions
// of the kernel, so it keeps the larger one's registers, not their union.  ROLL: a rollout
// (bb_rollout on relief banks; ro), K = ro.T
template <typename T, bool ROLL>
__global__ __launch_bounds__(64) void relief_pair1_kernel(ModelT<T> mg, EnvCfg cfg, Dev d, const float* __restrict__ act,
                                                          int K, float* __restrict__ obs, float* __restrict__ rew,
                                                          uint8_t* __restrict__ done, float* __restrict__ tobs,
                                                          float* __restrict__ pos2d, int auto_reset, int seg,
                                                          unsigned long long budget, const int* __restrict__ gate,
                                                          RolloutDev ro) {
  if (gate && *gate == ROUTE_PARK) return;
  int wg = 0;
  const int kind = pair_kind_of(int(blockIdx.x), d.slow_count[SC_ACTIVE], d.slow_count[SC_ACTIVE + 1], &wg);
  if (kind < 0) return;  // workgroup-uniform, before any barrier
  extern __shared__ __align__(16) unsigned char smem[];
  __shared__ ModelT<T> ms;
  __shared__ unsigned s_cnt[WAVE / TEAM][8];
  __shared__ int s_diag[WAVE / TEAM][3];
  __shared__ RollCarry s_roll[ROLL ? WAVE / TEAM : 1];
  if (kind == 0)
    pair_loop<T, false, ROLL>(mg, cfg, d, act, K, obs, rew, done, tobs, pos2d, auto_reset, seg, budget, gate, wg, smem,
                              ms, s_cnt, s_diag, ro, s_roll);
  else
    pair_loop<T, true, ROLL>(mg, cfg, d, act, K, obs, rew, done, tobs, pos2d, auto_reset, seg, budget, gate, wg, smem,
                             ms, s_cnt, s_diag, ro, s_roll);
}

// before the pair: every env's first route (predict_kernel's test) into the
// rings in env order, step counts to 0, counters reset.  One workgroup per 4 envs.
template <typename T>
__global__ __launch_bounds__(64) void pair_init_kernel(ModelT<T> mg, Dev d, const int* __restrict__ gate, int heavy_pct) {
  if (gate && *gate == ROUTE_PARK) return;
  __shared__ ModelT<T> ms;
  if (threadIdx.x == 0) ms = mg;
  __syncthreads();
  const int tl = int(threadIdx.x) & 15;
  const int e = blockIdx.x * (WAVE / 16) + int(threadIdx.x) / 16;
  if (e >= d.n) return;  // team-uniform
  const T* Q = (const T*)d.qpos;
  const T* V = (const T*)d.qvel;
  T Qe[NQ], Ve[6];
#pragma unroll
  for (int i = 0; i < NQ; i++) Qe[i] = Q[i * d.n + e];
#pragma unroll
  for (int i = 0; i < 6; i++) Ve[i] = V[i * d.n + e];
  const bool full = predict_env<T>(ms, d, d.terrain[e], Qe, Ve, tl, team_shift_of(16));
  if (tl == 0) {
    // heavy: the env's steps took more than heavy_pct % of the mean env's in the last
    // launch (its full steps then go to the solo waves, at most SC_SOLO envs)
    const unsigned long long tot = d.pair_busy[0] + d.pair_busy[1];
    const int nsolo = d.slow_count[SC_SOLO];
    bool heavy = false;
    if (nsolo > 0 && tot > 0 &&
        double(d.pair_env[e]) * double(d.n) > double(tot) * double(heavy_pct) * 0.01)
      heavy = atomicAdd(d.slow_count + SC_HEAVY, 1) < nsolo;
    d.pred_mark[e] = uint8_t((full ? 1 : 0) | (heavy ? 2 : 0));
    d.park[e] = 0;
    d.pair_env[e] = 0;
    ring_push(d, full ? (heavy ? 2 : 1) : 0, e);  // the rings were cleared by pair_clear_kernel
  }
}

// before pair_init_kernel: every ring slot empty (no ticket's entry) and the ring counters at 0
__global__ __launch_bounds__(256) void pair_clear_kernel(Dev d, const int* __restrict__ gate) {
  if (gate && *gate == ROUTE_PARK) return;
  const size_t tot = size_t(NRINGS) * d.ring_len;
  for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < tot; i += size_t(gridDim.x) * blockDim.x)
    d.ring[i] = ~0ull;
  if (blockIdx.x == 0 && threadIdx.x < 2 * NRINGS) d.rctr[threadIdx.x] = 0;
}

// after pair_init_kernel (which filled the rings): the launch's counters
__global__ void pair_rings_kernel(Dev d, const int* __restrict__ gate) {
  if ((gate && *gate == ROUTE_PARK) || threadIdx.x != 0) return;
  int* sc = d.slow_count;
  sc[SC_DONE] = 0; sc[SC_ERR] = 0;
  sc[SC_IDLE] = 0; sc[SC_IDLE + 1] = 0;
  sc[SC_CLAIMS] = 0; sc[SC_CLAIMS + 1] = 0; sc[SC_STEPS] = 0; sc[SC_STEPS + 1] = 0; sc[SC_PARKED] = 0;
  sc[SC_HEAVY_LAST] = sc[SC_HEAVY];
  sc[SC_HEAVY] = 0;
  for (int i = 0; i < 6; i++) d.pair_busy[i] = 0;
}

// after the pair: the next launch splits the resident workgroups in proportion
// to the team-cycles each kind spent stepping in this one (the work of the two
// kinds, whatever this launch's split was), keeping cap / 8 for each.  The
// counts only place work: every env's results are the same whatever they are.
__global__ void pair_adapt_kernel(Dev d, int cap, const int* __restrict__ gate) {
  if (threadIdx.x != 0 || (gate && *gate == ROUTE_PARK)) return;
  int* sc = d.slow_count;
  const double bf = double(d.pair_busy[0]), bs = double(d.pair_busy[1]);
  if (bf + bs <= 0) return;
  // whole groups of NXCD workgroups (pair_kind_of), at least cap / 8 per kind
  const int G = cap / NXCD, lo = (G + 7) / 8;
  int gs = int(double(G) * bs / (bf + bs) + 0.5);
  gs = gs < lo ? lo : (gs > G - lo ? G - lo : gs);
  sc[SC_ACTIVE] = (G - gs) * NXCD;
  sc[SC_ACTIVE + 1] = gs * NXCD;
}

// Between relief_multi_kernel launches: deal the envs over its workgroups so
// that each gets a mix of expensive and cheap ones.  An env's cost in the
// last launch (shader cycles of its steps) predicts the next one well (its
// terrain and posture persist for many steps), and a workgroup runs until its
// last env is done: without this, whole CUs idled for ~40% of a perlin launch
// while the workgroups holding toppled robots finished.  One workgroup: a
// 1024-bucket counting sort of the costs (scaled to the maximum), then a
// snake deal (round r of the sorted envs goes to workgroups 0..nwg-1, the next
// round back), and the costs restart from 0.  n must be nwg * QENV.
__global__ __launch_bounds__(1024) void balance_kernel(Dev d, int nwg) {
  constexpr int NB = 1024;
  __shared__ unsigned long long s_max;
  __shared__ int hist[NB];
  const int t = int(threadIdx.x), n = d.n;
  if (t == 0) s_max = 1;
  hist[t] = 0;
  __syncthreads();
  unsigned long long mx = 1;
  for (int e = t; e < n; e += NB) mx = d.cost[e] > mx ? d.cost[e] : mx;
  atomicMax(&s_max, mx);
  __syncthreads();
  const unsigned long long top = s_max;
  auto bucket = [&](int e) { return int((d.cost[e] * (NB - 1)) / top); };
  for (int e = t; e < n; e += NB) atomicAdd(&hist[NB - 1 - bucket(e)], 1);  // descending cost
  __syncthreads();
  if (t == 0) {  // exclusive scan (1024 entries, once per launch)
    int acc = 0;
    for (int b = 0; b < NB; b++) { const int c = hist[b]; hist[b] = acc; acc += c; }
  }
  __syncthreads();
  for (int e = t; e < n; e += NB) {  // position in the sorted order (ties: any order)
    const int p = atomicAdd(&hist[NB - 1 - bucket(e)], 1);
    const int r = p / nwg, j = p % nwg;
    const int wg = (r & 1) ? nwg - 1 - j : j;
    d.perm[wg * QENV + r] = e;
  }
  __syncthreads();
  for (int e = t; e < n; e += NB) d.cost[e] = 0;
}

// Stable split of 0..n-1 by pred_mark into fast_envs / pred_envs (one block).
__global__ __launch_bounds__(1024) void split_kernel(Dev d) {
  __shared__ int sf[1024], ss[1024];
  const int t = threadIdx.x, per = (d.n + 1023) / 1024, b = t * per, e_ = min(d.n, b + per);
  int nf = 0, ns = 0;
  for (int e = b; e < e_; e++) { if (d.pred_mark[e]) ns++; else nf++; }
  sf[t] = nf; ss[t] = ns;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {  // inclusive scan
    const int af = t >= off ? sf[t - off] : 0, as = t >= off ? ss[t - off] : 0;
    __syncthreads();
    sf[t] += af; ss[t] += as;
    __syncthreads();
  }
  int of = sf[t] - nf, os = ss[t] - ns;
  for (int e = b; e < e_; e++) {
    if (d.pred_mark[e]) d.pred_envs[os++] = e; else d.fast_envs[of++] = e;
  }
  if (t == 1023) { d.slow_count[0] = sf[t]; d.slow_count[1] = ss[t]; d.slow_count[2] = 0; }
}

// route 1: the hand-over count starts at zero for the fast kernel.  A kernel,
// not hipMemsetAsync: a captured step then holds only kernel nodes, ordered
// like any other launch on the stream.
__global__ void zero_count_kernel(int* c) {
  if (threadIdx.x == 0) *c = 0;
}

// after an adaptive bb_step_multi on a relief bank: the next launch takes the
// parked multi-step form when fewer than `max_touched` envs needed a full step
// in this one (1: none -- hills' flat centre in steady state), else the work
// queue.  One env parked early already costs the parked form a serial finish
// launch of nearly K steps, so the queue takes over at the first one.
// Deterministic: the choice depends on the envs' results only (no host sync).
__global__ void route_decide_kernel(int* sc, int max_touched) {
  if (threadIdx.x == 0) {
    sc[SC_ROUTE] = sc[SC_TOUCHED] < max_touched ? ROUTE_PARK : 0;
    sc[SC_TOUCHED] = 0;
  }
}

__global__ void assign_kernel(Dev d, const int32_t* ids) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= d.n) return;
  const int t = ids[e];
  d.pending_terrain[e] = (t >= 0 && t < d.n_terrains) ? t : -1;  // -1: back to the terrain stream
}

}  // namespace

struct bb_handle {
  int n, device, fp64, team, epw;
  int epw_full;  // envs per wave of the full kernel (its lists are a minority of the envs)
  hipStream_t side;                 // the concurrent full-kernel launch
  hipEvent_t fork, join;
  bb_params p;
  EnvCfg cfg;
  ModelT<float> mf;
  ModelT<double> md;
  Dev d;
  float* bank;
  float* size_z;
  float* offset;
  float* hmax;
  std::vector<float> h_offset;
  // optional HIP-event timing of the step kernels (bb_time_kernel): per timed
  // step 6 events, pairs around the fast kernel, the predicted full kernel
  // (route 0, on the side stream) and the hand-over full kernel
  std::vector<hipEvent_t> tev;
  std::vector<uint8_t> tpred;  // per timed step: the predicted full kernel was launched
  int tcap = 0, tn = 0;
  // step routing: 0 predict + concurrent full kernel; 1 serial fast-then-full;
  // -1 (default) serial while every terrain in the bank is flat, else 0.  On
  // flat banks hand-overs are rare and the serial route saves the predict and
  // split launches (3.66 M vs 3.57 M env-steps/s at 4096 flat envs)
  int route = -1;
  int multi_queue = 1;          // bb_step_multi on relief banks: relief_multi_kernel (BB_MULTI_QUEUE=0: off)
  int multi_park = 1;           // bb_step_multi, serial route: two launches, hand-overs parked (BB_MULTI_PARK=0: one)
  int multi_adapt = 1;          // bb_step_multi on relief banks: queue or parked launches per launch (BB_MULTI_ADAPT=0:
                                // always the queue; off when BB_ROUTE or BB_MULTI_QUEUE fixes the form)
  int balance = 1;              // relief_multi_kernel: cost-balanced env placement (BB_BALANCE=0: in order)
  int pair = 1;                 // relief banks: bb_step_multi's work queue is the relief pair (BB_RELIEF_PAIR=0:
                                // relief_multi_kernel, the one-launch queue)
  int pair_cap = 0;             // one-wave workgroups resident on the chip (4 per CU)
  int pair_seg = 16;            // steps a team holds an env before requeueing it (BB_PAIR_SEG)
  int pair_adapt = 1;           // split the workgroups by the last launch's work (BB_PAIR_ADAPT=0: keep the first split)
  int pair_one = 1;             // the pair as one launch (BB_PAIR_ONE=0: two concurrent launches on two streams)
  int pair_solo = 0;            // solo waves for heavy envs' full steps (BB_PAIR_SOLO; <= pair_cap / 8)
  int pair_heavy_pct = 150;     // heavy: last launch's cycles above this % of the mean env's (BB_PAIR_HEAVY)
  unsigned long long pair_budget = 0;  // wall-clock ticks a pair team may wait for an env (20 s)
  double pair_budget_s = 20;
  int count_memset = 0;         // diagnostic (BB_COUNT_MEMSET=1): reset the hand-over count with
                                // hipMemsetAsync instead of zero_count_kernel
  std::vector<uint8_t> relief;  // per terrain: max height > 0
  int n_relief = 0;
  int* tstream = nullptr;       // device copies of the terrain streams (bb_set_terrain_stream)
  int* env_stream = nullptr;
  size_t tstream_cap = 0;       // ints allocated at tstream (refilled in place while the table fits)
  int n_streams = 0;
  unsigned long long* rng = nullptr;  // per-env PCG64 words [5][n] (bb_set_terrain_rng), allocated once
  int* seed_slot = nullptr;           // [TERRAIN_SEEDS], allocated once
  TerrainSrc tsrc{};                  // host copy of the device record Dev.tsrc points at
  TerrainSrc* tsrc_dev = nullptr;
  CamRig rig;  // depth cameras in the base body (bb_render_depth)
  void* scenes = nullptr;
  volatile int* fault_host = nullptr;  // Dev.fault's host side (hipHostMalloc, mapped)
};

template <typename T> const ModelT<T>& model_of(const bb_handle* h);
template <> inline const ModelT<float>& model_of<float>(const bb_handle* h) { return h->mf; }
template <> inline const ModelT<double>& model_of<double>(const bb_handle* h) { return h->md; }

// bb_pair.hip's launch of the relief pair (declared again, with its comment, below)
extern "C" __attribute__((visibility("hidden"))) int bb_pair_launch_tu(bb_handle* h, int fp64, const float* a, int K,
                                                                      float* o, float* r, uint8_t* dn, float* t,
                                                                      float* p2, int ar, hipStream_t s,
                                                                      const int* gate, const void* ro);

namespace {
// init height offset (ballbot_env.py:546-563), incl. cell_size = size/nrows
float init_offset(const float* hf, float size_z) {
  const int n = HF_N;
  const double sz = 5.0, cell = sz / n, r = 0.09;
  const int center = n / 2;
  int x0 = center - abs((int)floor(-r / cell)), x1 = center + (int)floor(r / cell) + 1;
  int y0 = center - abs((int)floor(-r / cell)), y1 = center + (int)floor(r / cell) + 1;
  double mx = -1e300;
  for (int i = x0; i < x1; i++)
    for (int j = y0; j < y1; j++) mx = fmax(mx, (double)hf[i * n + j]);
  return float(mx * size_z + 0.01);
}

Dev balanced_dev(bb_handle* h, hipStream_t s) {
  Dev dq = h->d;
  if (h->n % QENV == 0 && h->balance)
    hipLaunchKernelGGL(balance_kernel, dim3(1), dim3(1024), 0, s, h->d, h->n / QENV);
  else
    dq.perm = nullptr;
  return dq;
}

template <typename T>
int launch_step(bb_handle* h, const float* a, float* o, float* r, uint8_t* dn, float* t, float* p2, int ar,
                hipStream_t s) {
  const ModelT<T>& m = model_of<T>(h);
  const int epw = h->epw;
  const int blocks = (h->n + epw - 1) / epw;
  const size_t lds = lds_bytes<T>(epw);
  const int epf = h->epw_full;
  const int fblocks = (h->n + epf - 1) / epf;
  const size_t flds = lds_bytes<T>(epf);
  int* cnt = h->d.slow_count;
  const int route = h->route >= 0 ? h->route : (h->n_relief == 0 ? 1 : 0);
  if (route == 1) {
    // serial route: the fast kernel over every env, then the full kernel over
    // the envs it handed over (no prediction, no second stream)
    if (h->count_memset)
      HIPCHK(hipMemsetAsync(cnt + 2, 0, sizeof(int), s));
    else
      hipLaunchKernelGGL(zero_count_kernel, dim3(1), dim3(64), 0, s, cnt + 2);
    const bool timed = h->tn < h->tcap;
    hipEvent_t* ev = timed ? &h->tev[6 * h->tn] : nullptr;
    if (timed) HIPCHK(hipEventRecord(ev[0], s));
    hipLaunchKernelGGL((step_kernel<T, false>), dim3(blocks), dim3(WAVE), lds, s, m, h->cfg, h->d, a, o, r, dn, t,
                       p2, ar, h->team, epw, (const int*)nullptr, (const int*)nullptr);
    if (timed) HIPCHK(hipEventRecord(ev[1], s));
    hipLaunchKernelGGL((step_kernel<T, true>), dim3(fblocks), dim3(WAVE), flds, s, m, h->cfg, h->d, a, o, r, dn, t,
                       p2, ar, h->team, epf, (const int*)h->d.slow_list, (const int*)(cnt + 2));
    if (timed) { HIPCHK(hipEventRecord(ev[5], s)); h->tpred[h->tn] = 0; h->tn++; }
    HIPCHK(hipGetLastError());
    return 0;
  }
  // route: envs near a base-tree contact -> full kernel (side stream,
  // concurrent); the rest -> fast kernel; its hand-overs -> full kernel after
  hipLaunchKernelGGL(predict_kernel<T>, dim3((h->n + WAVE / 16 - 1) / (WAVE / 16)), dim3(WAVE), 0, s, m, h->d);
  hipLaunchKernelGGL(split_kernel, dim3(1), dim3(1024), 0, s, h->d);
  HIPCHK(hipEventRecord(h->fork, s));
  HIPCHK(hipStreamWaitEvent(h->side, h->fork, 0));
  const bool timed = h->tn < h->tcap;
  hipEvent_t* ev = timed ? &h->tev[6 * h->tn] : nullptr;
  if (timed) HIPCHK(hipEventRecord(ev[2], h->side));
  hipLaunchKernelGGL((step_kernel<T, true>), dim3(fblocks), dim3(WAVE), flds, h->side, m, h->cfg, h->d, a, o, r, dn,
                     t, p2, ar, h->team, epf, (const int*)h->d.pred_envs, (const int*)(cnt + 1));
  if (timed) HIPCHK(hipEventRecord(ev[3], h->side));
  if (timed) HIPCHK(hipEventRecord(ev[0], s));
  hipLaunchKernelGGL((step_kernel<T, false>), dim3(blocks), dim3(WAVE), lds, s, m, h->cfg, h->d, a, o, r, dn, t, p2,
                     ar, h->team, epw, (const int*)h->d.fast_envs, (const int*)(cnt + 0));
  if (timed) HIPCHK(hipEventRecord(ev[1], s));
  HIPCHK(hipEventRecord(h->join, h->side));
  HIPCHK(hipStreamWaitEvent(s, h->join, 0));
  hipLaunchKernelGGL((step_kernel<T, true>), dim3(fblocks), dim3(WAVE), flds, s, m, h->cfg, h->d, a, o, r, dn, t, p2,
                     ar, h->team, epf, (const int*)h->d.slow_list, (const int*)(cnt + 2));
  if (timed) { HIPCHK(hipEventRecord(ev[5], s)); h->tpred[h->tn] = 1; h->tn++; }
  HIPCHK(hipGetLastError());
  return 0;
}
// bytes of dynamic LDS of multi_step_kernel: the teams' EnvWork + their step-start copies
template <typename T>
size_t multi_lds_bytes(int epw) { return lds_bytes<T>(epw) + size_t(epw) * (NQ + 2 * NV) * sizeof(T); }

// The Dev of a relief_multi_kernel launch: with n a multiple of QENV the envs
// are dealt by last launch's cost (balance_kernel, on stream s), else in order.
Dev balanced_dev(bb_handle* h, hipStream_t s);

// dynamic LDS of relief_multi_kernel: QENV EnvWork + their step-start copies
template <typename T>
size_t relief_lds_bytes() { return lds_bytes<T>(QENV) + size_t(QENV) * (NQ + 2 * NV) * sizeof(T); }

// dynamic LDS of rollout_kernel: multi_step_kernel's (the policy scratch lives in EnvWork)
template <typename T>
size_t rollout_lds_bytes(int epw) { return multi_lds_bytes<T>(epw); }

template <typename T>
int launch_rollout(bb_handle* h, const RolloutDev& ro, hipStream_t s) {
  const int epw = h->epw;
  const int blocks = (h->n + epw - 1) / epw;
  const int route = h->route >= 0 ? h->route : (h->n_relief == 0 ? 1 : 0);
  if (route == 0 && h->team == 16 && h->multi_queue && h->pair && h->pair_one) {
    // relief banks: the relief pair with the policy in it (pair_loop<.., ROLL>)
    if (bb_pair_launch_tu(h, sizeof(T) == 8, nullptr, ro.T, nullptr, nullptr, nullptr, nullptr, nullptr, 1, s, nullptr,
                          &ro))
      return fail("bb_rollout: relief pair launch failed");
  } else if (route == 0 && h->team == 16 && h->multi_queue) {  // relief banks: the work queue with the policy in it
    const Dev dq = balanced_dev(h, s);
    hipLaunchKernelGGL((relief_multi_kernel<T, true>), dim3((h->n + QENV - 1) / QENV), dim3(64 * QW),
                       relief_lds_bytes<T>(), s, model_of<T>(h), h->cfg, dq, (const float*)nullptr, ro.T,
                       (float*)nullptr, (float*)nullptr, (uint8_t*)nullptr, (float*)nullptr, (float*)nullptr, 1, ro,
                       (const int*)nullptr);
  } else if (h->multi_park) {  // the fast steps, then the parked envs' hand-overs and the rest of their steps
    hipLaunchKernelGGL((rollout_kernel<T, false>), dim3(blocks), dim3(WAVE), rollout_lds_bytes<T>(epw), s,
                       model_of<T>(h), h->cfg, h->d, ro, h->team, epw, h->d.park);
    hipLaunchKernelGGL((rollout_kernel<T, true>), dim3(blocks), dim3(WAVE), rollout_lds_bytes<T>(epw), s,
                       model_of<T>(h), h->cfg, h->d, ro, h->team, epw, h->d.park);
  } else
    hipLaunchKernelGGL((rollout_kernel<T, true>), dim3(blocks), dim3(WAVE), rollout_lds_bytes<T>(epw), s,
                       model_of<T>(h), h->cfg, h->d, ro, h->team, epw, (int*)nullptr);
  HIPCHK(hipGetLastError());
  return 0;
}

// the relief pair on relief banks (see relief_pair_kernel): routes, rings, the
// two persistent launches on the caller's stream and the handle's side stream,
// then the split adaptation.  gate: the adaptive route's flag (NULL: always run)
template <typename T>
int launch_pair(bb_handle* h, const float* a, int K, float* o, float* r, uint8_t* dn, float* t, float* p2, int ar,
                hipStream_t s, const int* gate, const RolloutDev* ro) {
  const ModelT<T>& m = model_of<T>(h);
  const size_t plb = multi_lds_bytes<T>(4);
  hipLaunchKernelGGL(pair_clear_kernel, dim3(64), dim3(256), 0, s, h->d, gate);
  hipLaunchKernelGGL(pair_init_kernel<T>, dim3((h->n + WAVE / 16 - 1) / (WAVE / 16)), dim3(WAVE), 0, s, m, h->d, gate,
                     h->pair_heavy_pct);
  hipLaunchKernelGGL(pair_rings_kernel, dim3(1), dim3(64), 0, s, h->d, gate);
  if (ro) {  // a rollout: the one-launch form (launch_rollout only comes here with pair_one)
    hipLaunchKernelGGL((relief_pair1_kernel<T, true>), dim3(h->pair_cap), dim3(WAVE), plb, s, m, h->cfg, h->d,
                       (const float*)nullptr, ro->T, (float*)nullptr, (float*)nullptr, (uint8_t*)nullptr,
                       (float*)nullptr, (float*)nullptr, 1, h->pair_seg, h->pair_budget, gate, *ro);
  } else if (h->pair_one) {
    hipLaunchKernelGGL((relief_pair1_kernel<T, false>), dim3(h->pair_cap), dim3(WAVE), plb, s, m, h->cfg, h->d, a, K, o,
                       r, dn, t, p2, ar, h->pair_seg, h->pair_budget, gate, RolloutDev{});
  } else {
    HIPCHK(hipEventRecord(h->fork, s));
    HIPCHK(hipStreamWaitEvent(h->side, h->fork, 0));
    hipLaunchKernelGGL((relief_pair_kernel<T, true>), dim3(h->pair_cap), dim3(WAVE), plb, h->side, m, h->cfg, h->d, a,
                       K, o, r, dn, t, p2, ar, h->pair_seg, h->pair_budget, gate);
    hipLaunchKernelGGL((relief_pair_kernel<T, false>), dim3(h->pair_cap), dim3(WAVE), plb, s, m, h->cfg, h->d, a, K, o,
                       r, dn, t, p2, ar, h->pair_seg, h->pair_budget, gate);
    HIPCHK(hipEventRecord(h->join, h->side));
    HIPCHK(hipStreamWaitEvent(s, h->join, 0));
  }
  if (h->pair_adapt) hipLaunchKernelGGL(pair_adapt_kernel, dim3(1), dim3(64), 0, s, h->d, h->pair_cap, gate);
  return 0;
}

}  // namespace

// The relief pair's kernels and their launch are compiled a second time in
// their own translation unit, bb_pair.hip (this file with BB_PAIR_TU), with
// -mllvm -disable-machine-licm: in the persistent loop MachineLICM hoists the
// ocml atan2/acos/sin/cos polynomial constants out of the loop and then
// spills them, and every call reloads ~20 of them one dependent scratch load
// at a time (448 B of scratch per lane; 16 B without the hoisting).  The
// other kernels keep the default (flat's multi-step kernel is 2% slower
// without it).  Both units compile the same source, so the structures agree.
// (internal to the library: hidden, not part of the C-ABI)
extern "C" __attribute__((visibility("hidden"))) int bb_pair_launch_tu(bb_handle* h, int fp64, const float* a, int K,
                                                                      float* o, float* r, uint8_t* dn, float* t,
                                                                      float* p2, int ar, hipStream_t s,
                                                                      const int* gate, const void* ro);
// Once per handle, in the unit whose pair kernels are the ones launched: their dynamic-LDS
// limit, and how many one-wave workgroups of relief_pair1_kernel<T> a CU holds at once
// (*per_cu; the persistent pair's grid is sized from it, bb_create).
extern "C" __attribute__((visibility("hidden"))) int bb_pair_setup_tu(int fp64, int* per_cu);
#ifdef BB_PAIR_TU
template <typename T>
int pair_setup(int* per_cu) {  // -> a hipError_t (this unit's error text is not the C-ABI's)
  const size_t plb = multi_lds_bytes<T>(4);
  const void* ks[4] = {(const void*)relief_pair1_kernel<T, false>, (const void*)relief_pair_kernel<T, false>,
                       (const void*)relief_pair_kernel<T, true>, (const void*)relief_pair1_kernel<T, true>};
  for (const void* k : ks) {
    const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, int(plb));
    if (e != hipSuccess) return int(e);
  }
  // the grid is sized for both one-launch forms (step_multi's and the rollout's)
  int nb = 0, nr = 0;
  hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, ks[0], WAVE, plb);
  if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nr, ks[3], WAVE, plb);
  *per_cu = nb < nr ? nb : nr;
  return int(e);
}
extern "C" __attribute__((visibility("hidden"))) int bb_pair_setup_tu(int fp64, int* per_cu) {
  return fp64 ? pair_setup<double>(per_cu) : pair_setup<float>(per_cu);
}
extern "C" __attribute__((visibility("hidden"))) int bb_pair_launch_tu(bb_handle* h, int fp64, const float* a, int K, float* o, float* r, uint8_t* dn,
                                 float* t, float* p2, int ar, hipStream_t s, const int* gate, const void* ro) {
  const RolloutDev* rd = static_cast<const RolloutDev*>(ro);
  return fp64 ? launch_pair<double>(h, a, K, o, r, dn, t, p2, ar, s, gate, rd)
              : launch_pair<float>(h, a, K, o, r, dn, t, p2, ar, s, gate, rd);
}
#endif

namespace {

template <typename T>
int pair_entry(bb_handle* h, const float* a, int K, float* o, float* r, uint8_t* dn, float* t, float* p2, int ar,
               hipStream_t s, const int* gate) {
  if (bb_pair_launch_tu(h, sizeof(T) == 8, a, K, o, r, dn, t, p2, ar, s, gate, nullptr))
    return fail("bb_step_multi: relief pair launch failed");
  return 0;
}

template <typename T>
int launch_multi(bb_handle* h, const float* a, int K, float* o, float* r, uint8_t* dn, float* t, float* p2, int ar,
                 hipStream_t s) {
  const int epw = h->epw;
  const int blocks = (h->n + epw - 1) / epw;
  const bool timed = h->tn < h->tcap;
  hipEvent_t* ev = timed ? &h->tev[6 * h->tn] : nullptr;
  const int route = h->route >= 0 ? h->route : (h->n_relief == 0 ? 1 : 0);
  if (timed) HIPCHK(hipEventRecord(ev[0], s));
  const size_t mlb = multi_lds_bytes<T>(epw);
  if (route == 0 && h->team == 16 && h->multi_queue && h->multi_adapt && h->multi_park) {
    // relief banks, adaptive: the parked launches or the work queue, as the
    // device flag chose after the last launch (the others exit at once)
    const int* gate = h->d.slow_count + SC_ROUTE;
    hipLaunchKernelGGL((multi_step_kernel<T, false>), dim3(blocks), dim3(WAVE), mlb, s, model_of<T>(h), h->cfg, h->d,
                       a, K, o, r, dn, t, p2, ar, h->team, epw, h->d.park, gate);
    hipLaunchKernelGGL((multi_step_kernel<T, true>), dim3(blocks), dim3(WAVE), mlb, s, model_of<T>(h), h->cfg, h->d,
                       a, K, o, r, dn, t, p2, ar, h->team, epw, h->d.park, gate);
    if (h->pair) {
      if (pair_entry<T>(h, a, K, o, r, dn, t, p2, ar, s, gate)) return -1;
    } else {
      const Dev dq = balanced_dev(h, s);
      hipLaunchKernelGGL((relief_multi_kernel<T, false>), dim3((h->n + QENV - 1) / QENV), dim3(64 * QW),
                         relief_lds_bytes<T>(), s, model_of<T>(h), h->cfg, dq, a, K, o, r, dn, t, p2, ar,
                         RolloutDev{}, gate);
    }
    if (timed) HIPCHK(hipEventRecord(ev[1], s));
    hipLaunchKernelGGL(route_decide_kernel, dim3(1), dim3(64), 0, s, h->d.slow_count, 1);
  } else if (route == 0 && h->team == 16 && h->multi_queue) {  // relief banks: the work queue
    if (h->pair) {
      if (pair_entry<T>(h, a, K, o, r, dn, t, p2, ar, s, (const int*)nullptr)) return -1;
    } else {
      const Dev dq = balanced_dev(h, s);
      hipLaunchKernelGGL((relief_multi_kernel<T, false>), dim3((h->n + QENV - 1) / QENV), dim3(64 * QW),
                         relief_lds_bytes<T>(), s, model_of<T>(h), h->cfg, dq, a, K, o, r, dn, t, p2, ar,
                         RolloutDev{}, (const int*)nullptr);
    }
    if (timed) HIPCHK(hipEventRecord(ev[1], s));
  } else if (h->multi_park) {  // the fast steps, then the parked envs' hand-overs and the rest of their steps
    hipLaunchKernelGGL((multi_step_kernel<T, false>), dim3(blocks), dim3(WAVE), mlb, s, model_of<T>(h), h->cfg, h->d,
                       a, K, o, r, dn, t, p2, ar, h->team, epw, h->d.park, (const int*)nullptr);
    if (timed) HIPCHK(hipEventRecord(ev[1], s));
    hipLaunchKernelGGL((multi_step_kernel<T, true>), dim3(blocks), dim3(WAVE), mlb, s, model_of<T>(h), h->cfg, h->d,
                       a, K, o, r, dn, t, p2, ar, h->team, epw, h->d.park, (const int*)nullptr);
  } else {
    hipLaunchKernelGGL((multi_step_kernel<T, true>), dim3(blocks), dim3(WAVE), mlb, s, model_of<T>(h), h->cfg, h->d,
                       a, K, o, r, dn, t, p2, ar, h->team, epw, (int*)nullptr, (const int*)nullptr);
    if (timed) HIPCHK(hipEventRecord(ev[1], s));
  }
  if (timed) {
    HIPCHK(hipEventRecord(ev[5], s));
    h->tpred[h->tn] = 0;
    h->tn++;
  }
  HIPCHK(hipGetLastError());
  return 0;
}
}  // namespace

#ifndef BB_PAIR_TU
extern "C" {

int bb_abi_version(void) { return BB_ABI_VERSION; }

int bb_last_error(char* buf, int len) {
  if (buf && len > 0) { strncpy(buf, g_err, len - 1); buf[len - 1] = 0; }
  return (int)strlen(g_err);
}

void bb_default_params(bb_params* p) {
  memset(p, 0, sizeof *p);
  p->max_ep_steps = 4000;
  p->max_allowed_tilt = 20.f;
  p->max_wheel_velocity = 10.f;
  p->reward_scale = 0.01f;
  p->action_reg_coef = -0.0001f;
  p->survival_bonus = 0.02f;
  p->target_dir[0] = 0.f; p->target_dir[1] = 1.f;
  p->reward_kind = BB_REWARD_DIRECTIONAL;
  p->goal_scale = 1.f;
  p->n_terrains = 1;
  p->seed = 0;
  p->fp64 = 1;  // fp64 arithmetic by default (parity 1e-9); fp32 opt-in
}

int bb_create(int n_envs, int device, const bb_params* p, bb_handle** out) {
  if (!out) return fail("bb_create: out is NULL");
  *out = nullptr;
  if (n_envs <= 0) return fail("bb_create: n_envs must be > 0 (got %d)", n_envs);
  bb_params pp;
  if (p) pp = *p; else bb_default_params(&pp);
  if (pp.n_terrains < 1) return fail("bb_create: n_terrains must be >= 1");
  if (!(pp.opt_timestep >= 0 && pp.opt_timestep <= 0.1))
    return fail("bb_create: opt_timestep %g out of range [0, 0.1] (0: ballbot.xml's 0.002)", pp.opt_timestep);
  if (pp.opt_disableflags & ~(BB_DSBL_PASSIVE | BB_DSBL_GRAVITY))
    return fail("bb_create: opt_disableflags 0x%x: only BB_DSBL_PASSIVE and BB_DSBL_GRAVITY are supported",
                pp.opt_disableflags);
  int ndev = 0;
  HIPCHK(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail("bb_create: device %d out of range (%d devices)", device, ndev);
  HIPCHK(hipSetDevice(device));
  bb_handle* h = new bb_handle();
  h->n = n_envs; h->device = device; h->fp64 = pp.fp64 ? 1 : 0; h->p = pp;
  EnvCfg& c = h->cfg;
  c.max_ep_steps = pp.max_ep_steps; c.max_allowed_tilt = pp.max_allowed_tilt;
  c.max_wheel_velocity = pp.max_wheel_velocity; c.reward_scale = pp.reward_scale;
  c.action_reg_coef = pp.action_reg_coef; c.survival_bonus = pp.survival_bonus;
  c.target[0] = pp.target_dir[0]; c.target[1] = pp.target_dir[1];
  c.reward_kind = pp.reward_kind; c.goal[0] = pp.goal[0]; c.goal[1] = pp.goal[1]; c.goal_scale = pp.goal_scale;
  SolverCfg sc = default_solver(h->fp64);
  if (pp.solver_maxiter > 0) sc.maxiter = pp.solver_maxiter;
  if (pp.solver_tol > 0) sc.tol = pp.solver_tol;
  // team size L (lanes per env) and envs per wave: aim for at least one wave
  // per SIMD (4 per CU) across the whole chip
  {
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, device));
    const int simds = prop.multiProcessorCount * 4;
    const int L = TEAM;  // one DPP row per env (bb_team16.h)
    // LDS caps envs per wave: one EnvWork per team + the staged model
    const size_t lds_max = 160 * 1024 - 2048;
    const int cap = (int)(lds_max / (h->fp64 ? work_stride<double>() : work_stride<float>()));
    int epw = 1;
    while (epw < WAVE / L && (long)epw * simds < (long)n_envs) epw *= 2;
    const char* ov = getenv("BB_EPW");
    if (ov && atoi(ov) > 0) epw = atoi(ov);
    if (epw > WAVE / L) epw = WAVE / L;
    if (epw > cap) epw = cap;
    h->team = L;
    h->epw = epw;
    // envs per wave of the full kernel: the same as the fast kernel's by
    // default.  Fewer (BB_EPW_FULL=1, 2) spread the full lists over more SIMDs
    // but cost more issue slots in total: perlin 1.51 M (1), 1.67 M (2),
    // 1.78 M (4) env-steps/s -- the step kernels are issue-bound, not latency-bound
    int epf = epw;
    const char* of = getenv("BB_EPW_FULL");
    if (of && atoi(of) > 0) epf = atoi(of);
    if (epf > epw) epf = epw;
    h->epw_full = epf;
    const char* rt = getenv("BB_ROUTE");
    if (rt) h->route = atoi(rt);
    const char* ad = getenv("BB_MULTI_ADAPT");
    if ((ad && atoi(ad) == 0) || rt || getenv("BB_MULTI_QUEUE")) h->multi_adapt = 0;
    const char* mp = getenv("BB_MULTI_PARK");
    if (mp) h->multi_park = atoi(mp) != 0;
    const char* mq = getenv("BB_MULTI_QUEUE");
    if (mq) h->multi_queue = atoi(mq) != 0;
    const char* bl = getenv("BB_BALANCE");
    if (bl) h->balance = atoi(bl) != 0;
    const char* cm = getenv("BB_COUNT_MEMSET");
    if (cm) h->count_memset = atoi(cm) != 0;
    const char* rp = getenv("BB_RELIEF_PAIR");
    if (rp) h->pair = atoi(rp) != 0;
    const char* ps = getenv("BB_PAIR_SEG");
    if (ps && atoi(ps) > 0) h->pair_seg = atoi(ps);
    const char* pa = getenv("BB_PAIR_ADAPT");
    if (pa) h->pair_adapt = atoi(pa) != 0;
    // the persistent pair needs its whole grid resident: as many one-wave workgroups as the
    // CUs hold at once (4 per CU: one 512-VGPR wave per SIMD), whole groups of NXCD
    int per_cu = 0;
    const int pe = bb_pair_setup_tu(h->fp64, &per_cu);
    if (pe) return fail("bb_create: relief pair setup: %s", hipGetErrorString(hipError_t(pe)));
    if (per_cu > 4) per_cu = 4;
    h->pair_cap = prop.multiProcessorCount * per_cu / NXCD * NXCD;
    if (h->pair_cap < 16 * NXCD) h->pair = 0;  // too small a chip for the pair: the one-launch work queue
    int wrate = 0;  // kHz
    if (hipDeviceGetAttribute(&wrate, hipDeviceAttributeWallClockRate, device) != hipSuccess || wrate <= 0)
      wrate = 100000;
    const char* po = getenv("BB_PAIR_ONE");
    if (po) h->pair_one = atoi(po) != 0;
    const char* so = getenv("BB_PAIR_SOLO");
    if (so) h->pair_solo = atoi(so) > 0 ? atoi(so) : 0;
    // the solo workgroups are the first full-kind ones: keep a whole group of non-solo full
    // workgroups (every XCD label) inside the adapt floor of pair_cap / 8
    if (h->pair_solo > h->pair_cap / 8 - NXCD) h->pair_solo = h->pair_cap / 8 - NXCD;
    if (h->pair_solo < 0) h->pair_solo = 0;
    const char* hv = getenv("BB_PAIR_HEAVY");
    if (hv && atoi(hv) > 0) h->pair_heavy_pct = atoi(hv);
    const char* pb = getenv("BB_PAIR_BUDGET_MS");  // diagnostics (profilers that serialise launches)
    const unsigned long long ms = pb && atoll(pb) > 0 ? (unsigned long long)atoll(pb) : 20000ull;
    h->pair_budget = ms * (unsigned long long)wrate;
    h->pair_budget_s = double(ms) * 1e-3;
  }
  OptCfg oc;
  if (pp.opt_timestep > 0) oc.timestep = pp.opt_timestep;
  oc.disable = pp.opt_disableflags;
  h->md = compile_model(sc, oc);
  h->mf = cast_model<float>(h->md);
  // cam_k: body cam_k_body (pos (+-0.17, -0.01, -0.06), euler 180 -+30 0) and
  // camera euler 180 0 0 in it (ballbot.xml:44-54)
  for (int cam = 0; cam < 2; cam++) {
    double qb[4], qc[4], q[4], R[9];
    bb::detail::euler_quat(qb, 180, cam == 0 ? -30 : 30, 0);
    bb::detail::euler_quat(qc, 180, 0, 0);
    qmul(q, qb, qc);
    q2mat(R, q);
    const double p[3] = {cam == 0 ? 0.17 : -0.17, -0.01, -0.06};
    for (int i = 0; i < 3; i++) h->rig.p[cam][i] = float(p[i]);
    for (int i = 0; i < 9; i++) h->rig.R[cam][i] = float(R[i]);
  }
  const size_t es = h->fp64 ? sizeof(double) : sizeof(float);
  const size_t n = n_envs, nt = pp.n_terrains;
  Dev& d = h->d;
  memset(&d, 0, sizeof d);
  d.n = n_envs; d.n_terrains = pp.n_terrains;
  HIPCHK(hipMalloc(&d.qpos, es * NQ * n));
  HIPCHK(hipMalloc(&d.qvel, es * NV * n));
  HIPCHK(hipMalloc(&d.warm, es * NV * n));
  HIPCHK(hipMalloc((void**)&d.steps, sizeof(int) * n));
  HIPCHK(hipMalloc((void**)&d.terrain, sizeof(int) * n));
  HIPCHK(hipMalloc((void**)&d.pending_terrain, sizeof(int) * n));
  HIPCHK(hipMalloc((void**)&d.episodes, sizeof(int) * n));
  HIPCHK(hipMalloc((void**)&d.tseed, sizeof(int) * n));
  HIPCHK(hipMemset(d.tseed, 0xFF, sizeof(int) * n));  // -1: no device draw yet
  HIPCHK(hipMalloc((void**)&h->tsrc_dev, sizeof(TerrainSrc)));
  HIPCHK(hipMemcpy(h->tsrc_dev, &h->tsrc, sizeof(TerrainSrc), hipMemcpyHostToDevice));  // no draws: terrain 0
  d.tsrc = h->tsrc_dev;
  HIPCHK(hipMalloc((void**)&h->bank, sizeof(float) * nt * HF_N * HF_N));
  HIPCHK(hipMalloc((void**)&h->size_z, sizeof(float) * nt));
  HIPCHK(hipMalloc((void**)&h->offset, sizeof(float) * nt));
  HIPCHK(hipMalloc((void**)&h->hmax, sizeof(float) * nt));
  HIPCHK(hipMemset(h->hmax, 0, sizeof(float) * nt));
  HIPCHK(hipMalloc((void**)&d.stats, sizeof(unsigned long long) * 8));
  HIPCHK(hipMalloc((void**)&d.slow_list, sizeof(int) * n));
  HIPCHK(hipMalloc((void**)&d.park, sizeof(int) * n));
  HIPCHK(hipMalloc((void**)&d.slow_count, sizeof(int) * 64));  // 4 used; a 256-B block of its own
  HIPCHK(hipMemset(d.slow_count, 0, sizeof(int) * 64));
  HIPCHK(hipMalloc((void**)&d.fast_envs, sizeof(int) * n));
  HIPCHK(hipMalloc((void**)&d.pred_envs, sizeof(int) * n));
  HIPCHK(hipMalloc((void**)&d.pred_mark, n));
  HIPCHK(hipMalloc(&d.body_spill, es * (MAXB - MAXB_LDS) * NBF * size_t(n)));
  HIPCHK(hipMalloc(&d.hand, es * HAND * size_t(n)));
  HIPCHK(hipMalloc((void**)&d.perm, sizeof(int) * n));
  // per ring: an XCD label's envs (32-env blocks) + its resident teams, with margin (the solo ring
  // holds at most SC_SOLO envs)
  {
    const int ring_min = (n + 255) / 256 * 32 + WAVE / TEAM * ((h->pair_cap + NXCD - 1) / NXCD) + 1;
    d.ring_len = ring_min + 63;
    // BB_RING_LEN (tests): a shorter ring, never below the bound above (envs + resident teams of
    // one XCD label + 1), so that the rings wrap more laps per launch at the bound itself
    const char* rl = getenv("BB_RING_LEN");
    if (rl && atoi(rl) > 0) d.ring_len = atoi(rl) < ring_min ? ring_min : atoi(rl);
  }
  HIPCHK(hipMalloc((void**)&d.ring, sizeof(unsigned long long) * NRINGS * size_t(d.ring_len)));
  HIPCHK(hipMalloc((void**)&d.rctr, sizeof(int) * 2 * NRINGS));
  HIPCHK(hipMalloc((void**)&d.pair_busy, sizeof(unsigned long long) * 6));
  HIPCHK(hipMalloc((void**)&d.pair_env, sizeof(unsigned long long) * 2 * size_t(n)));
  HIPCHK(hipMemset(d.pair_env, 0, sizeof(unsigned long long) * 2 * size_t(n)));
  {  // the relief pair's first split of the resident workgroups (BB_PAIR_FULL: percent full; default half)
    const char* pf = getenv("BB_PAIR_FULL");
    int pct = pf ? atoi(pf) : 50;
    pct = pct < 13 ? 13 : (pct > 87 ? 87 : pct);
    const int G = h->pair_cap / NXCD, lo = (G + 7) / 8;
    int gs = G * pct / 100;
    gs = gs < lo ? lo : (gs > G - lo ? G - lo : gs);
    int act[2] = {(G - gs) * NXCD, gs * NXCD};  // whole groups (pair_kind_of)
    HIPCHK(hipMemcpy(d.slow_count + SC_ACTIVE, act, sizeof act, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(d.slow_count + SC_SOLO, &h->pair_solo, sizeof(int), hipMemcpyHostToDevice));
  }
  HIPCHK(hipMalloc((void**)&d.cost, sizeof(unsigned long long) * n));
  // sticky fault word in host memory mapped into the device: a relief-pair launch that ends on its
  // budget sets it, and every later call (and bb_check) reports it without a device sync
  HIPCHK(hipHostMalloc((void**)&h->fault_host, sizeof(int), hipHostMallocMapped | hipHostMallocCoherent));
  *h->fault_host = 0;
  HIPCHK(hipHostGetDevicePointer((void**)&d.fault, (void*)h->fault_host, 0));
  HIPCHK(hipMemset(d.cost, 0, sizeof(unsigned long long) * n));
  HIPCHK(hipStreamCreateWithFlags(&h->side, hipStreamNonBlocking));
  HIPCHK(hipEventCreateWithFlags(&h->fork, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&h->join, hipEventDisableTiming));
  HIPCHK(hipMemset(d.steps, 0, sizeof(int) * n));
  HIPCHK(hipMemset(d.terrain, 0, sizeof(int) * n));
  HIPCHK(hipMemset(d.pending_terrain, 0xFF, sizeof(int) * n));  // -1: no pin
  HIPCHK(hipMemset(d.episodes, 0, sizeof(int) * n));
  HIPCHK(hipMemset(h->bank, 0, sizeof(float) * nt * HF_N * HF_N));
  HIPCHK(hipMemset(d.stats, 0, sizeof(unsigned long long) * 8));
  // default: every terrain flat (terrain/__init__.py:32-34), size_z 2.0 (ballbot.xml:23)
  std::vector<float> sz(nt, 2.0f);
  h->h_offset.assign(nt, 0.01f);
  h->relief.assign(nt, 0);
  h->n_relief = 0;
  HIPCHK(hipMemcpy(h->size_z, sz.data(), sizeof(float) * nt, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(h->offset, h->h_offset.data(), sizeof(float) * nt, hipMemcpyHostToDevice));
  d.bank = h->bank; d.size_z = h->size_z; d.offset = h->offset; d.hmax = h->hmax;
  // LDS for the ground-contact store (f64: 120 KiB, above the 64 KiB default)
  {
    const int lb = (int)(h->fp64 ? lds_bytes<double>(h->epw) : lds_bytes<float>(h->epw));
    const void* sk = h->fp64 ? (const void*)step_kernel<double, false> : (const void*)step_kernel<float, false>;
    const void* sk2 = h->fp64 ? (const void*)step_kernel<double, true> : (const void*)step_kernel<float, true>;
    HIPCHK(hipFuncSetAttribute(sk2, hipFuncAttributeMaxDynamicSharedMemorySize, lb));
    const void* fk = h->fp64 ? (const void*)forward_kernel<double> : (const void*)forward_kernel<float>;
    HIPCHK(hipFuncSetAttribute(sk, hipFuncAttributeMaxDynamicSharedMemorySize, lb));
    HIPCHK(hipFuncSetAttribute(fk, hipFuncAttributeMaxDynamicSharedMemorySize, lb));
    const int mlb = (int)(h->fp64 ? multi_lds_bytes<double>(h->epw) : multi_lds_bytes<float>(h->epw));
    const void* mk[2] = {h->fp64 ? (const void*)multi_step_kernel<double, false>
                                 : (const void*)multi_step_kernel<float, false>,
                         h->fp64 ? (const void*)multi_step_kernel<double, true>
                                 : (const void*)multi_step_kernel<float, true>};
    for (const void* k : mk) HIPCHK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, mlb));
    const int rlb = (int)(h->fp64 ? rollout_lds_bytes<double>(h->epw) : rollout_lds_bytes<float>(h->epw));
    const void* rk[2] = {h->fp64 ? (const void*)rollout_kernel<double, false> : (const void*)rollout_kernel<float, false>,
                         h->fp64 ? (const void*)rollout_kernel<double, true> : (const void*)rollout_kernel<float, true>};
    for (const void* k : rk) HIPCHK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, rlb));
    const int qlb = (int)(h->fp64 ? relief_lds_bytes<double>() : relief_lds_bytes<float>());
    const void* qk[2] = {h->fp64 ? (const void*)relief_multi_kernel<double, false>
                                 : (const void*)relief_multi_kernel<float, false>,
                         h->fp64 ? (const void*)relief_multi_kernel<double, true>
                                 : (const void*)relief_multi_kernel<float, true>};
    for (const void* k : qk) HIPCHK(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, qlb));
    // (the relief pair's kernels get theirs in their own unit: bb_pair_setup_tu)
  }
  *out = h;
  int rc = bb_reset(h, nullptr, nullptr, nullptr);
  if (rc) return rc;
  HIPCHK(hipDeviceSynchronize());
  return 0;
}

int bb_destroy(bb_handle* h) {
  if (!h) return 0;
  (void)hipSetDevice(h->device);
  (void)hipFree(h->d.qpos); (void)hipFree(h->d.qvel); (void)hipFree(h->d.warm);
  (void)hipFree(h->d.steps); (void)hipFree(h->d.terrain); (void)hipFree(h->d.pending_terrain); (void)hipFree(h->d.episodes);
  (void)hipFree(h->bank); (void)hipFree(h->size_z); (void)hipFree(h->offset); (void)hipFree(h->hmax); (void)hipFree(h->d.stats);
  (void)hipFree(h->d.slow_list); (void)hipFree(h->d.slow_count); (void)hipFree(h->d.park);
  (void)hipFree(h->d.fast_envs); (void)hipFree(h->d.pred_envs); (void)hipFree(h->d.pred_mark);
  (void)hipFree(h->d.body_spill); (void)hipFree(h->d.hand); (void)hipFree(h->d.perm); (void)hipFree(h->d.cost); (void)hipFree(h->d.ring); (void)hipFree(h->d.rctr);
  (void)hipFree(h->d.pair_busy); (void)hipFree(h->d.pair_env);
  (void)hipFree(h->tstream); (void)hipFree(h->env_stream); (void)hipFree(h->rng); (void)hipFree(h->seed_slot);
  (void)hipFree(h->d.tseed); (void)hipFree(h->tsrc_dev);
  (void)hipStreamDestroy(h->side); (void)hipEventDestroy(h->fork); (void)hipEventDestroy(h->join);
  for (hipEvent_t e : h->tev) (void)hipEventDestroy(e);
  (void)hipFree(h->scenes);
  if (h->fault_host) (void)hipHostFree((void*)h->fault_host);
  delete h;
  return 0;
}

static void set_relief(bb_handle* h, int t, bool r) {
  h->n_relief += int(r) - int(h->relief[t]);
  h->relief[t] = r ? 1 : 0;
}

int bb_set_hfield(bb_handle* h, int terrain_id, const float* data, float size_z) {
  if (!h) return fail("bb_set_hfield: NULL handle");
  if (terrain_id < 0 || terrain_id >= h->p.n_terrains)
    return fail("bb_set_hfield: terrain_id %d out of range [0,%d)", terrain_id, h->p.n_terrains);
  if (!data) return fail("bb_set_hfield: NULL data");
  if (!(size_z > 0)) return fail("bb_set_hfield: size_z must be > 0");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipMemcpy(h->bank + size_t(terrain_id) * HF_N * HF_N, data, sizeof(float) * HF_N * HF_N,
                   hipMemcpyHostToDevice));
  float off = init_offset(data, size_z);
  h->h_offset[terrain_id] = off;
  float hm = 0.f;
  for (int i = 0; i < HF_N * HF_N; i++) hm = data[i] > hm ? data[i] : hm;
  HIPCHK(hipMemcpy(h->hmax + terrain_id, &hm, sizeof(float), hipMemcpyHostToDevice));
  set_relief(h, terrain_id, hm > 0.f);
  HIPCHK(hipMemset(h->d.slow_count + SC_ROUTE, 0, sizeof(int)));  // a new bank: the adaptive route restarts at the queue
  HIPCHK(hipMemcpy(h->size_z + terrain_id, &size_z, sizeof(float), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(h->offset + terrain_id, &off, sizeof(float), hipMemcpyHostToDevice));
  return 0;
}

int bb_generate_perlin(bb_handle* h, int first, int count, const int32_t* seeds, const bb_perlin_cfg* cfg,
                       float size_z) {
  static_assert(HF_N == HF_N_, "terrain generator and physics disagree on the hfield size");
  if (!h || !seeds || !cfg) return fail("bb_generate_perlin: NULL argument");
  if (count < 0 || first < 0 || first + count > h->p.n_terrains)
    return fail("bb_generate_perlin: slots [%d,%d) out of range [0,%d)", first, first + count, h->p.n_terrains);
  if (!(cfg->scale > 0) || cfg->octaves < 1) return fail("bb_generate_perlin: need scale > 0 and octaves >= 1");
  if (!(size_z > 0)) return fail("bb_generate_perlin: size_z must be > 0");
  if (count == 0) return 0;
  HIPCHK(hipSetDevice(h->device));
  int32_t* ds = nullptr;
  HIPCHK(hipMalloc(&ds, sizeof(int32_t) * count));
  HIPCHK(hipMemcpy(ds, seeds, sizeof(int32_t) * count, hipMemcpyHostToDevice));
  PerlinCfg pc{cfg->scale, cfg->octaves, cfg->persistence, cfg->lacunarity, cfg->amplitude};
  std::vector<float> sz(count, size_z);
  HIPCHK(hipMemcpy(h->size_z + first, sz.data(), sizeof(float) * count, hipMemcpyHostToDevice));
  int rc = launch_perlin_bank(h->bank + size_t(first) * HF_N * HF_N, ds, count, pc, size_z, h->offset + first,
                              h->hmax + first, 0);
  HIPCHK(hipDeviceSynchronize());
  (void)hipFree(ds);
  if (rc) return fail("bb_generate_perlin: launch failed");
  HIPCHK(hipMemcpy(h->h_offset.data() + first, h->offset + first, sizeof(float) * count, hipMemcpyDeviceToHost));
  std::vector<float> hm(count);
  HIPCHK(hipMemcpy(hm.data(), h->hmax + first, sizeof(float) * count, hipMemcpyDeviceToHost));
  for (int i = 0; i < count; i++) set_relief(h, first + i, hm[i] > 0.f);
  HIPCHK(hipMemset(h->d.slow_count + SC_ROUTE, 0, sizeof(int)));  // a new bank: the adaptive route restarts at the queue
  return 0;
}

int bb_gae(const float* rew, const float* val, const uint8_t* start, const float* last_val, const uint8_t* last_done,
           int T, int n, double gamma, double lam, float* adv, float* ret, void* stream) {
  if (!rew || !val || !start || !last_val || !last_done || !adv || !ret) return fail("bb_gae: NULL argument");
  if (T < 1 || n < 1) return fail("bb_gae: need T >= 1 and n_envs >= 1 (got %d, %d)", T, n);
  if (launch_gae(rew, val, start, last_val, last_done, T, n, gamma, lam, adv, ret, (hipStream_t)stream))
    return fail("bb_gae: launch failed: %s", hipGetErrorString(hipGetLastError()));
  return 0;
}

int bb_render_depth(bb_handle* h, float* depth, float* rel_ts, int height, int width, int every, int force,
                    void* stream) {
  if (!h || !depth) return fail("bb_render_depth: NULL argument");
  if (height < 1 || width < 1 || height > 1024 || width > 1024)
    return fail("bb_render_depth: image size %dx%d out of range [1,1024]", height, width);
  if (every < 1) return fail("bb_render_depth: frame interval must be >= 1 step (got %d)", every);
  HIPCHK(hipSetDevice(h->device));
  RenderDev rd{h->n, h->d.qpos, h->d.steps, h->d.terrain, h->bank, h->size_z, h->hmax};
  if (!h->scenes) HIPCHK(hipMalloc(&h->scenes, scene_bytes(h->n)));
  if (launch_depth(h->fp64 != 0, h->mf, h->rig, rd, height, width, every, force, float(h->md.h), h->scenes, depth, rel_ts,
                   (hipStream_t)stream))
    return fail("bb_render_depth: launch failed: %s", hipGetErrorString(hipGetLastError()));
  return 0;
}

int bb_ppo_loss(const float* mean, const float* values, const float* log_std, const float* actions,
                const float* old_logp, const float* adv, const float* returns, const float* clip, int B, int normalize,
                float ent_coef, float vf_coef, float* terms, float* grad_mean, float* grad_values, void* stream) {
  if (!mean || !values || !log_std || !actions || !old_logp || !adv || !returns || !clip || !terms || !grad_mean ||
      !grad_values)
    return fail("bb_ppo_loss: NULL argument");
  if (B < 1) return fail("bb_ppo_loss: B must be >= 1 (got %d)", B);
  PPOLossArgs a{mean, values, log_std, actions, old_logp, adv, returns, clip, B, normalize ? 1 : 0, ent_coef, vf_coef,
                terms, grad_mean, grad_values};
  if (launch_ppo_loss(a, (hipStream_t)stream))
    return fail("bb_ppo_loss: launch failed: %s", hipGetErrorString(hipGetLastError()));
  return 0;
}

int bb_adamw_clip(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n, const float* lr,
                  float* step, float* coef, double beta1, double beta2, double eps, double weight_decay,
                  double max_norm, void* stream) {
  if (!param || !grad || !exp_avg || !exp_avg_sq || !lr || !step || !coef) return fail("bb_adamw_clip: NULL argument");
  if (n < 1) return fail("bb_adamw_clip: n must be >= 1 (got %lld)", (long long)n);
  if (!(beta1 >= 0.0 && beta1 < 1.0) || !(beta2 >= 0.0 && beta2 < 1.0))
    return fail("bb_adamw_clip: betas must be in [0, 1) (got %g, %g)", beta1, beta2);
  if (!(eps >= 0.0) || !(max_norm > 0.0)) return fail("bb_adamw_clip: eps must be >= 0 and max_norm > 0");
  if ((reinterpret_cast<uintptr_t>(grad) & 15) != 0) return fail("bb_adamw_clip: grad must be 16-byte aligned");
  AdamWArgs a{param, grad, exp_avg, exp_avg_sq, (long long)n, lr, step, coef, beta1, beta2, weight_decay,
              float(beta2), float(1.0 - beta1), float(1.0 - beta2), float(eps), float(max_norm),
              nullptr, 0};
  if (launch_adamw_clip(a, (hipStream_t)stream))
    return fail("bb_adamw_clip: launch failed: %s", hipGetErrorString(hipGetLastError()));
  return 0;
}

int bb_ppo_mlp_workspace_bytes(int B, int64_t* bytes) {
  if (!bytes) return fail("bb_ppo_mlp_workspace_bytes: NULL argument");
  if (B < 256 || B % 256 || B > 16384)
    return fail("bb_ppo_mlp_workspace_bytes: B must be a multiple of 256 in [256, 16384] (got %d)", B);
  *bytes = mlp_workspace_bytes(B);
  return 0;
}

int bb_ppo_mlp_step(const bb_ppo_mlp_args* a, void* stream) {
  if (!a) return fail("bb_ppo_mlp_step: NULL argument");
  if (!a->params || !a->grad || !a->exp_avg || !a->exp_avg_sq || !a->obs || !a->actions || !a->old_logp ||
      !a->advantages || !a->returns || !a->perm || !a->mb_counter || !a->row_counter || !a->log || !a->clip ||
      !a->lr || !a->step || !a->coef || !a->workspace)
    return fail("bb_ppo_mlp_step: NULL argument");
  if (a->B < 256 || a->B % 256 || a->B > 16384)
    return fail("bb_ppo_mlp_step: B must be a multiple of 256 in [256, 16384] (got %d)", a->B);
  if (a->workspace_bytes < mlp_workspace_bytes(a->B))
    return fail("bb_ppo_mlp_step: workspace of %lld bytes < %lld", (long long)a->workspace_bytes,
                mlp_workspace_bytes(a->B));
  if (!(a->beta1 >= 0.0 && a->beta1 < 1.0) || !(a->beta2 >= 0.0 && a->beta2 < 1.0) || !(a->eps >= 0.0) ||
      !(a->max_grad_norm > 0.0))
    return fail("bb_ppo_mlp_step: bad optimiser hyper-parameters");
  // sizes of the 21 tensors: their extents must fit the flat buffer, 16-byte aligned
  if (a->obs_dim != 15 && a->obs_dim != 56) return fail("bb_ppo_mlp_step: obs_dim must be 15 or 56 (got %d)", a->obs_dim);
  const int sizes[MLP_NSLOTS] = {128 * a->obs_dim, 128 * 128, 128 * 128, 128 * 128, 128, 128, 128, 128,
                                 128 * a->obs_dim, 128 * 128, 128 * 128, 128 * 128, 128, 128, 128, 128,
                                 3 * 128, 3, 128, 1, 3};
  for (int i = 0; i < MLP_NSLOTS; i++)
    if (a->offsets[i] < 0 || a->offsets[i] % 4 || (int64_t)a->offsets[i] + sizes[i] > a->n_params)
      return fail("bb_ppo_mlp_step: offsets[%d] = %d is not a 4-aligned slot inside the %lld-float buffer", i,
                  a->offsets[i], (long long)a->n_params);
  if ((reinterpret_cast<uintptr_t>(a->params) | reinterpret_cast<uintptr_t>(a->grad)) & 15)
    return fail("bb_ppo_mlp_step: params and grad must be 16-byte aligned");
  if (a->phase < 0 || a->phase > 2) return fail("bb_ppo_mlp_step: phase must be 0, 1 or 2 (got %d)", a->phase);
  MlpStepArgs m;
  m.params = a->params; m.grad = a->grad; m.exp_avg = a->exp_avg; m.exp_avg_sq = a->exp_avg_sq;
  m.n_params = a->n_params;
  for (int i = 0; i < MLP_NSLOTS; i++) m.off[i] = a->offsets[i];
  m.obs = a->obs; m.actions = a->actions; m.old_logp = a->old_logp; m.adv = a->advantages; m.returns = a->returns;
  m.perm = reinterpret_cast<const long long*>(a->perm);
  m.mb_counter = reinterpret_cast<long long*>(a->mb_counter);
  m.row_counter = reinterpret_cast<long long*>(a->row_counter);
  m.log = a->log; m.clip = a->clip; m.lr = a->lr; m.step = a->step; m.coef = a->coef;
  m.B = a->B; m.normalize = a->normalize_advantage ? 1 : 0; m.in_dim = a->obs_dim; m.obs_direct = a->obs_direct ? 1 : 0; m.ent_coef = a->ent_coef; m.vf_coef = a->vf_coef;
  m.beta1 = a->beta1; m.beta2 = a->beta2; m.eps = a->eps; m.weight_decay = a->weight_decay;
  m.max_norm = a->max_grad_norm; m.ws = a->workspace; m.ws_bytes = a->workspace_bytes;
  m.phase = a->phase; m.adv_stats = a->adv_stats;
  const int rc = launch_mlp_step(m, (hipStream_t)stream);
  if (rc) return fail("bb_ppo_mlp_step: launch failed (%d): %s", rc, hipGetErrorString(hipGetLastError()));
  return 0;
}

int bb_ppo_mlp_act(const float* params, const int32_t* offsets, int64_t n_params, const float* obs, int obs_dim,
                   const float* noise, int n, float* obs_copy, float* actions, float* clipped, float* values,
                   float* log_prob, void* stream) {
  if (!params || !offsets || !obs || !actions || !values || !log_prob) return fail("bb_ppo_mlp_act: NULL argument");
  if (n < 0) return fail("bb_ppo_mlp_act: n must be >= 0 (got %d)", n);
  if (obs_dim != 15 && obs_dim != 56) return fail("bb_ppo_mlp_act: obs_dim must be 15 or 56 (got %d)", obs_dim);
  // the same slot check as bb_ppo_mlp_step: every tensor inside the n_params-float buffer
  const int sizes[MLP_NSLOTS] = {128 * obs_dim, 128 * 128, 128 * 128, 128 * 128, 128, 128, 128, 128,
                                 128 * obs_dim, 128 * 128, 128 * 128, 128 * 128, 128, 128, 128, 128,
                                 3 * 128, 3, 128, 1, 3};
  for (int i = 0; i < MLP_NSLOTS; i++)
    if (offsets[i] < 0 || offsets[i] % 4 || (int64_t)offsets[i] + sizes[i] > n_params)
      return fail("bb_ppo_mlp_act: offsets[%d] = %d is not a 4-aligned slot inside the %lld-float buffer", i,
                  offsets[i], (long long)n_params);
  if (reinterpret_cast<uintptr_t>(params) & 15) return fail("bb_ppo_mlp_act: params must be 16-byte aligned");
  MlpActArgs m;
  m.params = params;
  for (int i = 0; i < MLP_NSLOTS; i++) m.off[i] = offsets[i];
  m.obs = obs; m.in_dim = obs_dim; m.noise = noise; m.n = n; m.obs_copy = obs_copy; m.actions = actions; m.clipped = clipped;
  m.values = values; m.log_prob = log_prob;
  if (launch_mlp_act(m, (hipStream_t)stream))
    return fail("bb_ppo_mlp_act: launch failed: %s", hipGetErrorString(hipGetLastError()));
  return 0;
}

int bb_rollout_track(const float* reward, const uint8_t* flags, int mask, int n, float* rewards_out, double* ep_ret,
                     int64_t* ep_len, double* ep_r_out, int64_t* ep_l_out, uint8_t* starts, uint8_t* starts_next,
                     void* stream) {
  if (!reward || !flags || !rewards_out || !ep_ret || !ep_len || !ep_r_out || !ep_l_out || !starts)
    return fail("bb_rollout_track: NULL argument");
  if (n < 0) return fail("bb_rollout_track: n must be >= 0 (got %d)", n);
  if (launch_track(reward, flags, mask, n, rewards_out, ep_ret, reinterpret_cast<long long*>(ep_len), ep_r_out,
                   reinterpret_cast<long long*>(ep_l_out), starts, starts_next, (hipStream_t)stream))
    return fail("bb_rollout_track: launch failed: %s", hipGetErrorString(hipGetLastError()));
  return 0;
}

int bb_depth_encoder_workspace_bytes(int64_t n, int64_t* bytes) {
  if (!bytes) return fail("bb_depth_encoder_workspace_bytes: NULL argument");
  if (n < 0) return fail("bb_depth_encoder_workspace_bytes: n must be >= 0");
  *bytes = encoder_workspace_bytes(n);
  return 0;
}

int bb_depth_encoder(const bb_encoder_params* p, const float* images, int64_t image_stride, const int64_t* index,
                     int64_t n, int height, int width, int train, float momentum, float eps, float* out,
                     int64_t out_stride, float* ws, int64_t ws_bytes, void* stream) {
  if (!p || !images || !out || !ws) return fail("bb_depth_encoder: NULL argument");
  if (!p->conv1_w || !p->conv1_b || !p->bn1_w || !p->bn1_b || !p->bn1_mean || !p->bn1_var || !p->conv2_w ||
      !p->conv2_b || !p->bn2_w || !p->bn2_b || !p->bn2_mean || !p->bn2_var || !p->fc_w || !p->fc_b || !p->bn3_w ||
      !p->bn3_b || !p->bn3_mean || !p->bn3_var)
    return fail("bb_depth_encoder: NULL parameter pointer");
  if (height != 64 || width != 64) return fail("bb_depth_encoder: only 64x64 images (got %dx%d)", height, width);
  if (n < 0 || (train && n < 2)) return fail("bb_depth_encoder: need n >= 2 in train mode (got %lld)", (long long)n);
  if ((reinterpret_cast<uintptr_t>(images) & 15) || image_stride % 4 || image_stride < 64 * 64)
    return fail("bb_depth_encoder: images must be 16-byte aligned with a stride of >= 4096 floats, a multiple of 4");
  if (out_stride < 20) return fail("bb_depth_encoder: out_stride must be >= 20");
  if (ws_bytes < encoder_workspace_bytes(n))
    return fail("bb_depth_encoder: workspace of %lld bytes < %lld", (long long)ws_bytes, encoder_workspace_bytes(n));
  EncArgs a{};
  a.p = EncParams{p->conv1_w, p->conv1_b, p->bn1_w, p->bn1_b, p->bn1_mean, p->bn1_var,
                  reinterpret_cast<long long*>(p->bn1_count), p->conv2_w, p->conv2_b, p->bn2_w, p->bn2_b,
                  p->bn2_mean, p->bn2_var, reinterpret_cast<long long*>(p->bn2_count), p->fc_w, p->fc_b, p->bn3_w,
                  p->bn3_b, p->bn3_mean, p->bn3_var, reinterpret_cast<long long*>(p->bn3_count)};
  a.images = images; a.image_stride = image_stride; a.index = reinterpret_cast<const long long*>(index);
  a.n = n; a.train = train ? 1 : 0;
  a.momentum = momentum; a.eps = eps; a.out = out; a.out_stride = out_stride;
  if (launch_encoder(a, ws, (hipStream_t)stream))
    return fail("bb_depth_encoder: launch failed: %s", hipGetErrorString(hipGetLastError()));
  return 0;
}

int bb_get_hfield(bb_handle* h, int terrain_id, float* out) {
  if (!h || !out) return fail("bb_get_hfield: NULL argument");
  if (terrain_id < 0 || terrain_id >= h->p.n_terrains)
    return fail("bb_get_hfield: terrain_id %d out of range [0,%d)", terrain_id, h->p.n_terrains);
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(out, h->bank + size_t(terrain_id) * HF_N * HF_N, sizeof(float) * HF_N * HF_N,
                   hipMemcpyDeviceToHost));
  return 0;
}

int bb_assign_terrain(bb_handle* h, const int32_t* ids, void* stream) {
  if (!h || !ids) return fail("bb_assign_terrain: NULL argument");
  HIPCHK(hipSetDevice(h->device));
  hipLaunchKernelGGL(assign_kernel, dim3((h->n + 255) / 256), dim3(256), 0, (hipStream_t)stream, h->d, ids);
  HIPCHK(hipGetLastError());
  return 0;
}

int bb_reset(bb_handle* h, const uint8_t* mask, float* obs, void* stream) {
  if (!h) return fail("bb_reset: NULL handle");
  int blocks = (h->n + WAVE - 1) / WAVE;
  if (h->fp64)
    hipLaunchKernelGGL(reset_kernel<double>, dim3(blocks), dim3(WAVE), 0, (hipStream_t)stream, h->md, h->d, mask, obs);
  else
    hipLaunchKernelGGL(reset_kernel<float>, dim3(blocks), dim3(WAVE), 0, (hipStream_t)stream, h->mf, h->d, mask, obs);
  HIPCHK(hipGetLastError());
  // A full reset clears a budget fault. reset_kernel clears the device word in stream order, but
  // bb_step* read the host side as soon as they are called: with a fault set, wait for the reset
  // so that reset-then-step works without a bb_check in between (no wait when no fault is set,
  // so a captured or asynchronous full reset stays asynchronous).
  if (!mask && *h->fault_host) {
    HIPCHK(hipStreamSynchronize((hipStream_t)stream));
    *h->fault_host = 0;
  }
  return 0;
}

// A relief-pair launch that ended on its wall-clock budget left the envs it had not finished
// with their state at the launch's start but their terrain draws and counters advanced: the
// handle refuses to step until a full bb_reset (which clears the fault on the device).
static int faulted(const bb_handle* h, const char* what) {
  return fail("%s: a bb_step_multi launch ended on its wall-clock budget (an env waited %.0f s for a step that "
              "never came); the envs' states are inconsistent -- bb_reset(h, NULL, ...) clears this",
              what, h->pair_budget_s);
}

int bb_check(bb_handle* h, void* stream) {
  if (!h) return fail("bb_check: NULL handle");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  if (*h->fault_host) return faulted(h, "bb_check");
  return 0;
}

int bb_step(bb_handle* h, const float* a, float* o, float* r, uint8_t* dn, float* t, float* p2, int ar, void* s) {
  if (!h) return fail("bb_step: NULL handle");
  if (*h->fault_host) return faulted(h, "bb_step");
  if (!a || !o || !r || !dn) return fail("bb_step: actions/obs/reward/done must be non-NULL");
  return h->fp64 ? launch_step<double>(h, a, o, r, dn, t, p2, ar, (hipStream_t)s)
                 : launch_step<float>(h, a, o, r, dn, t, p2, ar, (hipStream_t)s);
}

int bb_step_multi(bb_handle* h, const float* a, int k, float* o, float* r, uint8_t* dn, float* t, float* p2, int ar,
                  void* s) {
  if (!h) return fail("bb_step_multi: NULL handle");
  if (*h->fault_host) return faulted(h, "bb_step_multi");
  if (!a || !o || !r || !dn) return fail("bb_step_multi: actions/obs/reward/done must be non-NULL");
  if (k < 1) return fail("bb_step_multi: k_steps must be >= 1 (got %d)", k);
  return h->fp64 ? launch_multi<double>(h, a, k, o, r, dn, t, p2, ar, (hipStream_t)s)
                 : launch_multi<float>(h, a, k, o, r, dn, t, p2, ar, (hipStream_t)s);
}

int bb_rollout(bb_handle* h, const bb_rollout_args* a, void* stream) {
  if (!h) return fail("bb_rollout: NULL handle");
  if (*h->fault_host) return faulted(h, "bb_rollout");
  if (!a || !a->params || !a->noise || !a->obs || !a->last_starts || !a->ep_ret || !a->ep_len || !a->buf_obs ||
      !a->buf_actions || !a->buf_values || !a->buf_log_prob || !a->buf_rewards || !a->buf_starts || !a->ep_r_out ||
      !a->ep_l_out)
    return fail("bb_rollout: NULL argument");
  if (a->n_steps < 1) return fail("bb_rollout: n_steps must be >= 1 (got %d)", a->n_steps);
  if (h->cfg.reward_kind == BB_REWARD_NONE)
    return fail("bb_rollout: the reward is a host-side plugin (BB_REWARD_NONE); step with bb_step instead");
  const int sizes[MLP_NSLOTS] = {128 * 15, 128 * 128, 128 * 128, 128 * 128, 128, 128, 128, 128,
                                 128 * 15, 128 * 128, 128 * 128, 128 * 128, 128, 128, 128, 128,
                                 3 * 128, 3, 128, 1, 3};
  for (int i = 0; i < MLP_NSLOTS; i++)
    if (a->offsets[i] < 0 || a->offsets[i] % 4 || (int64_t)a->offsets[i] + sizes[i] > a->n_params)
      return fail("bb_rollout: offsets[%d] = %d is not a 4-aligned slot inside the %lld-float buffer", i,
                  a->offsets[i], (long long)a->n_params);
  if (reinterpret_cast<uintptr_t>(a->params) & 15) return fail("bb_rollout: params must be 16-byte aligned");
  RolloutDev ro;
  ro.P = a->params;
  for (int i = 0; i < MLP_NSLOTS; i++) ro.off[i] = a->offsets[i];
  ro.noise = a->noise; ro.T = a->n_steps; ro.obs = a->obs; ro.last_starts = a->last_starts; ro.ep_ret = a->ep_ret;
  ro.ep_len = reinterpret_cast<long long*>(a->ep_len); ro.b_obs = a->buf_obs; ro.b_act = a->buf_actions;
  ro.b_val = a->buf_values; ro.b_logp = a->buf_log_prob; ro.b_rew = a->buf_rewards; ro.b_starts = a->buf_starts;
  ro.ep_r = a->ep_r_out; ro.ep_l = reinterpret_cast<long long*>(a->ep_l_out);
  return h->fp64 ? launch_rollout<double>(h, ro, (hipStream_t)stream) : launch_rollout<float>(h, ro, (hipStream_t)stream);
}

int bb_get_state(bb_handle* h, double* qpos, double* qvel, double* warm, int32_t* steps) {
  if (!h) return fail("bb_get_state: NULL handle");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipDeviceSynchronize());
  const size_t n = h->n, es = h->fp64 ? 8 : 4;
  std::vector<unsigned char> buf(es * NQ * n);
  auto conv = [&](void* dsrc, int nf, double* dst) -> int {
    if (!dst) return 0;
    HIPCHK(hipMemcpy(buf.data(), dsrc, es * nf * n, hipMemcpyDeviceToHost));
    for (size_t e = 0; e < n; e++)
      for (int i = 0; i < nf; i++)
        dst[e * nf + i] = h->fp64 ? ((double*)buf.data())[i * n + e] : (double)((float*)buf.data())[i * n + e];
    return 0;
  };
  if (conv(h->d.qpos, NQ, qpos) || conv(h->d.qvel, NV, qvel) || conv(h->d.warm, NV, warm)) return -1;
  if (steps) HIPCHK(hipMemcpy(steps, h->d.steps, sizeof(int) * n, hipMemcpyDeviceToHost));
  return 0;
}

int bb_set_state(bb_handle* h, const double* qpos, const double* qvel, const double* warm, const int32_t* steps) {
  if (!h) return fail("bb_set_state: NULL handle");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipDeviceSynchronize());
  const size_t n = h->n, es = h->fp64 ? 8 : 4;
  std::vector<unsigned char> buf(es * NQ * n);
  auto conv = [&](void* ddst, int nf, const double* src) -> int {
    if (!src) return 0;
    for (size_t e = 0; e < n; e++)
      for (int i = 0; i < nf; i++) {
        if (h->fp64) ((double*)buf.data())[i * n + e] = src[e * nf + i];
        else ((float*)buf.data())[i * n + e] = (float)src[e * nf + i];
      }
    HIPCHK(hipMemcpy(ddst, buf.data(), es * nf * n, hipMemcpyHostToDevice));
    return 0;
  };
  if (conv(h->d.qpos, NQ, qpos) || conv(h->d.qvel, NV, qvel) || conv(h->d.warm, NV, warm)) return -1;
  if (steps) HIPCHK(hipMemcpy(h->d.steps, steps, sizeof(int) * n, hipMemcpyHostToDevice));
  return 0;
}

int bb_forward(bb_handle* h, const double* ctrl, double* qacc, int32_t* ncon) {
  if (!h || !ctrl || !qacc) return fail("bb_forward: NULL argument");
  HIPCHK(hipSetDevice(h->device));
  const size_t n = h->n;
  double *dc = nullptr, *dq = nullptr;
  int* dn = nullptr;
  HIPCHK(hipMalloc(&dc, sizeof(double) * 3 * n));
  HIPCHK(hipMalloc(&dq, sizeof(double) * NV * n));
  HIPCHK(hipMalloc(&dn, sizeof(int) * 2 * n));
  HIPCHK(hipMemcpy(dc, ctrl, sizeof(double) * 3 * n, hipMemcpyHostToDevice));
  const int epw = h->epw;
  int blocks = (h->n + epw - 1) / epw;
  if (h->fp64)
    hipLaunchKernelGGL(forward_kernel<double>, dim3(blocks), dim3(WAVE), lds_bytes<double>(epw), 0, h->md, h->d, dc, dq,
                       dn, h->team, epw);
  else
    hipLaunchKernelGGL(forward_kernel<float>, dim3(blocks), dim3(WAVE), lds_bytes<float>(epw), 0, h->mf, h->d, dc, dq,
                       dn, h->team, epw);
  HIPCHK(hipGetLastError());
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(qacc, dq, sizeof(double) * NV * n, hipMemcpyDeviceToHost));
  if (ncon) HIPCHK(hipMemcpy(ncon, dn, sizeof(int) * 2 * n, hipMemcpyDeviceToHost));
  (void)hipFree(dc); (void)hipFree(dq); (void)hipFree(dn);
  return 0;
}

int bb_get_stats(bb_handle* h, int64_t* out, int n) {
  if (!h || !out) return fail("bb_get_stats: NULL argument");
  if (n < 0 || n > BB_NSTATS) return fail("bb_get_stats: n must be in [0, %d] (got %d)", BB_NSTATS, n);
  HIPCHK(hipSetDevice(h->device));
  unsigned long long s[8];
  HIPCHK(hipMemcpy(s, h->d.stats, sizeof s, hipMemcpyDeviceToHost));
  const int64_t v[BB_NSTATS] = {(int64_t)s[0], (int64_t)s[1], (int64_t)s[2], (int64_t)s[3], (int64_t)s[4],
                                (int64_t)s[5], (int64_t)s[6], (int64_t)s[7]};
  for (int i = 0; i < n; i++) out[i] = v[i];
  return 0;
}

int bb_pair_counters(bb_handle* h, int64_t* out, int n) {
  if (!h || !out) return fail("bb_pair_counters: NULL argument");
  if (n < 0 || n > BB_NPAIR) return fail("bb_pair_counters: n must be in [0, %d] (got %d)", BB_NPAIR, n);
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipDeviceSynchronize());
  int sc[64];
  unsigned long long busy[6];
  HIPCHK(hipMemcpy(sc, h->d.slow_count, sizeof sc, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(busy, h->d.pair_busy, sizeof busy, hipMemcpyDeviceToHost));
  int rc[2 * NRINGS];
  HIPCHK(hipMemcpy(rc, h->d.rctr, sizeof rc, hipMemcpyDeviceToHost));
  int push_min[2] = {INT_MAX, INT_MAX};  // appends to the least-used fast / full ring of the launch
  for (int r = 0; r < 2 * NXCD; r++) push_min[r / NXCD] = std::min(push_min[r / NXCD], rc[2 * r + 1]);
  const int64_t v[BB_NPAIR] = {(int64_t)busy[0], (int64_t)busy[1], sc[SC_IDLE], sc[SC_IDLE + 1], sc[SC_ACTIVE],
                               sc[SC_ACTIVE + 1], sc[SC_CLAIMS], sc[SC_CLAIMS + 1], sc[SC_STEPS], sc[SC_STEPS + 1],
                               sc[SC_PARKED], (int64_t)busy[2], (int64_t)busy[3], (int64_t)busy[4],
                               (int64_t)busy[5], sc[SC_HEAVY_LAST], h->d.ring_len, push_min[0], push_min[1]};
  for (int i = 0; i < n; i++) out[i] = v[i];
  return 0;
}

int bb_pair_env_times(bb_handle* h, uint64_t* out) {
  if (!h || !out) return fail("bb_pair_env_times: NULL argument");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(out, h->d.pair_env, sizeof(uint64_t) * 2 * size_t(h->d.n), hipMemcpyDeviceToHost));
  return 0;
}

// the handle's terrain-draw record to the device (setters run after a device sync)
static int put_tsrc(bb_handle* h) {
  HIPCHK(hipMemcpy(h->tsrc_dev, &h->tsrc, sizeof(TerrainSrc), hipMemcpyHostToDevice));
  return 0;
}

int bb_set_terrain_stream(bb_handle* h, const int32_t* slots, int n_streams, int length, const int32_t* env_stream) {
  if (!h) return fail("bb_set_terrain_stream: NULL handle");
  if (n_streams < 0) return fail("bb_set_terrain_stream: n_streams must be >= 0 (got %d)", n_streams);
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipDeviceSynchronize());
  if (n_streams == 0) {
    h->n_streams = 0;
    h->tsrc.tstream = nullptr; h->tsrc.env_stream = nullptr; h->tsrc.tlen = 0;
    return put_tsrc(h);
  }
  if (!slots) return fail("bb_set_terrain_stream: NULL slots");
  if (length < 1) return fail("bb_set_terrain_stream: length must be >= 1 (got %d)", length);
  const size_t cnt = size_t(n_streams) * size_t(length);
  for (size_t i = 0; i < cnt; i++)
    if (slots[i] < 0 || slots[i] >= h->p.n_terrains)
      return fail("bb_set_terrain_stream: slots[%zu] = %d out of range [0,%d)", i, slots[i], h->p.n_terrains);
  if (env_stream) {
    for (int e = 0; e < h->n; e++)
      if (env_stream[e] < 0 || env_stream[e] >= n_streams)
        return fail("bb_set_terrain_stream: env_stream[%d] = %d out of range [0,%d)", e, env_stream[e], n_streams);
  } else if (n_streams != 1) {
    return fail("bb_set_terrain_stream: %d streams need an env_stream map", n_streams);
  }
  // refill in place while the table fits; a larger table is a new allocation, whose address
  // goes into the device record that graphs captured before this call read at replay
  if (cnt > h->tstream_cap) {
    (void)hipFree(h->tstream);
    h->tstream = nullptr;
    h->tstream_cap = 0;
    HIPCHK(hipMalloc((void**)&h->tstream, sizeof(int) * cnt));
    h->tstream_cap = cnt;
  }
  HIPCHK(hipMemcpy(h->tstream, slots, sizeof(int) * cnt, hipMemcpyHostToDevice));
  if (env_stream) {
    if (!h->env_stream) HIPCHK(hipMalloc((void**)&h->env_stream, sizeof(int) * h->n));
    HIPCHK(hipMemcpy(h->env_stream, env_stream, sizeof(int) * h->n, hipMemcpyHostToDevice));
  }
  HIPCHK(hipMemset(h->d.episodes, 0, sizeof(int) * h->n));  // the next reset takes draw 0
  h->n_streams = n_streams;
  h->tsrc.tstream = h->tstream; h->tsrc.env_stream = env_stream ? h->env_stream : nullptr; h->tsrc.tlen = length;
  h->tsrc.rng = nullptr;  // the table replaces any device generators
  return put_tsrc(h);
}

int bb_set_terrain_rng(bb_handle* h, const uint64_t* words, const int32_t* seed_slot) {
  if (!h) return fail("bb_set_terrain_rng: NULL handle");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipDeviceSynchronize());
  if (!words) {
    h->tsrc.rng = nullptr;
    return put_tsrc(h);
  }
  if (seed_slot)
    for (int s = 0; s < TERRAIN_SEEDS; s++)
      if (seed_slot[s] >= h->p.n_terrains)
        return fail("bb_set_terrain_rng: seed_slot[%d] = %d out of range [-1,%d)", s, seed_slot[s], h->p.n_terrains);
  if (!seed_slot && h->p.n_terrains < TERRAIN_SEEDS)
    return fail("bb_set_terrain_rng: slot == seed needs a bank of %d terrains (have %d): pass seed_slot",
                TERRAIN_SEEDS, h->p.n_terrains);
  const size_t n = h->n;
  for (size_t e = 0; e < n; e++)
    if ((words[5 * e + 4] >> 32) > 1)
      return fail("bb_set_terrain_rng: env %zu: buffer word has bits above 32 other than has_uint32", e);
  std::vector<unsigned long long> soa(5 * n);
  for (size_t e = 0; e < n; e++)
    for (int j = 0; j < 5; j++) soa[j * n + e] = words[5 * e + j];
  if (!h->rng) HIPCHK(hipMalloc((void**)&h->rng, sizeof(unsigned long long) * 5 * n));
  HIPCHK(hipMemcpy(h->rng, soa.data(), sizeof(unsigned long long) * 5 * n, hipMemcpyHostToDevice));
  if (seed_slot) {
    if (!h->seed_slot) HIPCHK(hipMalloc((void**)&h->seed_slot, sizeof(int) * TERRAIN_SEEDS));
    HIPCHK(hipMemcpy(h->seed_slot, seed_slot, sizeof(int) * TERRAIN_SEEDS, hipMemcpyHostToDevice));
  }
  HIPCHK(hipMemset(h->d.episodes, 0, sizeof(int) * n));
  HIPCHK(hipMemset(h->d.tseed, 0xFF, sizeof(int) * n));
  h->tsrc.rng = h->rng;
  h->tsrc.seed_slot = seed_slot ? h->seed_slot : nullptr;
  return put_tsrc(h);
}

int bb_get_terrain_rng(bb_handle* h, uint64_t* words, int32_t* last_seed) {
  if (!h) return fail("bb_get_terrain_rng: NULL handle");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipDeviceSynchronize());
  const size_t n = h->n;
  if (words) {
    if (!h->tsrc.rng) return fail("bb_get_terrain_rng: no device generators (bb_set_terrain_rng)");
    std::vector<unsigned long long> soa(5 * n);
    HIPCHK(hipMemcpy(soa.data(), h->rng, sizeof(unsigned long long) * 5 * n, hipMemcpyDeviceToHost));
    for (size_t e = 0; e < n; e++)
      for (int j = 0; j < 5; j++) words[5 * e + j] = soa[j * n + e];
  }
  if (last_seed) HIPCHK(hipMemcpy(last_seed, h->d.tseed, sizeof(int) * n, hipMemcpyDeviceToHost));
  return 0;
}

int bb_get_env_terrain(bb_handle* h, int32_t* terrain, int32_t* draws) {
  if (!h) return fail("bb_get_env_terrain: NULL handle");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipDeviceSynchronize());
  if (terrain) HIPCHK(hipMemcpy(terrain, h->d.terrain, sizeof(int) * h->n, hipMemcpyDeviceToHost));
  if (draws) HIPCHK(hipMemcpy(draws, h->d.episodes, sizeof(int) * h->n, hipMemcpyDeviceToHost));
  return 0;
}

int bb_get_config(bb_handle* h, int32_t* out5) {
  if (!h || !out5) return fail("bb_get_config: NULL argument");
  out5[0] = h->n; out5[1] = h->epw; out5[2] = h->fp64;
  out5[3] = (int32_t)(h->fp64 ? lds_bytes<double>(h->epw) : lds_bytes<float>(h->epw));
  out5[4] = h->team;
  return 0;
}

#ifdef BB_PHASE_CLOCKS
// diagnostic build only: read and clear the per-phase cycle counters
int bb_debug_phase_cycles(unsigned long long* out16) {
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpyFromSymbol(out16, HIP_SYMBOL(bb::bb_phase_cycles), sizeof(unsigned long long) * 100));
  unsigned long long z[100] = {0};
  HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(bb::bb_phase_cycles), z, sizeof z));
  return 0;
}
#endif

int bb_time_kernel(bb_handle* h, int max_launches) {
  if (!h) return fail("bb_time_kernel: NULL handle");
  if (max_launches < 0) return fail("bb_time_kernel: max_launches must be >= 0");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipDeviceSynchronize());
  for (hipEvent_t e : h->tev) (void)hipEventDestroy(e);
  h->tev.assign(6 * (size_t)max_launches, nullptr);
  h->tpred.assign((size_t)max_launches, 0);
  for (hipEvent_t& e : h->tev) HIPCHK(hipEventCreate(&e));
  // record each once now: the runtime sets an event up at its first record, which would
  // otherwise land inside the caller's timed window, between its launches
  for (hipEvent_t& e : h->tev) HIPCHK(hipEventRecord(e, nullptr));
  HIPCHK(hipDeviceSynchronize());
  h->tcap = max_launches;
  h->tn = 0;
  return 0;
}

int bb_kernel_times(bb_handle* h, double* avg_ms3, int32_t* launches) {
  if (!h || !avg_ms3) return fail("bb_kernel_times: NULL argument");
  HIPCHK(hipSetDevice(h->device));
  double sum[3] = {0, 0, 0};
  int npred = 0;
  for (int i = 0; i < h->tn; i++) {
    hipEvent_t* ev = &h->tev[6 * i];
    HIPCHK(hipEventSynchronize(ev[5]));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, ev[0], ev[1]));  // fast kernel
    sum[0] += ms;
    float a = 0.f, b = 0.f;
    HIPCHK(hipEventElapsedTime(&a, ev[1], ev[5]));  // hand-over full kernel after the fast kernel ...
    if (h->tpred[i]) {                              // ... or after the predicted full kernel (side stream)
      HIPCHK(hipEventElapsedTime(&ms, ev[2], ev[3]));
      sum[1] += ms;
      npred++;
      HIPCHK(hipEventElapsedTime(&b, ev[3], ev[5]));
      a = a < b ? a : b;
    }
    sum[2] += a;
  }
  avg_ms3[0] = h->tn ? sum[0] / h->tn : 0.0;
  avg_ms3[1] = npred ? sum[1] / npred : 0.0;
  avg_ms3[2] = h->tn ? sum[2] / h->tn : 0.0;
  if (launches) *launches = h->tn;
  return 0;
}

int bb_kernel_ms(bb_handle* h, double* avg_ms, int32_t* launches) {
  if (!h || !avg_ms) return fail("bb_kernel_ms: NULL argument");
  double t[3];
  const int rc = bb_kernel_times(h, t, launches);
  if (rc) return rc;
  *avg_ms = t[0];
  return 0;
}

int bb_get_offsets(bb_handle* h, float* out) {
  if (!h || !out) return fail("bb_get_offsets: NULL argument");
  memcpy(out, h->h_offset.data(), sizeof(float) * h->h_offset.size());
  return 0;
}

}  // extern "C"
#endif  // BB_PAIR_TU
