// solver_stats.cpp -- host-side statistics of the constraint solve on a
// steady-state population of envs (test/tool code, never shipped).
//
// Runs n envs x s steps of the product's per-env templates (bb_step.h, host
// path: team of one lane, bb_solve.h:solve_team) with uniform random actions
// on flat terrain, auto-resetting terminated envs, and prints the Newton
// iterations per forward and line-search evaluations per Newton iteration.
// Used to compare solver variants by work done, before timing them on the GPU.
//
//   g++ -O2 -std=c++17 -DBB_SOLVE_STATS -I openballbot-rl_amd/csrc -x c++ \
//       -D__HIP_PLATFORM_AMD__ tools/solver_stats.cpp -o tools/_build/solver_stats
#include <stdio.h>
#include <stdlib.h>
#include <random>
#include <vector>

#include "bb_model.h"
#include "bb_step.h"

using namespace bb;

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 64;
  const int steps = argc > 2 ? atoi(argv[2]) : 600;
  const int skip = argc > 3 ? atoi(argv[3]) : 200;  // burn-in steps not counted
  SolverCfg sc = default_solver(true);
  if (getenv("BB_LSTOL")) sc.ls_tol = atof(getenv("BB_LSTOL"));
  ModelT<double> m = compile_model(sc);
  EnvCfg cfg{4000, 20.f, 10.f, 0.01f, -1e-4f, 0.02f, {0.f, 1.f}, 0, {0.f, 0.f}, 1.f};
  std::vector<float> hf(HF_N * HF_N, 0.f);
  const TerrainRef<double> tr{hf.data(), 2.0, 0.0};
  static EnvWork<double> W;
  std::vector<double> q(n * NQ), v(n * NV), w(n * NV);
  std::vector<int> st(n, 0);
  for (int e = 0; e < n; e++) reset_state(m, 0.01, &q[e * NQ], &v[e * NV], &w[e * NV]);
  std::mt19937_64 rng(12345);
  std::uniform_real_distribution<float> U(-1.f, 1.f);
  long fwd = 0, newton = 0, ls0 = 0, resets = 0;
  long hist[32] = {0};
  long nghist[32] = {0};  // ball-terrain contacts at the last RK stage
  FILE* dump = getenv("BB_DUMP_ITERS") ? fopen(getenv("BB_DUMP_ITERS"), "w") : nullptr;
  for (int t = 0; t < steps; t++) {
    for (int e = 0; e < n; e++) {
      float a[3] = {U(rng), U(rng), U(rng)}, obs[15], r, p2[2];
      int it = 0;
      const long lsb = g_ls_evals;
      int fl = env_step<double, false>(m, cfg, &q[e * NQ], &v[e * NV], &w[e * NV], st[e], a, tr, W, obs, r, p2, &it,
                                       Team{1, 0});
      if (dump && t >= skip)
        fprintf(dump, "%d %d %d %d %d %d %d %d\n", t, e, it, st[e], g_stage_iters[0], g_stage_iters[1], g_stage_iters[2],
                g_stage_iters[3]);
      if (t >= skip) {
        nghist[W.so.ng < 31 ? W.so.ng : 31]++;
        fwd += 4; newton += it; ls0 += g_ls_evals - lsb;
        hist[it / 4 < 31 ? it / 4 : 31]++;
      }
      if (fl & 5) {
        reset_state(m, 0.01, &q[e * NQ], &v[e * NV], &w[e * NV]);
        st[e] = 0; resets++;
      }
    }
  }
  printf("{\"envs\": %d, \"steps\": %d, \"forwards\": %ld, \"newton_per_forward\": %.4f, "
         "\"ls_evals_per_newton\": %.4f, \"ls_evals_per_forward\": %.4f, \"resets\": %ld, \"iters_per_step_hist4\": [",
         n, steps - skip, fwd, double(newton) / fwd, double(ls0) / newton, double(ls0) / fwd, resets);
  for (int i = 0; i < 12; i++) printf("%s%ld", i ? ", " : "", hist[i]);
  printf("], \"ground_contacts_hist\": [");
  for (int i = 0; i < 20; i++) printf("%s%ld", i ? ", " : "", nghist[i]);
  printf("], \"ls_evals_hist\": [");
  for (int i = 1; i < 16; i++) printf("%s%ld", i > 1 ? ", " : "", g_ls_hist[i]);
  printf("]}\n");
  return 0;
}
