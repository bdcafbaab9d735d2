// Host phase timing of the per-env templates (diagnostic only).
#include <chrono>
#include <cstdio>
#include <vector>
#include "bb_model.h"
#include "bb_step.h"
using namespace bb;
using clk = std::chrono::steady_clock;

template <typename T>
void run(const char* path, int fp64) {
  FILE* f = fopen(path, "rb");
  int n; fread(&n, 4, 1, f);
  std::vector<double> Q(n * NQ), V(n * NV), W(n * NV), C(n * 3);
  fread(Q.data(), 8, n * NQ, f); fread(V.data(), 8, n * NV, f); fread(W.data(), 8, n * NV, f); fread(C.data(), 8, n * 3, f);
  fclose(f);
  ModelT<T> m = cast_model<T>(compile_model(default_solver(fp64)));
  std::vector<float> hf(HF_N * HF_N, 0.f);
  static EnvWork<T> EW;
  GStore<T> st{EW.g, 1};
  double tk = 0, tw = 0, tc = 0, ts = 0; long iters = 0, ngs = 0;
  for (int rep = 0; rep < 3; rep++)
  for (int e = 0; e < n; e++) {
    T q[NQ], v[NV], a[NV], c[3];
    for (int i = 0; i < NQ; i++) q[i] = Q[e * NQ + i];
    for (int i = 0; i < NV; i++) { v[i] = V[e * NV + i]; a[i] = W[e * NV + i]; }
    for (int i = 0; i < 3; i++) c[i] = C[e * 3 + i];
    auto t0 = clk::now();
    Kin<T> k; kinematics(m, q, k);
    Mass<T>& M = EW.M; T Iw[3][6]; build_mass(m, k, M, Iw);
    T qfs[NV]; bias_forces(m, k, Iw, v, qfs);
    for (int i = 0; i < NV; i++) qfs[i] = -qfs[i];
    for (int w = 0; w < 3; w++) qfs[6 + w] += -m.damping * v[6 + w] + c[w];
    auto t1 = clk::now();
    WheelCon<T>* WC = EW.wc;
    for (int w = 0; w < 3; w++) wheel_contact(m, k, v, w, WC[w]);
    auto t2 = clk::now();
    int ov = 0;
    int ng = collide_ground(m, k, v, hf.data(), T(2.0), st, &ov);
    auto t3 = clk::now();
    int it = solve_team(m, EW, qfs, ng, a, Team{1, 0});
    auto t4 = clk::now();
    tk += std::chrono::duration<double>(t1 - t0).count(); tw += std::chrono::duration<double>(t2 - t1).count();
    tc += std::chrono::duration<double>(t3 - t2).count(); ts += std::chrono::duration<double>(t4 - t3).count();
    iters += it; ngs += ng;
  }
  n *= 3;
#ifdef BB_SOLVE_STATS
  printf("ls evals per newton iter %.2f\n", double(g_ls_evals) / iters); g_ls_evals = 0;
#endif
  printf("fp64=%d per forward: kin+mass+bias %.2f us, wheel %.2f us, collide %.2f us, solve %.2f us (iters %.2f, ng %.2f)\n",
         fp64, tk / n * 1e6, tw / n * 1e6, tc / n * 1e6, ts / n * 1e6, double(iters) / n, double(ngs) / n);
}
int main(int argc, char** argv) { run<double>(argv[1], 1); run<float>(argv[1], 0); }
