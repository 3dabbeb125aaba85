// sanitize_main.cpp -- ASan/UBSan driver for the CPU oracle (TEST INFRASTRUCTURE ONLY).
// Built by `make -C oracle sanitize` with -fsanitize=address,undefined together with
// pbg_oracle.cpp, run by tests/test_oracle_sanitizers.py: for every robot, reset a few envs
// and step them with random actions (single thread and OpenMP), including the pack on a
// NaN-bearing input and every physics-rule variant switch; any sanitizer report aborts.
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

extern "C" {
int pbg_oracle_info(int robot, int* out);
int pbg_oracle_reset(int robot, int n, double* state, double* aux, const double* qinit, float* obs);
int pbg_oracle_reset_mask(int robot, int n, double* state, double* aux, const double* qinit, float* obs,
                          const uint8_t* mask);
int pbg_oracle_step(int robot, int n, double* state, double* aux, const float* act, float* obs, double* rew,
                    uint8_t* done, int32_t* ncontact, int nthreads, uint32_t* csig, double* rew_terms);
int pbg_oracle_set_physics(const double* v, int n);
}

int main(int argc, char** argv) {
  const int steps = argc > 1 ? atoi(argv[1]) : 40;
  uint64_t x = 88172645463325252ull;
  auto rnd = [&]() {  // xorshift64 -> [-1, 1)
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    return (double)(x >> 11) * (2.0 / 9007199254740992.0) - 1.0;
  };
  const double variants[][2] = {{-1, 0}, {7, 0.85}, {6, 1}, {6, 2}, {4, 1}, {5, 1}, {11, 1}};
  for (int robot = 0; robot < 17; robot++) {
    int info[16];
    if (pbg_oracle_info(robot, info) != 0) return 2;
    const int NA = info[3], NR = info[5], OBS = info[10], SD = info[11], AD = info[12];
    for (const auto& var : variants) {
      double opt[32];
      const int nopt = pbg_oracle_set_physics(nullptr, 0);
      pbg_oracle_set_physics(nullptr, 0);
      if (var[0] >= 0) {
        const double def[] = {-1.0, -1.0, -0.04, 0, 0, 0, 0, 0, 0, 0.2, 5, 0, 0, 1, 1};
        memcpy(opt, def, sizeof(def));
        opt[(int)var[0]] = var[1];
        pbg_oracle_set_physics(opt, nopt);
      }
      const int n = 6;
      std::vector<double> st((size_t)n * SD), aux((size_t)n * AD), q((size_t)n * NR), rew(n), terms((size_t)n * 5);
      std::vector<float> obs((size_t)n * OBS), act((size_t)n * NA);
      std::vector<uint8_t> done(n), mask(n);
      std::vector<int32_t> nc(n);
      std::vector<uint32_t> sig(n);
      for (auto& v : q) v = 0.1 * rnd();
      if (pbg_oracle_reset(robot, n, st.data(), aux.data(), q.data(), obs.data()) != 0) return 3;
      if (robot == 15)  // HumanoidFlagrunHarder: frame 120, so the first step launches the cube
        for (int e = 0; e < n; e++) aux[(size_t)e * AD + 8 + info[6]] = 120.0;
      for (int t = 0; t < steps; t++) {
        for (auto& v : act) v = (float)rnd();
        if (t == steps / 2) act[0] = NAN;  // non-finite action path
        if (pbg_oracle_step(robot, n, st.data(), aux.data(), act.data(), obs.data(), rew.data(), done.data(), nc.data(),
                            t & 1 ? 2 : 1, sig.data(), terms.data()) != 0)
          return 4;
        for (int e = 0; e < n; e++) mask[e] = done[e];
        pbg_oracle_reset_mask(robot, n, st.data(), aux.data(), q.data(), obs.data(), mask.data());
      }
    }
  }
  pbg_oracle_set_physics(nullptr, 0);
  printf("sanitize ok\n");
  return 0;
}
