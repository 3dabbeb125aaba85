// mca.h -- Monte Carlo arithmetic at float32 precision for the oracle's physics
// (pbg_physics.h with T = Mca).  TEST INFRASTRUCTURE ONLY: the parity tests' explanation of
// outliers (tests/test_gpu.py, "every outlier must be explained").
//
// Every +, -, *, /, sqrt, sin and cos is evaluated in double and then rounded to a float32
// neighbour chosen at random -- down or up with probability 1/2 when the double result is not
// a float (Parker's Monte Carlo arithmetic in "random rounding" mode at t = 24 bits, as
// Verificarlo implements it).  Each operation thus carries an error of up to one float32 ulp,
// the accuracy class of the kernels' own arithmetic (v_rcp_f32 / v_sqrt_f32 / v_rsq_f32 and
// the short sincos are ~1 ulp; FMA contraction and the Cholesky-space PGS reorder the
// roundings).  A batch of MCA runs from the same input samples the spread of results that
// float32 arithmetic of this algorithm admits on that input: a GPU deviation inside that
// spread is a float32 effect, one far outside it is not.  The random stream is seeded per
// env-step (pbg_oracle_set_mca_seed), so a run is reproducible.
#pragma once
#include <math.h>
#include <stdint.h>

extern thread_local uint64_t g_mca_state;

inline uint64_t mca_next() {  // splitmix64
  uint64_t z = (g_mca_state += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

struct Mca {
  float v;
  Mca() = default;
  explicit Mca(double x) : v((float)x) {}  // constants: round to nearest (not an operation)
  explicit operator double() const { return v; }
};

// random rounding of an exact (or double-accurate) result to one of its float neighbours
inline Mca mca_round(double d) {
  Mca r;
  float f = (float)d;
  if ((double)f != d && isfinite(d)) {
    if (mca_next() & 1) f = (double)f > d ? nextafterf(f, -INFINITY) : nextafterf(f, INFINITY);
  }
  r.v = f;
  return r;
}
inline Mca operator+(Mca a, Mca b) { return mca_round((double)a.v + (double)b.v); }
inline Mca operator-(Mca a, Mca b) { return mca_round((double)a.v - (double)b.v); }
inline Mca operator*(Mca a, Mca b) { return mca_round((double)a.v * (double)b.v); }
inline Mca operator/(Mca a, Mca b) { return mca_round((double)a.v / (double)b.v); }
inline bool operator<(Mca a, Mca b) { return a.v < b.v; }
inline bool operator>(Mca a, Mca b) { return a.v > b.v; }
inline bool operator<=(Mca a, Mca b) { return a.v <= b.v; }
inline bool operator>=(Mca a, Mca b) { return a.v >= b.v; }
inline bool operator==(Mca a, Mca b) { return a.v == b.v; }
inline bool operator!=(Mca a, Mca b) { return a.v != b.v; }
inline Mca sqrt(Mca a) { return mca_round(::sqrt((double)a.v)); }
inline Mca sin(Mca a) { return mca_round(::sin((double)a.v)); }
inline Mca cos(Mca a) { return mca_round(::cos((double)a.v)); }
inline Mca fabs(Mca a) { Mca r; r.v = fabsf(a.v); return r; }
