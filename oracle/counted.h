// counted.h -- an op-counting float32 scalar for the oracle's physics (pbg_physics.h with
// T = Counted).  TEST INFRASTRUCTURE ONLY: algorithmic FP32 work per env-step (SURVEY.md
// section 8d) for the flop roofline.  Each +, -, *, / and sqrt is one
// flop; sin and cos are counted apart (transcendentals: one each); comparisons, min/max,
// fabs and negation are not arithmetic and are not counted.  The restatement is dense (full
// Jacobians, dense Cholesky), so adds and muls are also counted without the ones that have an
// exactly-zero operand: that "nonzero" count is the algorithmic work the roofline uses.  No mixed-type operators and an
// explicit constructor: a double constant that was not cast to T does not compile.
#pragma once
#include <math.h>
#include <stdint.h>

struct FlopCount {
  uint64_t add, mul, div, sqrt, trans;
  uint64_t add_nz, mul_nz;  // the adds / muls with no exactly-zero operand (structural zeros
                            // of the dense restatement -- Jacobian columns of other branches,
                            // the mass matrix's uncoupled entries -- are not work)
};
extern thread_local FlopCount g_flops;

struct Counted {
  float v;
  Counted() = default;
  explicit Counted(double x) : v((float)x) {}
  explicit operator double() const { return v; }
};
inline Counted mkc(float x) { Counted c; c.v = x; return c; }
inline Counted operator+(Counted a, Counted b) {
  g_flops.add++;
  g_flops.add_nz += a.v != 0.f && b.v != 0.f;
  return mkc(a.v + b.v);
}
inline Counted operator-(Counted a, Counted b) {
  g_flops.add++;
  g_flops.add_nz += a.v != 0.f && b.v != 0.f;
  return mkc(a.v - b.v);
}
inline Counted operator*(Counted a, Counted b) {
  g_flops.mul++;
  g_flops.mul_nz += a.v != 0.f && b.v != 0.f;
  return mkc(a.v * b.v);
}
inline Counted operator/(Counted a, Counted b) { g_flops.div++; return mkc(a.v / b.v); }
inline bool operator<(Counted a, Counted b) { return a.v < b.v; }
inline bool operator>(Counted a, Counted b) { return a.v > b.v; }
inline bool operator<=(Counted a, Counted b) { return a.v <= b.v; }
inline bool operator>=(Counted a, Counted b) { return a.v >= b.v; }
inline bool operator==(Counted a, Counted b) { return a.v == b.v; }
inline bool operator!=(Counted a, Counted b) { return a.v != b.v; }
inline Counted sqrt(Counted a) { g_flops.sqrt++; return mkc(sqrtf(a.v)); }
inline Counted sin(Counted a) { g_flops.trans++; return mkc(sinf(a.v)); }
inline Counted cos(Counted a) { g_flops.trans++; return mkc(cosf(a.v)); }
inline Counted fabs(Counted a) { return mkc(fabsf(a.v)); }
