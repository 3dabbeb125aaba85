"""Accuracy of the float64 kernels' sin / cos (pybullet-gym_amd/csrc/pbg_sincos64.h; CPU test).

The float64 physics (joint rotations, the base's exponential map) uses a Cody-Waite reduction and the
FreeBSD msun minimax kernels instead of the device library's sincos.  The header is plain C++: this
test compiles it with g++ and measures the error against long-double sinl / cosl (x86 80-bit) over
random arguments in ranges from 1e-8 to 1e6, next to the C library's own error.  Bound: 1 ulp for
|x| <= 1e5 (the joint angles and half-angle increments of the physics are far smaller), and 1e-15
absolute in every range.  The float64 parity tests hold the state to 1e-9 relative, ~1e7 ulp.
"""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "pybullet-gym_amd", "csrc")
PROG = r'''
#include <cmath>
#include <cstdio>
#include <random>
#include "pbg_sincos64.h"
static double ulp_err(double got, long double ref) {
  const double r = (double)ref;
  if (std::fabs(r) < 1e-300) return 0;
  const double u = std::nextafter(std::fabs(r), INFINITY) - std::fabs(r);
  return (double)(std::fabs((long double)got - ref) / u);
}
int main() {
  std::mt19937_64 g(1);
  const double ranges[] = {1e-8, 1e-3, 0.7853981633974483, 3.2, 10.0, 1e3, 1e5, 1e6};
  for (double R : ranges) {
    std::uniform_real_distribution<double> d(-R, R);
    double ms = 0, mc = 0, ls = 0, lc = 0, ma = 0;
    for (int i = 0; i < 250000; i++) {
      double x = d(g), s, c;
      pbg::sincos_reduced64(x, &s, &c);
      const long double rs = sinl((long double)x), rc = cosl((long double)x);
      ms = std::fmax(ms, ulp_err(s, rs)); mc = std::fmax(mc, ulp_err(c, rc));
      ls = std::fmax(ls, ulp_err(std::sin(x), rs)); lc = std::fmax(lc, ulp_err(std::cos(x), rc));
      ma = std::fmax(ma, (double)std::fmax(std::fabs((long double)s - rs), std::fabs((long double)c - rc)));
    }
    printf("%g %.4f %.4f %.4f %.4f %.3g\n", R, ms, mc, ls, lc, ma);
  }
  double s, c;
  pbg::sincos_reduced64(NAN, &s, &c);
  printf("nan %d %d\n", (int)std::isnan(s), (int)std::isnan(c));
  return 0;
}
'''


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_sincos64_within_one_ulp(tmp_path):
    src = tmp_path / "t.cpp"
    src.write_text(PROG)
    exe = tmp_path / "t"
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-I", CSRC, "-o", str(exe), str(src)])
    out = subprocess.check_output([str(exe)], text=True).split("\n")
    rows = [l.split() for l in out if l and not l.startswith("nan")]
    for r in rows:
        R, ms, mc, ls, lc, ma = float(r[0]), *map(float, r[1:])
        if R <= 1e5:
            assert ms <= 1.0 and mc <= 1.0, (R, ms, mc, "libm", ls, lc)
        assert ma <= 1e-15, (R, ma)  # absolute, every range (near a zero of sin at |x| ~ 1e6 the
        # relative error of a ~1e-12 result can reach 1e-9: the neglected part of pi/2 times n)
    assert [l for l in out if l.startswith("nan")] == ["nan 1 1"]
