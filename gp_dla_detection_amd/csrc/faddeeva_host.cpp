// Host-side Faddeeva function and line-profile table fitting (product code, runs at engine
// creation; the per-sample evaluation happens on the GPU from the fitted tables).
//
// libcerf (the reference's dependency, voigt.c:5,288) is not available here; this file supplies
// the w(z) the tables are fitted from.  Method (extended precision, long double):
//   * |x| <= kTaylorX: analytic continuation by Taylor series.  w solves
//       w'(z) = -2 z w(z) + 2i/sqrt(pi),  w(0) = 1,
//     so its Taylor coefficients at z0 obey  a1 = -2 z0 a0 + 2i/sqrt(pi),
//       (n+1) a_{n+1} = -2 z0 a_n - 2 a_{n-1}.
//     A real-axis table w(m h) is marched from w(0) = 1 (forward marching is stable: the
//     homogeneous solution exp(-z^2) decays along +x), then one Taylor step reaches x + iy.
//   * |x| >  kTaylorX: the Laplace asymptotic series  w(z) ~ (i/sqrt(pi)) sum (2n-1)!!/(2z^2)^n / z,
//     truncated at its smallest term (relative error < exp(-x^2) ~ 1e-62 at x = 12).
// Only Im z >= 0 with small Im z is needed (Lyman-series y_j <= 4.8e-4); the standalone API
// documents |y| <= 1.
#include <algorithm>
#include <cmath>
#include <complex>
#include <mutex>
#include <vector>

#include "line_profile.h"
#include "lyman_series.h"

namespace gpdla {

using cld = std::complex<long double>;

namespace {

constexpr long double kPiL = 3.141592653589793238462643383279502884L;
constexpr long double kTaylorX = 12.0L;
constexpr long double kStepH = 1.0L / 32.0L;
constexpr int kTaylorTerms = 48;

const long double kTwoOverSqrtPi = 2.0L / std::sqrt(kPiL);

cld taylor_step(cld w0, cld z0, cld delta) {
  // sum_n a_n delta^n with the recurrence above
  const cld i2sp(0.0L, kTwoOverSqrtPi);
  cld a_prev = w0;
  cld a_cur = -2.0L * z0 * w0 + i2sp;
  cld sum = w0 + a_cur * delta;
  cld dpow = delta;
  for (int n = 1; n < kTaylorTerms; ++n) {
    cld a_next = -(2.0L * z0 * a_cur + 2.0L * a_prev) / (long double)(n + 1);
    dpow *= delta;
    cld term = a_next * dpow;
    sum += term;
    a_prev = a_cur;
    a_cur = a_next;
    if (std::abs(term) < 1e-24L * std::abs(sum) && n > 8) break;
  }
  return sum;
}

struct RealAxisTable {
  std::vector<cld> w;  // w(m h), m = 0 .. M
  RealAxisTable() {
    const int M = (int)(kTaylorX / kStepH) + 2;
    w.resize(M + 1);
    w[0] = cld(1.0L, 0.0L);
    for (int m = 0; m < M; ++m)
      w[m + 1] = taylor_step(w[m], cld(m * kStepH, 0.0L), cld(kStepH, 0.0L));
  }
};

const RealAxisTable& real_axis() {
  static RealAxisTable t;
  return t;
}

cld w_asymptotic(cld z) {
  const cld z2 = z * z;
  cld term = 1.0L / z;
  cld sum = term;
  long double prev = std::abs(term);
  for (int n = 0; n < 400; ++n) {
    cld next = term * ((long double)(2 * n + 1) / (2.0L * z2));
    long double an = std::abs(next);
    if (an > prev) break;  // optimal truncation of the divergent series
    sum += next;
    term = next;
    prev = an;
    if (an < 1e-26L * std::abs(sum)) break;
  }
  return cld(0.0L, 1.0L / std::sqrt(kPiL)) * sum;
}

}  // namespace

// Faddeeva w(x + iy), y >= 0 (small); long double.
cld faddeeva_w(long double x, long double y) {
  const long double ax = std::fabs(x);
  cld w;
  if (ax <= kTaylorX) {
    const RealAxisTable& t = real_axis();
    int m = (int)std::lround(ax / kStepH);
    w = taylor_step(t.w[m], cld(m * kStepH, 0.0L), cld(ax - m * kStepH, y));
  } else {
    w = w_asymptotic(cld(ax, y));
  }
  // w(-conj z) = conj(w(z)): Re even in x, Im odd in x
  if (x < 0) w = cld(w.real(), -w.imag());
  return w;
}

namespace {

// Chebyshev interpolation of f on [-1, 1] at n+1 first-kind nodes -> monomial coefficients in s.
std::vector<long double> cheb_fit_monomial(const std::vector<long double>& fvals) {
  const int N = (int)fvals.size();  // nodes s_k = cos(pi (k + 1/2) / N)
  std::vector<long double> c(N, 0.0L);
  for (int j = 0; j < N; ++j) {
    long double acc = 0;
    for (int k = 0; k < N; ++k) acc += fvals[k] * std::cos(kPiL * j * (k + 0.5L) / N);
    c[j] = acc * (j == 0 ? 1.0L : 2.0L) / N;
  }
  // sum_j c_j T_j(s) -> monomials
  std::vector<long double> mono(N, 0.0L), tprev(N, 0.0L), tcur(N, 0.0L), tnext(N, 0.0L);
  tprev[0] = 1.0L;                  // T0
  if (N > 1) tcur[1] = 1.0L;        // T1
  for (int i = 0; i < N; ++i) mono[i] += c[0] * tprev[i];
  if (N > 1) for (int i = 0; i < N; ++i) mono[i] += c[1] * tcur[i];
  for (int j = 2; j < N; ++j) {
    std::fill(tnext.begin(), tnext.end(), 0.0L);
    for (int i = 0; i < N - 1; ++i) tnext[i + 1] += 2.0L * tcur[i];
    for (int i = 0; i < N; ++i) tnext[i] -= tprev[i];
    for (int i = 0; i < N; ++i) mono[i] += c[j] * tnext[i];
    tprev = tcur;
    tcur = tnext;
  }
  return mono;
}

}  // namespace

namespace {

// (a T + b)^n expansion of a polynomial given in s = a T + b (monomials), -> powers of T
std::vector<long double> shift_to_T(const std::vector<long double>& mono_s, long double a, long double b) {
  const int N = (int)mono_s.size();
  std::vector<long double> t(N, 0.0L);
  for (int n = 0; n < N; ++n) {
    long double binom = 1.0L;
    for (int r = 0; r <= n; ++r) {
      t[r] += mono_s[n] * binom * std::pow(a, (long double)r) * std::pow(b, (long double)(n - r));
      binom = binom * (n - r) / (r + 1);
    }
  }
  return t;
}

// Line j's profile scale lc_j / (sigma sqrt(2 pi)) and damping y_j = gamma_j / (sigma sqrt 2).
void line_scale(int j, long double* scale, long double* y) {
  const long double sig = (long double)kSigma;
  *y = (long double)kLorentzGammas[j] / (sig * std::sqrt(2.0L));
  *scale = (long double)kLeadingConstants[j] / (sig * std::sqrt(2.0L * kPiL));
}

// f_j(x) x^2 = sum_n c[n] T^n on T = 1/x^2 in (0, 1/xmin^2] at degree deg (Chebyshev
// interpolation at deg + 1 first-kind nodes, then monomials in T), zero-padded to len.
void fit_T_poly(int j, long double xmin, int deg, int len, double* c) {
  long double scale, y;
  line_scale(j, &scale, &y);
  const long double Tmax = 1.0L / (xmin * xmin);
  const int N = deg + 1;
  std::vector<long double> fv(N);
  for (int k = 0; k < N; ++k) {
    const long double T = Tmax * (std::cos(kPiL * (k + 0.5L) / N) + 1.0L) / 2.0L;
    fv[k] = scale * faddeeva_w(1.0L / std::sqrt(T), y).real() / T;
  }
  const std::vector<long double> t = shift_to_T(cheb_fit_monomial(fv), 2.0L / Tmax, -1.0L);
  for (int n = 0; n < len; ++n) c[n] = n < N ? (double)t[n] : 0.0;
}

}  // namespace

// Wing block of line j (kWingStride doubles): the wing polynomial for |x| >= kCoreX at 0, the
// outer polynomial for |x| >= kOuterX at kOuterOff.
void fit_wing_line(int j, double* wing) {
  fit_T_poly(j, (long double)kCoreX, kWingDeg, kOuterOff, wing);
  fit_T_poly(j, (long double)kOuterX, kOuterDeg, kWingStride - kOuterOff, wing + kOuterOff);
}

// Core table of line j (kPieces x kCoreStride, polynomial in u = |x| - centre).
void fit_core_table(int j, double* core) {
  long double scale, y;
  line_scale(j, &scale, &y);
  const int N = kCoreDeg + 1;
  for (int p = 0; p < kPieces; ++p) {
    const long double centre = (p + 0.5L) * kPieceW, half = 0.5L * kPieceW;
    std::vector<long double> fv(N);
    for (int k = 0; k < N; ++k)
      fv[k] = scale * faddeeva_w(centre + half * std::cos(kPiL * (k + 0.5L) / N), y).real();
    std::vector<long double> mono = cheb_fit_monomial(fv);  // in s = u / half
    long double sc = 1.0L;
    for (int n = 0; n < N; ++n) {
      core[p * kCoreStride + n] = (double)(mono[n] * sc);
      sc /= half;
    }
  }
}

// Max relative error of the double-precision line profile of line j against the long-double
// source on a dense grid (core: 36k points, wing: geometric out to |x| = 2e6).
double line_profile_error(int j) {
  std::vector<double> core(kCoreTable), wing(kWingStride);
  fit_core_table(j, core.data());
  fit_wing_line(j, wing.data());
  long double scale, y;
  line_scale(j, &scale, &y);
  double maxrel = 0;
  for (int i = 0; i <= 48000; ++i) {
    const double x = (i < 36000) ? i * (kCoreX / 36000.0) : kCoreX * std::pow(1.0004, i - 36000);
    const double got = line_profile_eval(core.data(), wing.data(), x);
    const long double ref = scale * faddeeva_w((long double)x, y).real();
    double rel = (double)std::fabs((got - ref) / ref);
    if (x >= kOuterX)  // the batched sweeps' outer polynomial
      rel = std::max(rel, (double)std::fabs((outer_poly(wing.data(), 1.0 / (x * x)) - ref) / ref));
    if (rel > maxrel) maxrel = rel;
  }
  return maxrel;
}

}  // namespace gpdla

extern "C" int gpdla_diag_faddeeva_w(double x, double y, double* re, double* im) {
  if (!re || !im || !(y >= 0.0) || !(y <= 1.0)) return -1;
  const gpdla::cld w = gpdla::faddeeva_w((long double)x, (long double)y);
  *re = (double)w.real();
  *im = (double)w.imag();
  return 0;
}
