// Self-test of oracle/cpu_ref.cpp for the sanitizer build (oracle/Makefile: make selftest-asan):
// a small synthetic prepared spectrum through the OpenMP sample loop, log_mvnpdf_low_rank against
// a dense Cholesky of K = M M' + diag(d), and Faddeeva symmetry / limits.  TEST INFRASTRUCTURE.
#include "cpu_ref.cpp"

#include <cstdio>
#include <random>

static double dense_logpdf(const std::vector<double>& y, const std::vector<double>& mu,
                           const std::vector<double>& M, const std::vector<double>& d, int n, int k) {
  std::vector<double> K((size_t)n * n, 0.0);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      double s = i == j ? d[i] : 0.0;
      for (int c = 0; c < k; ++c) s += M[(size_t)c * n + i] * M[(size_t)c * n + j];
      K[(size_t)i * n + j] = s;
    }
  double logdet = 0.0;
  for (int j = 0; j < n; ++j) {  // lower Cholesky in place
    for (int l = 0; l < j; ++l) K[(size_t)j * n + j] -= K[(size_t)j * n + l] * K[(size_t)j * n + l];
    const double ljj = std::sqrt(K[(size_t)j * n + j]);
    K[(size_t)j * n + j] = ljj;
    logdet += 2.0 * std::log(ljj);
    for (int i = j + 1; i < n; ++i) {
      for (int l = 0; l < j; ++l) K[(size_t)i * n + j] -= K[(size_t)i * n + l] * K[(size_t)j * n + l];
      K[(size_t)i * n + j] /= ljj;
    }
  }
  std::vector<double> t(n);
  for (int i = 0; i < n; ++i) {
    double s = y[i] - mu[i];
    for (int l = 0; l < i; ++l) s -= K[(size_t)i * n + l] * t[l];
    t[i] = s / K[(size_t)i * n + i];
  }
  double q = 0.0;
  for (double v : t) q += v * v;
  return -0.5 * (q + logdet + n * kLog2Pi);
}

int main() {
  std::mt19937_64 rng(7);
  std::normal_distribution<double> nd;
  std::uniform_real_distribution<double> ud(0.01, 0.09);
  int fails = 0;
  {  // log_mvnpdf_low_rank vs dense
    const int n = 60, k = 5;
    std::vector<double> y(n), mu(n), M((size_t)n * k), d(n);
    for (int i = 0; i < n; ++i) { y[i] = nd(rng); mu[i] = 0.3 * nd(rng); d[i] = ud(rng); }
    for (auto& v : M) v = 0.2 * nd(rng);
    double got = 0.0;
    gpdla_cpu_log_mvnpdf_low_rank(y.data(), mu.data(), M.data(), d.data(), n, k, &got);
    const double ref = dense_logpdf(y, mu, M, d, n, k);
    if (!(std::fabs(got - ref) <= 1e-10 * std::max(1.0, std::fabs(ref)))) {
      std::printf("log_mvnpdf %.17g vs dense %.17g\n", got, ref);
      ++fails;
    }
  }
  {  // Faddeeva: symmetry and the large-|z| limit w ~ i / (sqrt(pi) z)
    for (double x : {0.0, 0.1, 1.0, 5.9, 6.1, 50.0, 1e4}) {
      double a, b, c, e;
      gpdla_cpu_faddeeva_w(x, 1e-4, &a, &b);
      gpdla_cpu_faddeeva_w(-x, 1e-4, &c, &e);
      if (a != c || b != -e) { std::printf("w symmetry at %g\n", x); ++fails; }
    }
    double a, b;
    gpdla_cpu_faddeeva_w(1e4, 3e-4, &a, &b);
    const double ra = 3e-4 / (std::sqrt(M_PI) * 1e8), rb = 1.0 / (std::sqrt(M_PI) * 1e4);
    if (std::fabs(a / ra - 1) > 1e-7 || std::fabs(b / rb - 1) > 1e-7) { std::printf("w asymptote\n"); ++fails; }
  }
  {  // the OpenMP sample loop on a synthetic prepared spectrum
    const int n = 200, k = 8, m = 210;
    std::vector<double> y(n), noise(n), mu(n), M((size_t)n * k), om2(n), padded(m + 6);
    std::vector<int64_t> aind(n);
    for (int i = 0; i < n; ++i) {
      mu[i] = 1.0 + 0.1 * nd(rng); y[i] = mu[i] + 0.2 * nd(rng); noise[i] = ud(rng);
      om2[i] = 0.04; aind[i] = i;
    }
    for (auto& v : M) v = 0.05 * nd(rng);
    for (int i = 0; i < m + 6; ++i) padded[i] = std::pow(10.0, std::log10(4000.0) + 1e-4 * (i - 3));
    const int S = 37;
    std::vector<double> off(S), nhi(S), out(S);
    for (int s = 0; s < S; ++s) { off[s] = (s + 0.5) / S; nhi[s] = std::pow(10.0, 20.0 + 3.0 * off[s]); }
    const int rc = gpdla_cpu_sample_lls(n, k, y.data(), noise.data(), mu.data(), M.data(), om2.data(), m,
                                        padded.data(), aind.data(), 2.25, 2.29, S, off.data(), nhi.data(), 3,
                                        2, out.data());
    for (int s = 0; s < S; ++s)
      if (!std::isfinite(out[s])) { std::printf("sample %d not finite\n", s); ++fails; }
    if (rc != 0) { std::printf("sample_lls rc %d\n", rc); ++fails; }
  }
  std::printf(fails ? "cpu_ref selftest FAILED (%d)\n" : "cpu_ref selftest ok\n", fails);
  return fails ? 1 : 0;
}
