/* gpdla_mex.c -- MATLAB gateway of the batched engine: the reference-side binding that replaces the
 * per-quasar loop of process_qsos.m:88-220 (its parfor over DLA samples, :184-198, included) with
 * one engine call.  The caller keeps process_qsos.m's loading (:1-63), priors and posteriors
 * (:122-132, 222-232) and save (:235-249); see matlab/process_qsos_gpu.m.
 *
 * Build (MATLAB R2018a+, interleaved-complex API):
 *   mex -R2018a matlab/gpdla_mex.c -Iinclude -Lgp_dla_detection_amd -lgpdla
 *
 *   eng = gpdla_mex('create', device, rest_wavelengths, mu, M, log_omega, log_c_0, log_tau_0,
 *                   log_beta, offset_samples, nhi_samples, num_lines, width, pixel_spacing,
 *                   min_lambda, max_lambda, lya_wavelength, lyman_limit, min_z_cut, max_z_cut
 *                   [, absorption_mode [, path]])
 *       The learned model (learned_qso_model_*.mat, process_qsos.m:30-35), the DLA samples
 *       (dla_samples.mat, :38-40) and the set_parameters.m knobs the path reads, in gpdla_model /
 *       gpdla_samples / gpdla_params order (include/gpdla.h).  absorption_mode: 0 = the reference's
 *       absorption(1:n) quirk (process_qsos.m:180,189, default), 1 = unmasked pixels.  path: 'auto'
 *       (default), 'fused', 'panel_gemm', 'fused_i8', 'panel_gemm_i8', 'panel_gemm_i8_24'.
 *       Returns a uint64 handle.
 *
 *   [log_likelihoods_no_dla, sample_log_likelihoods_dla, log_likelihoods_dla, min_z_dlas,
 *    max_z_dlas, num_pixels] = gpdla_mex('process', eng, all_wavelengths, all_flux,
 *                                        all_noise_variance, all_pixel_mask, z_qsos)
 *       The preloaded_qsos cells of the selected spectra (process_qsos.m:45-61) and their z_QSO,
 *       double or single (fitsread's class for the speclite columns; widened exactly, mex_widen.h).
 *       Outputs as process_qsos.m:74-82 shapes them: Q x 1 vectors and the Q x S sample matrix
 *       (:195), with NaN where a spectrum has no usable pixel.  A non-positive pivot (MATLAB's chol
 *       would raise, log_mvnpdf_low_rank.m:24) leaves NaN likelihoods and raises 'MATLAB:posdef'
 *       after every output is filled.
 *
 *   gpdla_mex('destroy', eng)
 *
 * The Python mirror of the same three calls (argument meaning and order) is
 * gp_dla_detection_amd.engine.Engine(model, samples, params, device, path) and Engine.process(
 * packed) -> dict of the same outputs; process.run_process_qsos wraps it on files.
 *
 * Cells are packed into the engine's CSR layout (gpdla_spectra: offsets[Q+1] + concatenated
 * pixels, the mask as uint8) once, then processed in batches of kBatch spectra so the host staging
 * of the spectrum-major [q][s] engine output stays ~0.3 GB; each batch is transposed into the
 * column-major Q x S result in cache-sized tiles. */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "mex.h"
#include "gpdla.h"
#include "mex_widen.h"

enum { kMaxEngines = 64, kBatch = 4096, kTile = 64 };
static gpdla_engine* g_engines[kMaxEngines];
static int64_t g_num_samples[kMaxEngines];     /* S of each live engine (its samples at create) */

static void destroy_all(void) {
  for (int i = 0; i < kMaxEngines; ++i)
    if (g_engines[i]) {
      gpdla_engine_destroy(g_engines[i]);
      g_engines[i] = NULL;
    }
}

static void fail(int rc, const char* what) {
  if (rc == GPDLA_ENUMERIC) mexErrMsgIdAndTxt("MATLAB:posdef", "%s: %s", what, gpdla_last_error());
  mexErrMsgIdAndTxt("gpdla:engine", "%s failed (%d): %s", what, rc, gpdla_last_error());
}

static const double* dbl(const mxArray* a, const char* name, size_t want) { return widen(a, name, want); }

static double scalar(const mxArray* a, const char* name) { return widen_scalar(a, name); }

static int path_code(const mxArray* a) {
  if (!mxIsChar(a)) return (int)scalar(a, "path");
  static const char* names[] = {"auto", "fused", "panel_gemm", "fused_i8", "panel_gemm_i8", "panel_gemm_i8_24"};
  static const int codes[] = {GPDLA_PATH_AUTO, GPDLA_PATH_FUSED, GPDLA_PATH_PANEL_GEMM, GPDLA_PATH_FUSED_I8,
                              GPDLA_PATH_PANEL_GEMM_I8, GPDLA_PATH_PANEL_GEMM_I8_24};
  char* s = mxArrayToString(a);
  int code = -1;
  for (int i = 0; i < 6; ++i)
    if (s && strcmp(s, names[i]) == 0) code = codes[i];
  mxFree(s);
  if (code < 0) mexErrMsgIdAndTxt("gpdla:path", "unknown path");
  return code;
}

static int slot_of(const mxArray* h) {
  if (!mxIsUint64(h) || mxGetNumberOfElements(h) != 1) mexErrMsgIdAndTxt("gpdla:handle", "not an engine handle");
  const uint64_t v = *mxGetUint64s(h);
  for (int i = 0; i < kMaxEngines; ++i)
    if (g_engines[i] && (uint64_t)(uintptr_t)g_engines[i] == v) return i;
  mexErrMsgIdAndTxt("gpdla:handle", "unknown or destroyed engine handle");
  return -1;
}

static void do_create(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
  if (nrhs < 20) mexErrMsgIdAndTxt("gpdla:args", "create: expected at least 19 arguments after 'create'");
  int slot = -1;
  for (int i = 0; i < kMaxEngines && slot < 0; ++i)
    if (!g_engines[i]) slot = i;
  if (slot < 0) mexErrMsgIdAndTxt("gpdla:engines", "too many live engines (%d)", kMaxEngines);
  const int32_t device = (int32_t)scalar(prhs[1], "device");
  const size_t G = mxGetNumberOfElements(prhs[2]);
  gpdla_model m;
  m.num_rest = (int32_t)G;
  m.k = (int32_t)mxGetN(prhs[4]);
  m.rest_wavelengths = dbl(prhs[2], "rest_wavelengths", 0);
  m.mu = dbl(prhs[3], "mu", G);
  if (mxGetM(prhs[4]) != G) mexErrMsgIdAndTxt("gpdla:size", "M must be numel(rest_wavelengths) x k");
  m.M = dbl(prhs[4], "M", 0);                     /* column-major, as MATLAB stores it */
  m.log_omega = dbl(prhs[5], "log_omega", G);
  m.log_c_0 = scalar(prhs[6], "log_c_0");
  m.log_tau_0 = scalar(prhs[7], "log_tau_0");
  m.log_beta = scalar(prhs[8], "log_beta");
  const size_t S = mxGetNumberOfElements(prhs[9]);
  gpdla_samples s;
  s.num_samples = (int64_t)S;
  s.offset_samples = dbl(prhs[9], "offset_samples", 0);
  s.nhi_samples = dbl(prhs[10], "nhi_samples", S);
  gpdla_params p;
  memset(&p, 0, sizeof p);
  p.num_lines = (int32_t)scalar(prhs[11], "num_lines");
  p.width = (int32_t)scalar(prhs[12], "width");
  p.pixel_spacing = scalar(prhs[13], "pixel_spacing");
  p.min_lambda = scalar(prhs[14], "min_lambda");
  p.max_lambda = scalar(prhs[15], "max_lambda");
  p.lya_wavelength = scalar(prhs[16], "lya_wavelength");
  p.lyman_limit = scalar(prhs[17], "lyman_limit");
  p.min_z_cut = scalar(prhs[18], "min_z_cut");
  p.max_z_cut = scalar(prhs[19], "max_z_cut");
  p.absorption_mode = nrhs > 20 ? (int32_t)scalar(prhs[20], "absorption_mode") : GPDLA_ABSORPTION_REFERENCE;
  p.path = nrhs > 21 ? path_code(prhs[21]) : GPDLA_PATH_AUTO;
  p.max_batch_spectra = 0;
  gpdla_engine* e = NULL;
  const int rc = gpdla_engine_create(device, &m, &s, &p, &e);
  if (rc != GPDLA_OK) fail(rc, "gpdla_engine_create");
  g_engines[slot] = e;
  g_num_samples[slot] = (int64_t)S;
  mexLock();                       /* engines live until 'destroy' (or MATLAB exits) */
  plhs[0] = mxCreateNumericMatrix(1, 1, mxUINT64_CLASS, mxREAL);
  *mxGetUint64s(plhs[0]) = (uint64_t)(uintptr_t)e;
  (void)nlhs;
}

/* dst (Q x S column-major, rows q0..q0+nq) <- src ([nq][S] spectrum-major), in kTile tiles */
static void transpose_rows(double* dst, size_t Q, size_t q0, const double* src, size_t nq, size_t S) {
  for (size_t s0 = 0; s0 < S; s0 += kTile)
    for (size_t r0 = 0; r0 < nq; r0 += kTile) {
      const size_t s1 = s0 + kTile < S ? s0 + kTile : S, r1 = r0 + kTile < nq ? r0 + kTile : nq;
      for (size_t s = s0; s < s1; ++s)
        for (size_t r = r0; r < r1; ++r) dst[(q0 + r) + s * Q] = src[r * S + s];
    }
}

static void do_process(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
  if (nrhs != 7) mexErrMsgIdAndTxt("gpdla:args", "process: expected (eng, wavelengths, flux, noise_variance, pixel_mask, z_qsos)");
  const int slot = slot_of(prhs[1]);
  gpdla_engine* e = g_engines[slot];
  const size_t S = (size_t)g_num_samples[slot];
  for (int i = 2; i <= 5; ++i)
    if (!mxIsCell(prhs[i])) mexErrMsgIdAndTxt("gpdla:type", "argument %d must be a cell array", i);
  const size_t Q = mxGetNumberOfElements(prhs[2]);
  for (int i = 3; i <= 5; ++i)
    if (mxGetNumberOfElements(prhs[i]) != Q) mexErrMsgIdAndTxt("gpdla:size", "cell arrays differ in length");
  const double* z = dbl(prhs[6], "z_qsos", Q);
  /* CSR packing of the cells (gpdla_spectra) */
  int64_t* off = (int64_t*)mxMalloc((Q + 1) * sizeof(int64_t));
  off[0] = 0;
  for (size_t q = 0; q < Q; ++q) {
    const mxArray* w = mxGetCell(prhs[2], q);
    const size_t n = w ? mxGetNumberOfElements(w) : 0;
    for (int i = 3; i <= 5; ++i) {
      const mxArray* c = mxGetCell(prhs[i], q);
      if ((c ? mxGetNumberOfElements(c) : 0) != n)
        mexErrMsgIdAndTxt("gpdla:size", "spectrum %zu: cells differ in length", q + 1);
    }
    off[q + 1] = off[q] + (int64_t)n;
  }
  const size_t npix = (size_t)off[Q];
  double* wl = (double*)mxMalloc((npix ? npix : 1) * sizeof(double));
  double* fl = (double*)mxMalloc((npix ? npix : 1) * sizeof(double));
  double* nv = (double*)mxMalloc((npix ? npix : 1) * sizeof(double));
  uint8_t* mk = (uint8_t*)mxMalloc(npix ? npix : 1);
  for (size_t q = 0; q < Q; ++q) {
    const size_t a = (size_t)off[q], n = (size_t)(off[q + 1] - off[q]);
    if (!n) continue;
    widen_into(wl + a, mxGetCell(prhs[2], q), "wavelengths", n);
    widen_into(fl + a, mxGetCell(prhs[3], q), "flux", n);
    widen_into(nv + a, mxGetCell(prhs[4], q), "noise_variance", n);
    const mxArray* m = mxGetCell(prhs[5], q);
    if (mxIsLogical(m)) {
      const mxLogical* src = mxGetLogicals(m);
      for (size_t i = 0; i < n; ++i) mk[a + i] = src[i] ? 1 : 0;
    } else {
      widen_check(m, "pixel_mask", n);
      if (mxIsDouble(m)) {
        const double* src = mxGetDoubles(m);
        for (size_t i = 0; i < n; ++i) mk[a + i] = src[i] != 0.0;
      } else {
        const float* src = mxGetSingles(m);
        for (size_t i = 0; i < n; ++i) mk[a + i] = src[i] != 0.0f;
      }
    }
  }
  /* outputs in process_qsos.m's shapes (nan(num_quasars, 1), nan(num_quasars, num_dla_samples)) */
  mxArray* out[6];
  out[0] = mxCreateDoubleMatrix(Q, 1, mxREAL);
  out[1] = mxCreateUninitNumericMatrix(Q, S, mxDOUBLE_CLASS, mxREAL);
  out[2] = mxCreateDoubleMatrix(Q, 1, mxREAL);
  out[3] = mxCreateDoubleMatrix(Q, 1, mxREAL);
  out[4] = mxCreateDoubleMatrix(Q, 1, mxREAL);
  out[5] = mxCreateNumericMatrix(Q, 1, mxINT32_CLASS, mxREAL);
  const size_t nb_max = Q < (size_t)kBatch ? Q : (size_t)kBatch;
  double* stage = (double*)mxMalloc((nb_max ? nb_max : 1) * (S ? S : 1) * sizeof(double));
  int numeric = 0;
  for (size_t q0 = 0; q0 < Q; q0 += kBatch) {
    const size_t nq = Q - q0 < (size_t)kBatch ? Q - q0 : (size_t)kBatch;
    gpdla_spectra sp;
    sp.memory = GPDLA_MEM_HOST;
    sp.num_spectra = (int64_t)nq;
    sp.offsets = off + q0;                   /* absolute offsets into the packed pixel arrays */
    sp.wavelengths = wl; sp.flux = fl; sp.noise_variance = nv; sp.pixel_mask = mk; sp.z_qsos = z + q0;
    gpdla_results r;
    r.memory = GPDLA_MEM_HOST;
    r.log_likelihoods_no_dla = mxGetDoubles(out[0]) + q0;
    r.sample_log_likelihoods_dla = stage;    /* [nq][S] spectrum-major */
    r.sample_ld = (int64_t)S;
    r.log_likelihoods_dla = mxGetDoubles(out[2]) + q0;
    r.min_z_dlas = mxGetDoubles(out[3]) + q0;
    r.max_z_dlas = mxGetDoubles(out[4]) + q0;
    r.num_pixels = mxGetInt32s(out[5]) + q0;
    const int rc = gpdla_engine_process(e, &sp, &r);
    if (rc == GPDLA_ENUMERIC) numeric = 1;          /* NaN outputs; raised once all are filled */
    else if (rc != GPDLA_OK) {
      mxFree(stage); mxFree(off); mxFree(wl); mxFree(fl); mxFree(nv); mxFree(mk);
      for (int i = 0; i < 6; ++i) mxDestroyArray(out[i]);
      fail(rc, "gpdla_engine_process");
    }
    transpose_rows(mxGetDoubles(out[1]), Q, q0, stage, nq, S);
  }
  mxFree(stage); mxFree(off); mxFree(wl); mxFree(fl); mxFree(nv); mxFree(mk);
  /* plhs holds max(nlhs, 1) slots */
  const int nout = nlhs < 1 ? 1 : (nlhs > 6 ? 6 : nlhs);
  for (int i = 0; i < 6; ++i) {
    if (i < nout) plhs[i] = out[i];
    else mxDestroyArray(out[i]);
  }
  if (numeric) fail(GPDLA_ENUMERIC, "gpdla_engine_process");
}

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
  static int registered = 0;
  if (!registered) {
    mexAtExit(destroy_all);
    registered = 1;
  }
  g_num_widened = 0;   /* copies of a call an error unwound were freed by MATLAB */
  if (nrhs < 1 || !mxIsChar(prhs[0])) mexErrMsgIdAndTxt("gpdla:args", "first argument: 'create', 'process' or 'destroy'");
  char* cmd = mxArrayToString(prhs[0]);
  const int c = !strcmp(cmd, "create") ? 0 : !strcmp(cmd, "process") ? 1 : !strcmp(cmd, "destroy") ? 2 : -1;
  mxFree(cmd);
  if (c == 0) {
    do_create(nlhs, plhs, nrhs, prhs);
  } else if (c == 1) {
    do_process(nlhs, plhs, nrhs, prhs);
  } else if (c == 2) {
    if (nrhs != 2) mexErrMsgIdAndTxt("gpdla:args", "destroy: expected the engine handle");
    const int slot = slot_of(prhs[1]);
    gpdla_engine_destroy(g_engines[slot]);
    g_engines[slot] = NULL;
    mexUnlock();
  } else {
    mexErrMsgIdAndTxt("gpdla:args", "unknown command");
  }
  widen_release();
}
