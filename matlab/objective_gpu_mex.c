/* objective_gpu_mex.c -- GPU drop-in for objective.m under minFunc (learn_qso_model.m:100-101):
 *   [f, g] = objective_gpu(x, centered_rest_fluxes_t, lya_1pzs_t, rest_noise_variances_t)
 *
 *   mex -R2018a -output objective_gpu matlab/objective_gpu_mex.c -Iinclude -Lgp_dla_detection_amd -lgpdla
 *
 * x = [M(:); log_omega; log_c_0; log_tau_0; log_beta] (objective.m:21-30).  The training matrices
 * of learn_qso_model.m:63-84 are num_quasars x num_pixels in MATLAB (column-major); the ABI takes
 * them row-major ([quasar][pixel]), which is the column-major layout of their transposes: pass
 * centered_rest_fluxes.' etc.  The handle (data resident on the device) is kept across calls and
 * rebuilt when the data pointer or shape changes, so minFunc's repeated evaluations cost one
 * f/g evaluation each. */
#include <stdint.h>

#include "mex.h"
#include "gpdla.h"

static gpdla_objective* g_obj;
static const double* g_key;
static int64_t g_P, g_Q;
static int32_t g_k;

static void release(void) {
  if (g_obj) gpdla_objective_destroy(g_obj);
  g_obj = NULL;
  g_key = NULL;
}

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
  static int registered = 0;
  if (!registered) { mexAtExit(release); registered = 1; }
  if (nrhs != 4) mexErrMsgIdAndTxt("gpdla:objective", "usage: objective_gpu(x, fluxes.', lya_1pzs.', noise.')");
  for (int i = 0; i < 4; ++i)
    if (!mxIsDouble(prhs[i])) mexErrMsgIdAndTxt("gpdla:objective", "argument %d must be double", i + 1);
  const int64_t P = (int64_t)mxGetM(prhs[1]), Q = (int64_t)mxGetN(prhs[1]);  /* transposed inputs */
  const int64_t nx = (int64_t)mxGetNumberOfElements(prhs[0]);
  if (P < 1 || (nx - 3) % P != 0) mexErrMsgIdAndTxt("gpdla:objective", "numel(x) - 3 must be a multiple of num_pixels");
  const int32_t k = (int32_t)((nx - 3) / P - 1);
  const double* F = mxGetDoubles(prhs[1]);
  if (!g_obj || g_key != F || g_P != P || g_Q != Q || g_k != k) {
    release();
    const int rc = gpdla_objective_create(0, Q, P, k, F, mxGetDoubles(prhs[2]), mxGetDoubles(prhs[3]),
                                          GPDLA_MEM_HOST, &g_obj);
    if (rc != GPDLA_OK) { g_obj = NULL; mexErrMsgIdAndTxt("gpdla:objective", "%s", gpdla_last_error()); }
    g_key = F; g_P = P; g_Q = Q; g_k = k;
  }
  mxArray* f = mxCreateDoubleScalar(0.0);
  mxArray* g = mxCreateDoubleMatrix((size_t)nx, 1, mxREAL);
  const int rc = gpdla_objective_eval(g_obj, mxGetDoubles(prhs[0]), mxGetDoubles(f), nlhs > 1 ? mxGetDoubles(g) : NULL);
  if (rc != GPDLA_OK) {
    mxDestroyArray(f); mxDestroyArray(g);
    mexErrMsgIdAndTxt("gpdla:objective", "%s", gpdla_last_error());
  }
  plhs[0] = f;
  if (nlhs > 1) plhs[1] = g; else mxDestroyArray(g);
}
