/* log_mvnpdf_low_rank_mex.c -- GPU replacement of log_mvnpdf_low_rank.m:5-33,
 *   log_p = log_mvnpdf_low_rank(y, mu, M, d)
 * (called at process_qsos.m:151 for the null model and :196 per DLA sample).
 *
 *   mex -R2018a -output log_mvnpdf_low_rank matlab/log_mvnpdf_low_rank_mex.c -Iinclude \
 *       -Lgp_dla_detection_amd -lgpdla
 *
 * y, mu, d: n-vectors; M: n x k (column-major, as MATLAB stores it).  A non-positive-definite
 * B = I + M' D^-1 M raises 'MATLAB:posdef', as chol does at log_mvnpdf_low_rank.m:24. */
#include <stdint.h>

#include "mex.h"
#include "gpdla.h"
#include "mex_widen.h"

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
  (void)nlhs;
  if (nrhs != 4) mexErrMsgIdAndTxt("gpdla:mvn", "usage: log_mvnpdf_low_rank(y, mu, M, d)");
  g_num_widened = 0;   /* copies of a call an error unwound were freed by MATLAB */
  const int64_t n = (int64_t)mxGetM(prhs[2]);
  const int32_t k = (int32_t)mxGetN(prhs[2]);
  if ((int64_t)mxGetNumberOfElements(prhs[0]) != n || (int64_t)mxGetNumberOfElements(prhs[1]) != n ||
      (int64_t)mxGetNumberOfElements(prhs[3]) != n)
    mexErrMsgIdAndTxt("gpdla:mvn", "y, mu and d must have size(M, 1) elements");
  /* double or single (e.g. process_qsos.m:196's this_flux from single preloaded cells), widened */
  const double* y = widen(prhs[0], "y", 0);
  const double* mu = widen(prhs[1], "mu", 0);
  const double* M = widen(prhs[2], "M", 0);
  const double* d = widen(prhs[3], "d", 0);
  double out = 0.0;
  const int rc = gpdla_log_mvnpdf_low_rank_f64(y, mu, M, d, n, k, &out);
  widen_release();
  if (rc == GPDLA_ENUMERIC) mexErrMsgIdAndTxt("MATLAB:posdef", "%s", gpdla_last_error());
  if (rc != GPDLA_OK) mexErrMsgIdAndTxt("gpdla:mvn", "%s", gpdla_last_error());
  plhs[0] = mxCreateDoubleScalar(out);
}
