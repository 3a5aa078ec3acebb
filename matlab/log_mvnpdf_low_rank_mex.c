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

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
  (void)nlhs;
  if (nrhs != 4) mexErrMsgIdAndTxt("gpdla:mvn", "usage: log_mvnpdf_low_rank(y, mu, M, d)");
  for (int i = 0; i < 4; ++i)
    if (!mxIsDouble(prhs[i])) mexErrMsgIdAndTxt("gpdla:mvn", "argument %d must be double", i + 1);
  const int64_t n = (int64_t)mxGetM(prhs[2]);
  const int32_t k = (int32_t)mxGetN(prhs[2]);
  if ((int64_t)mxGetNumberOfElements(prhs[0]) != n || (int64_t)mxGetNumberOfElements(prhs[1]) != n ||
      (int64_t)mxGetNumberOfElements(prhs[3]) != n)
    mexErrMsgIdAndTxt("gpdla:mvn", "y, mu and d must have size(M, 1) elements");
  double out = 0.0;
  const int rc = gpdla_log_mvnpdf_low_rank_f64(mxGetDoubles(prhs[0]), mxGetDoubles(prhs[1]),
                                               mxGetDoubles(prhs[2]), mxGetDoubles(prhs[3]), n, k, &out);
  if (rc == GPDLA_ENUMERIC) mexErrMsgIdAndTxt("MATLAB:posdef", "%s", gpdla_last_error());
  if (rc != GPDLA_OK) mexErrMsgIdAndTxt("gpdla:mvn", "%s", gpdla_last_error());
  plhs[0] = mxCreateDoubleScalar(out);
}
