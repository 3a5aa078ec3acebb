/* voigt_mex.c -- drop-in GPU replacement of the reference's voigt MEX (voigt.c:253-304), called at
 * process_qsos.m:186-187 as  absorption = voigt(lambdas, z, N[, num_lines]).
 *
 *   mex -R2018a -output voigt matlab/voigt_mex.c -Iinclude -Lgp_dla_detection_amd -lgpdla
 *
 * Same convention: num_lines defaults to 31 (voigt.c:8-13,266) and the output is the
 * (numel(lambdas) - 2 width) x 1 column of voigt.c:271 (width = 3).  Unlike the original, a bad
 * num_lines (outside 1..31; voigt.c:266,279 read out of bounds) is an error. */
#include <stdint.h>

#include "mex.h"
#include "gpdla.h"

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
  (void)nlhs;
  if (nrhs < 3 || nrhs > 4) mexErrMsgIdAndTxt("gpdla:voigt", "usage: voigt(lambdas, z, N[, num_lines])");
  if (!mxIsDouble(prhs[0])) mexErrMsgIdAndTxt("gpdla:voigt", "lambdas must be double");
  const int64_t n = (int64_t)mxGetNumberOfElements(prhs[0]);
  if (n <= 6) mexErrMsgIdAndTxt("gpdla:voigt", "need more than 6 wavelengths (2 width)");
  const double z = mxGetScalar(prhs[1]), N = mxGetScalar(prhs[2]);
  const int32_t num_lines = nrhs > 3 ? (int32_t)mxGetScalar(prhs[3]) : 31;
  mxArray* out = mxCreateDoubleMatrix((size_t)(n - 6), 1, mxREAL);
  const int rc = gpdla_voigt_f64(mxGetDoubles(prhs[0]), n, z, N, num_lines, mxGetDoubles(out));
  if (rc != GPDLA_OK) {
    mxDestroyArray(out);
    mexErrMsgIdAndTxt("gpdla:voigt", "%s", gpdla_last_error());
  }
  plhs[0] = out;
}
