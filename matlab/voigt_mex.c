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
#include "mex_widen.h"

static double ref_scalar(const mxArray* a, const char* name) {
  if (mxIsCell(a) || mxIsChar(a) || mxGetNumberOfElements(a) == 0)
    mexErrMsgIdAndTxt("gpdla:voigt", "%s must be a numeric scalar", name);
  return mxGetScalar(a);
}

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
  (void)nlhs;
  if (nrhs < 3 || nrhs > 4) mexErrMsgIdAndTxt("gpdla:voigt", "usage: voigt(lambdas, z, N[, num_lines])");
  g_num_widened = 0;   /* copies of a call an error unwound were freed by MATLAB */
  /* a single lambdas (process_qsos.m:171-177 on single preloaded cells) is widened exactly, where
   * voigt.c:262's mxGetPr would reinterpret its bytes as doubles */
  const double* lambdas = widen(prhs[0], "lambdas", 0);
  const int64_t n = (int64_t)mxGetNumberOfElements(prhs[0]);
  if (n <= 6) mexErrMsgIdAndTxt("gpdla:voigt", "need more than 6 wavelengths (2 width)");
  /* z, N and num_lines are read like voigt.c:263-266 does, with mxGetScalar: any numeric or logical
   * class, the first element (voigt(lam, z, N, int32(3)) works as with the original) */
  const double z = ref_scalar(prhs[1], "z"), N = ref_scalar(prhs[2], "N");
  const int32_t num_lines = nrhs > 3 ? (int32_t)ref_scalar(prhs[3], "num_lines") : 31;
  mxArray* out = mxCreateDoubleMatrix((size_t)(n - 6), 1, mxREAL);
  const int rc = gpdla_voigt_f64(lambdas, n, z, N, num_lines, mxGetDoubles(out));
  widen_release();
  if (rc != GPDLA_OK) {
    mxDestroyArray(out);
    mexErrMsgIdAndTxt("gpdla:voigt", "%s", gpdla_last_error());
  }
  plhs[0] = out;
}
