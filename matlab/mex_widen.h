/* mex_widen.h -- numeric MATLAB arguments as doubles for the C ABI (libgpdla computes in fp64).
 *
 * Double arrays are borrowed.  Single arrays are widened exactly (every float is a double) into
 * copies: single is the class fitsread gives the speclite float columns (read_spec.m:11-31), so it
 * is the class of the preloaded_qsos.mat cells preload_qsos.m:77-80 saves and process_qsos.m:57-60
 * passes on.  Copies come from mxMalloc and are released by widen_release() at the end of the call
 * (MATLAB frees them by itself when an error unwinds the call).  Shared by the gateways in matlab/. */
#ifndef GPDLA_MEX_WIDEN_H
#define GPDLA_MEX_WIDEN_H

#include <stddef.h>
#include <string.h>

#include "mex.h"

#define GPDLA_MAX_WIDENED 64
static void* g_widened[GPDLA_MAX_WIDENED];
static int g_num_widened;

static inline void widen_release(void) {
  for (int i = 0; i < g_num_widened; ++i) mxFree(g_widened[i]);
  g_num_widened = 0;
}

static inline void widen_check(const mxArray* a, const char* name, size_t want) {
  if ((!mxIsDouble(a) && !mxIsSingle(a)) || mxIsComplex(a))
    mexErrMsgIdAndTxt("gpdla:type", "%s must be real double or single", name);
  if (want && mxGetNumberOfElements(a) != want)
    mexErrMsgIdAndTxt("gpdla:size", "%s has %zu elements, expected %zu", name, mxGetNumberOfElements(a), want);
}

/* dst[0..n) <- the n elements of a (double or single; n must equal numel(a)) */
static inline void widen_into(double* dst, const mxArray* a, const char* name, size_t n) {
  widen_check(a, name, n);
  if (mxIsDouble(a)) {
    memcpy(dst, mxGetDoubles(a), n * sizeof(double));
  } else {
    const float* src = mxGetSingles(a);
    for (size_t i = 0; i < n; ++i) dst[i] = (double)src[i];
  }
}

/* the elements of a as doubles (want = required numel, 0 = any): borrowed or a widened copy */
static inline const double* widen(const mxArray* a, const char* name, size_t want) {
  widen_check(a, name, want);
  if (mxIsDouble(a)) return mxGetDoubles(a);
  if (g_num_widened == GPDLA_MAX_WIDENED) mexErrMsgIdAndTxt("gpdla:internal", "too many widened arguments");
  const size_t n = mxGetNumberOfElements(a);
  double* copy = (double*)mxMalloc((n ? n : 1) * sizeof(double));
  g_widened[g_num_widened++] = copy;
  widen_into(copy, a, name, n);
  return copy;
}

static inline double widen_scalar(const mxArray* a, const char* name) { return *widen(a, name, 1); }

#endif
