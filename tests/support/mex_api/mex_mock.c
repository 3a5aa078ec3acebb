#define _POSIX_C_SOURCE 200809L
/* A minimal in-process MEX runtime for testing this repository's MATLAB gateways (matlab/ sources)
 * without MATLAB: mxArrays are plain heap objects, mexErrMsgIdAndTxt longjmps back to the caller.
 * Built with a gateway into one shared library (gp_dla_detection_amd/build.py build_mex_mock) and
 * driven from Python by tests/test_matlab_gateways.py.  Test infrastructure only. */
#include <setjmp.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mex.h"

struct mxArray_tag {
  mxClassID cls;
  size_t m, n;
  void* data;        /* numeric / logical / char (NUL-terminated) */
  mxArray** cells;   /* cell arrays */
};

static jmp_buf g_jmp;
static char g_err[1024];
static void (*g_atexit)(void);
static int g_locks;

static size_t elsize(mxClassID c) {
  switch (c) {
    case mxDOUBLE_CLASS: case mxINT64_CLASS: case mxUINT64_CLASS: return 8;
    case mxINT32_CLASS: case mxUINT32_CLASS: case mxSINGLE_CLASS: return 4;
    case mxINT16_CLASS: case mxUINT16_CLASS: return 2;
    default: return 1;
  }
}

static mxArray* make(mxClassID cls, size_t m, size_t n) {
  mxArray* a = (mxArray*)calloc(1, sizeof(mxArray));
  a->cls = cls; a->m = m; a->n = n;
  a->data = calloc(m * n > 0 ? m * n : 1, elsize(cls));
  return a;
}

mxArray* mxCreateDoubleMatrix(mwSize m, mwSize n, mxComplexity c) { (void)c; return make(mxDOUBLE_CLASS, m, n); }
mxArray* mxCreateDoubleScalar(double v) { mxArray* a = make(mxDOUBLE_CLASS, 1, 1); *(double*)a->data = v; return a; }
mxArray* mxCreateNumericMatrix(mwSize m, mwSize n, mxClassID cls, mxComplexity c) { (void)c; return make(cls, m, n); }
mxArray* mxCreateUninitNumericMatrix(size_t m, size_t n, mxClassID cls, mxComplexity c) { (void)c; return make(cls, m, n); }
double* mxGetDoubles(const mxArray* a) { return a->cls == mxDOUBLE_CLASS ? (double*)a->data : NULL; }
float* mxGetSingles(const mxArray* a) { return a->cls == mxSINGLE_CLASS ? (float*)a->data : NULL; }
uint64_t* mxGetUint64s(const mxArray* a) { return a->cls == mxUINT64_CLASS ? (uint64_t*)a->data : NULL; }
int32_t* mxGetInt32s(const mxArray* a) { return a->cls == mxINT32_CLASS ? (int32_t*)a->data : NULL; }
mxLogical* mxGetLogicals(const mxArray* a) { return a->cls == mxLOGICAL_CLASS ? (mxLogical*)a->data : NULL; }
/* MATLAB's mxGetScalar: the first element of any numeric, logical or char array as a double (0 if
 * empty); extra elements are ignored */
double mxGetScalar(const mxArray* a) {
  if (a->m * a->n == 0 || a->cls == mxCELL_CLASS) return 0.0;
  switch (a->cls) {
    case mxDOUBLE_CLASS: return *(const double*)a->data;
    case mxSINGLE_CLASS: return (double)*(const float*)a->data;
    case mxINT8_CLASS: return (double)*(const int8_t*)a->data;
    case mxUINT8_CLASS: case mxLOGICAL_CLASS: case mxCHAR_CLASS: return (double)*(const uint8_t*)a->data;
    case mxINT16_CLASS: return (double)*(const int16_t*)a->data;
    case mxUINT16_CLASS: return (double)*(const uint16_t*)a->data;
    case mxINT32_CLASS: return (double)*(const int32_t*)a->data;
    case mxUINT32_CLASS: return (double)*(const uint32_t*)a->data;
    case mxINT64_CLASS: return (double)*(const int64_t*)a->data;
    case mxUINT64_CLASS: return (double)*(const uint64_t*)a->data;
    default: return 0.0;
  }
}
size_t mxGetM(const mxArray* a) { return a->m; }
size_t mxGetN(const mxArray* a) { return a->n; }
size_t mxGetNumberOfElements(const mxArray* a) { return a->m * a->n; }
bool mxIsCell(const mxArray* a) { return a->cls == mxCELL_CLASS; }
bool mxIsDouble(const mxArray* a) { return a->cls == mxDOUBLE_CLASS; }
bool mxIsSingle(const mxArray* a) { return a->cls == mxSINGLE_CLASS; }
bool mxIsLogical(const mxArray* a) { return a->cls == mxLOGICAL_CLASS; }
bool mxIsUint64(const mxArray* a) { return a->cls == mxUINT64_CLASS; }
bool mxIsChar(const mxArray* a) { return a->cls == mxCHAR_CLASS; }
bool mxIsComplex(const mxArray* a) { (void)a; return false; }
mxArray* mxGetCell(const mxArray* a, mwIndex i) { return a->cells[i]; }
char* mxArrayToString(const mxArray* a) { return a->cls == mxCHAR_CLASS ? strdup((const char*)a->data) : NULL; }
void mxFree(void* p) { free(p); }
void* mxMalloc(size_t n) { return malloc(n); }
void mxDestroyArray(mxArray* a) {
  if (!a) return;
  if (a->cells)
    for (size_t i = 0; i < a->m * a->n; ++i) mxDestroyArray(a->cells[i]);
  free(a->cells);
  free(a->data);
  free(a);
}
void mexErrMsgIdAndTxt(const char* id, const char* fmt, ...) {
  int k = snprintf(g_err, sizeof g_err, "%s: ", id);
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err + k, sizeof g_err - (size_t)k, fmt, ap);
  va_end(ap);
  longjmp(g_jmp, 1);
}
void mexWarnMsgIdAndTxt(const char* id, const char* fmt, ...) { (void)id; (void)fmt; }
int mexAtExit(void (*fn)(void)) { g_atexit = fn; return 0; }
void mexLock(void) { ++g_locks; }
void mexUnlock(void) { --g_locks; }

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]);

/* ---- harness (ctypes) ---- */
mxArray* mock_numeric(int cls, size_t m, size_t n, const void* src) {
  mxArray* a = make((mxClassID)cls, m, n);
  if (src) memcpy(a->data, src, m * n * elsize((mxClassID)cls));
  return a;
}
mxArray* mock_string(const char* s) {
  mxArray* a = make(mxCHAR_CLASS, 1, strlen(s));
  free(a->data);
  a->data = strdup(s);
  return a;
}
mxArray* mock_cell(size_t n, mxArray** elems) {   /* n x 1; takes ownership of elems[i] */
  mxArray* a = make(mxCELL_CLASS, n, 1);
  a->cells = (mxArray**)calloc(n ? n : 1, sizeof(mxArray*));
  for (size_t i = 0; i < n; ++i) a->cells[i] = elems[i];
  return a;
}
void* mock_data(const mxArray* a) { return a->data; }
size_t mock_m(const mxArray* a) { return a->m; }
size_t mock_n(const mxArray* a) { return a->n; }
int mock_class(const mxArray* a) { return (int)a->cls; }
void mock_free(mxArray* a) { mxDestroyArray(a); }
const char* mock_error(void) { return g_err; }
int mock_locks(void) { return g_locks; }
void mock_at_exit(void) { if (g_atexit) g_atexit(); }
/* mexFunction under the harness: 0 = returned, 1 = raised (message in mock_error()) */
int mock_call(int nlhs, mxArray** plhs, int nrhs, mxArray** prhs) {
  g_err[0] = 0;
  if (setjmp(g_jmp)) return 1;
  mexFunction(nlhs, plhs, nrhs, (const mxArray**)prhs);
  return 0;
}
