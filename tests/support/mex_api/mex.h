/* Declarations of the documented MATLAB MEX C API (interleaved-complex API, `mex -R2018a`) that
 * this repository's own gateways in matlab/ call -- ONLY so that tests/test_matlab_gateways.py can
 * compile-check those gateways (gcc -fsyntax-only) in a container without MATLAB.  Nothing is
 * linked against it and no reference code is built with it; a real build uses MATLAB's mex.h. */
#ifndef GPDLA_TEST_MEX_API_H
#define GPDLA_TEST_MEX_API_H
#include <stddef.h>
#include <stdint.h>
#include <stdbool.h>

typedef struct mxArray_tag mxArray;
typedef size_t mwSize;
typedef size_t mwIndex;
typedef bool mxLogical;
typedef enum { mxUNKNOWN_CLASS, mxCELL_CLASS, mxSTRUCT_CLASS, mxLOGICAL_CLASS, mxCHAR_CLASS, mxVOID_CLASS,
               mxDOUBLE_CLASS, mxSINGLE_CLASS, mxINT8_CLASS, mxUINT8_CLASS, mxINT16_CLASS, mxUINT16_CLASS,
               mxINT32_CLASS, mxUINT32_CLASS, mxINT64_CLASS, mxUINT64_CLASS } mxClassID;
typedef enum { mxREAL, mxCOMPLEX } mxComplexity;

mxArray* mxCreateDoubleMatrix(mwSize m, mwSize n, mxComplexity c);
mxArray* mxCreateDoubleScalar(double v);
mxArray* mxCreateNumericMatrix(mwSize m, mwSize n, mxClassID cls, mxComplexity c);
mxArray* mxCreateUninitNumericMatrix(size_t m, size_t n, mxClassID cls, mxComplexity c);
double* mxGetDoubles(const mxArray* a);
float* mxGetSingles(const mxArray* a);
uint64_t* mxGetUint64s(const mxArray* a);
int32_t* mxGetInt32s(const mxArray* a);
mxLogical* mxGetLogicals(const mxArray* a);
double mxGetScalar(const mxArray* a);
size_t mxGetM(const mxArray* a);
size_t mxGetN(const mxArray* a);
size_t mxGetNumberOfElements(const mxArray* a);
bool mxIsCell(const mxArray* a);
bool mxIsDouble(const mxArray* a);
bool mxIsSingle(const mxArray* a);
bool mxIsLogical(const mxArray* a);
bool mxIsUint64(const mxArray* a);
bool mxIsChar(const mxArray* a);
bool mxIsComplex(const mxArray* a);
mxArray* mxGetCell(const mxArray* a, mwIndex i);
char* mxArrayToString(const mxArray* a);
void mxFree(void* p);
void mxDestroyArray(mxArray* a);
void* mxMalloc(size_t n);
void mexErrMsgIdAndTxt(const char* id, const char* fmt, ...);
void mexWarnMsgIdAndTxt(const char* id, const char* fmt, ...);
int mexAtExit(void (*fn)(void));
void mexLock(void);
void mexUnlock(void);

#endif
